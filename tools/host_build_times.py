"""Host symbolic-phase (AMG plan build) time at a chord-network scale, split by
phase (MFEA_BUILD_TIMES): the global build and the distributed one for W ranks.

    python3 tools/host_build_times.py NX NY [W]     (C5: 20 23)
"""
import os, sys, time, ctypes as C
import numpy as np
sys.path[:0] = ['/root/repo/tests', '/root/repo/mycelium-fea-project_amd', '/root/repo/tools']
os.environ['MFEA_BUILD_TIMES'] = '1'
from conftest import build_host_shim
from mfea import synth
nx, ny = int(sys.argv[1]), int(sys.argv[2])
t = time.time(); xyz, e2n = synth.tiled_mesh(nx, ny, chords=True); top, bot = synth.grips(xyz)
print(f"mesh {len(xyz)} nodes {len(e2n)} elems {time.time()-t:.1f} s", flush=True)
lib = C.CDLL(build_host_shim())
P = C.c_void_p
def p(a): return a.ctypes.data_as(P)
xyz = np.ascontiguousarray(xyz, np.float64); e2n = np.ascontiguousarray(e2n, np.int64)
top = np.ascontiguousarray(top, np.int64); bot = np.ascontiguousarray(bot, np.int64)
sizes = np.zeros(5, np.int64); err = C.create_string_buffer(256)
lib.shim_build.restype = C.c_int
t = time.time()
assert lib.shim_build(C.c_int64(len(xyz)), p(xyz), C.c_int64(len(e2n)), p(e2n), 0, C.c_int64(len(top)), p(top), C.c_int64(len(bot)), p(bot), -1, p(sizes), err, 256) == 0, err.value
print(f"pattern {time.time()-t:.1f} s", flush=True)
act = np.ones(len(e2n), np.uint8)
lib.shim_amg.restype = C.c_int
t = time.time(); n = lib.shim_amg(p(act), 2, err, 256); print(f"global build: {n} levels {time.time()-t:.2f} s", flush=True)
if len(sys.argv) > 3:
    W = int(sys.argv[3])
    owner = np.zeros(len(xyz), np.int32)
    lib.shim_node_owner(C.c_int64(len(xyz)), p(xyz), C.c_int64(len(e2n)), p(e2n), C.c_int64(len(top)), p(top), C.c_int64(len(bot)), p(bot), W, -1, C.c_double(0.35), p(owner))
    lib.shim_amg_dist.restype = C.c_int
    t = time.time(); n = lib.shim_amg_dist(p(act), 2, W, p(owner), C.c_int64(32768), err, 256); print(f"dist build W={W}: {n} levels {time.time()-t:.2f} s", flush=True)
