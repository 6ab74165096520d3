"""bench.py with the process's memory map written out before the first step.

For symbolising a native stack trace printed by a signal handler (addresses
only): run as `rocprofv3 ... -- python3 tools/maps_bench.py <bench args>`;
the map lands in gpurun_out/maps_<pid>.txt, taken after every library the
step uses (libmfea, libamdhip64, libhsa-runtime64, the tracer's own) is
loaded.  Offsets = address − the mapping's start + its file offset.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mycelium-fea-project_amd"))

import bench  # noqa: E402
import mfea  # noqa: E402

_orig = mfea.Engine.step
_done = []


def _step(self, *a, **k):
    if not _done:
        _done.append(1)
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        with open("/proc/self/maps") as f, \
                open(os.path.join(REPO, "gpurun_out", f"maps_{os.getpid()}.txt"), "w") as g:
            g.write(f.read())
    return _orig(self, *a, **k)


mfea.Engine.step = _step

if __name__ == "__main__":
    sys.argv[0] = "bench.py"
    bench.main()
