"""Benchmark: DOF solved/s of one full FEA load step on MI355X.

A "step" = one pass of the hot path over the synthetic mesh: device assembly
(all elements active) → Dirichlet elimination/RHS → PCG (SA-AMG "gamg" V-cycle
by default, as the reference's -pc_type gamg sweep) to ‖r‖ ≤ 1e-8‖b‖ (x0 = 0)
→ reaction + stress/failure update.  Inputs are resident in HBM before the
timed region; no CSV IO.  Workload (BASELINE.json configs[2]): C3_1M = 6×8
tiles of results/sim_20251117_181147 (1.06 M DOF).

N > 1 (one process per GPU): the partitioned solve over RCCL,
one part of the network per GPU (partition.hpp: the min-cut px × py grid).
  --scaling weak   (default) the network is (6N)×8 tiles — C3 per GPU;
  --scaling strong the C3 network itself is cut into N parts.
`value` is the whole network's DOF/s.  `--mode replicas` runs N independent
copies of the 1-GPU step instead.  torch.distributed (gloo) only carries the
RCCL unique id, the barriers and the max-over-ranks time.

Launch: `python bench.py --gpus N` with no WORLD_SIZE in the environment
starts the N ranks itself (child processes with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_*; the parent touches no GPU) and exits with the first
failing rank's code — the reference's `mpirun -np N ./fea_petsc`
(README.md:18).  Under torch.distributed.run, --gpus must equal WORLD_SIZE
(or be omitted).  A rank whose partitioned solve fails ends the run with a
non-zero exit; `--allow-replicas` turns that into N independent copies
(labelled in `parallelism` and `note`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3_1M] [--scaling weak|strong]

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mycelium-fea-project_amd"))

import numpy as np  # noqa: E402,F401

PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); default WORLD_SIZE, else 1.  N > 1 without WORLD_SIZE: "
                         "this process launches the N ranks")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3_1M", choices=["C2_100k", "C3_1M", "C5_10M_dense"])
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--precond", default="gamg", choices=["gamg", "jacobi", "bjacobi"])
    ap.add_argument("--load-step", type=int, default=20, help="load step index of 40 (dy)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu1-its", type=int, default=150,
                    help="PCG iterations of the bounded 1-core CPU sample")
    ap.add_argument("--traffic", default=None,
                    help="PMC-derived HBM bytes per SpMV launch (rocprofv3 pass), if present")
    ap.add_argument("--mode", default="partitioned", choices=["partitioned", "replicas"],
                    help="N > 1: one network cut over the GPUs, or N independent copies")
    ap.add_argument("--allow-replicas", action="store_true",
                    help="N > 1 partitioned: if the RCCL solve fails on some rank, run replicas "
                         "instead of exiting non-zero")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1 partitioned: C3 per GPU (weak) or C3 cut N ways (strong)")
    ap.add_argument("--device", type=int, default=None,
                    help="HIP device of this rank (default LOCAL_RANK; rehearsal: several ranks on one GPU)")
    ap.add_argument("--parts", type=int, default=1,
                    help="1 GPU: run the partitioned solve with this many partitions on it")
    ap.add_argument("--no-full-run", action="store_true",
                    help="skip the 40-step run (all load steps, with failures) after the timed steps")
    ap.add_argument("--amg-dist", type=int, default=1, choices=[-1, 0, 1],
                    help="N > 1 GAMG form: 1 the global hierarchy's distributed V-cycle (default: holds the "
                         "one-partition iteration count on any network), 0 block Jacobi over per-partition "
                         "hierarchies (as fast only where the cuts follow weak couplings, e.g. the tiled "
                         "network's seams), -1 the engine's automatic choice")
    ap.add_argument("--no-jacobi", action="store_true",
                    help="skip the Jacobi-PCG leg (SURVEY §8d's iteration metric) after the timed steps")
    return ap.parse_args(argv)


def amg_iteration_bytes(ai, compact=None):
    """Algorithmic HBM bytes of one GAMG-PCG iteration: every
    launch of the iteration, each array counted once per launch.  The V-cycle
    is f32 (B = 4·ND² bytes per block, V = 4·ND per row vector), the CG f64
    (V8 = 8·ND) except the V-cycle output u, stored f32.  A_0's blocks are
    symmetric and stored as upper triangles (NS = ND(ND+1)/2 values: f64 for
    w = A u, Bs8 = 8·NS; f32 for the level-0 V-cycle, Bs = 4·NS).  Per level l
    (n rows, nb blocks of A_l, pb blocks of P_l = R_l; level 0's b is the
    CG's f64 r, Vb = V8 there, V elsewhere; BA = Bs at level 0, B elsewhere):
      resid    nb·(BA+4) + (2V + Vb)·n             (A, x, b in; t out)
      restrict pb·(B+4) + V·n + (2V + B)·n'        (Pᵀ, t in; b', x' out, D⁻¹')
      prolong  pb·(B+4) + 2V·n + V·n'              (P, x in/out, e' in)
      post     nb·(BA+4) + (2V + B + Vb)·n         (A, x, D⁻¹, b in; e out)
    The compact cycle (amg_cycle 1; tb blocks of P̃_l = of R̂_l per level; its
    sweeps read the level's f32 iterate x alone and Ã = ω D⁻¹ A as full f32
    blocks, level 0 included):
      down     tb·(B+4) + nb·(B+4) + 2V·n + V·n'   (R̂, Ã, x in; c out, x' out)
      up       tb·(B+4) + 2V·n + V·n'              (P̃, c in, e out; e' in)
    collapsed below level kc (collapse_level > 0; vb blocks of V): the levels
    ≥ kc are one sweep  vapply  vb·(B+4) + 2V·n_kc  (V, x in; e out).
    Levels 0 and 1 merged around kc = 2 (merged; dqb blocks of DQ, ub of U):
      down     dqb·(B+4) + nb0·(B+4) + 2V·n0 + V·(n1 + n2)   (DQ, Ã_0, x_0 in; c_0, c_1, x_2 out)
      up       ub·(B+4) + 2V·n0 + V·(n1 + n2)                (U, c_0, c_1, e_2 in; u out)
    CG: update (9·V8 + V + B + V)·n0 (u w p s x r in, p s x r out, D⁻¹, x₀ out);
        w      nb0·(Bs8+4) + (2·V8 + V)·n0         (A_0, r, u in; w out).
    """
    nd = ai["nd"]
    ns = nd * (nd + 1) // 2
    B, V, V8, Bs, Bs8 = 4 * nd * nd, 4 * nd, 8 * nd, 4 * ns, 8 * ns
    rows, blocks, pbl = ai["rows"], ai["blocks"], ai["pblocks"]
    if compact is None:
        compact = ai.get("cycle", 0) == 1
    kc = ai.get("collapse_level", 0) if compact else 0
    b = 0
    if compact and kc == 2 and ai.get("merged"):
        n0, n1, n2 = rows[0], rows[1], rows[2]
        b += ai["merge_dq_blocks"] * (B + 4) + blocks[0] * (B + 4) + 2 * V * n0 + V * (n1 + n2)
        b += ai["collapse_blocks"] * (B + 4) + 2 * V * n2
        b += ai["merge_u_blocks"] * (B + 4) + 2 * V * n0 + V * (n1 + n2)
        b += (9 * V8 + V + B + V) * n0 + blocks[0] * (Bs8 + 4) + (2 * V8 + V) * n0
        return b
    for l in range(ai["levels"] - 1):
        n, nn = rows[l], rows[l + 1]
        Vb = V8 if l == 0 else V
        BA = Bs if l == 0 else B
        if compact:
            if kc and l == kc:
                b += ai["collapse_blocks"] * (B + 4) + 2 * V * n
                break
            tb = ai["ptblocks"][l]
            b += tb * (B + 4) + blocks[l] * (B + 4) + 2 * V * n + V * nn
            b += tb * (B + 4) + 2 * V * n + V * nn
            continue
        b += blocks[l] * (BA + 4) + (2 * V + Vb) * n
        b += pbl[l] * (B + 4) + V * n + (2 * V + B) * nn
        b += pbl[l] * (B + 4) + 2 * V * n + V * nn
        b += blocks[l] * (BA + 4) + (2 * V + B + Vb) * n
    n0 = rows[0]
    b += (9 * V8 + V + B + V) * n0 + blocks[0] * (Bs8 + 4) + (2 * V8 + V) * n0
    return b


def amg_spmv_bytes(ai):
    """Algorithmic bytes of one SpMV launch k_amg_cg_w: A_0's
    symmetric f64 blocks with their column indices, r in and w out (f64), u in
    (f32)."""
    nd = ai["nd"]
    return ai["blocks"][0] * (8 * nd * (nd + 1) // 2 + 4) + (2 * 8 + 4) * nd * ai["rows"][0]


def iteration_bytes(info, block):
    """Algorithmic HBM bytes of one iteration launch.

    Lane kernel (ell.hip), nd DOFs per node, NB = 3 (nd 2) or 6 block
    components, NM = nd (Jacobi) or NB (block-Jacobi) M components:
      per lane read  8·(5·nd + NB + NL_M + 3·NB) + 8 (r s w p x, D, the lane's
                     M — NL_M = NB for block Jacobi, 0 for Jacobi, whose
                     M = 1/(D_ii + reg) is formed in registers — three slot
                     blocks, code + partner)
      halo records   read 8·(3·nd + NM) (r s w + M of the out-of-wave
                     neighbour) by every lane (one record per lane, small
                     systems) or by halo lanes only + 16 B per wave (mask and
                     base; compact records, large systems); written 8·3·nd per
                     halo lane (the record it fills)
      per free row   written 8·5·nd (p x s r w)
    SELL kernel (cg.hip): per free row 120 + minv + 120 + 48 + 4 B, per slot 52 B.
    """
    if info["cg_lanes"]:
        nd = 2 if info["planar"] else 3
        nb = 3 if nd == 2 else 6
        nm = nb if block else nd
        per_lane = 8 * (5 * nd + nb + (nb if block else 0) + 3 * nb) + 8
        rec = 8 * (3 * nd + nm)  # a halo record r s w + M
        if info["halo_compact"]:  # only halo lanes read one; + mask and base per wave
            reads = info["n_halo"] * rec + info["n_lanes"] // 64 * 16
        else:                     # one record per lane, read by every lane
            reads = info["n_lanes"] * rec
        b = (info["n_lanes"] * per_lane + reads + info["n_free_nodes"] * 40 * nd
             + info["n_halo"] * 24 * nd)
        return b, f"k_ell_iter (lanes, {nd} DOF/node: update + SpMV + reduction)"
    minv = 48 if block else 24
    b = info["n_free_nodes"] * (120 + minv + 120 + 48 + 4) + info["free_incidences"] * 52
    return b, "k_cg_iter (SELL: update + SpMV + reduction)"


def new_set_steps(n_act, n_elems):
    """Per step of a full run, 1 if it ran on an active set other than the
    step before it.  `eng.step` reports the count AFTER its own failure
    update, so step k runs on the set step k-1 left (step 0 on the intact
    mesh, n_elems): step k is on a new set when n_act[k-1] != n_act[k-2]."""
    if not n_act:
        return []
    ran_on = [n_elems] + list(n_act[:-1])
    return [0] + [int(ran_on[k] != ran_on[k - 1]) for k in range(1, len(ran_on))]


def full_run(eng, opts, fs, dmax=None):
    """The reference's whole driver loop on the bench network (src/fea_solver.py:
    216-295): N_STEPS load steps from the intact mesh, elements failing as they
    go, every step on device (no CSV IO).  Reports the wall time of the run, each
    step's wall time and iteration count, the steps that ran on a new active set
    (failures in the step before), and those that rebuilt the GAMG hierarchy
    (host symbolic phase + upload + graph capture) — by default the hierarchy
    is kept over failures until the iterations degrade (option amg_reuse)."""
    import time as _t
    dmax = fs.DISPLACEMENT_MAX if dmax is None else dmax
    eng.set_active(None)
    per, its, rebuilt, reused, n_act = [], [], [], [], []
    t0 = _t.perf_counter()
    for step in range(fs.N_STEPS):
        dy = dmax * step / (fs.N_STEPS - 1)
        t = _t.perf_counter()
        f, na, st = eng.step(dy, -dy, opts, fs.MAX_STRAIN)
        per.append(1e3 * (_t.perf_counter() - t))
        its.append(st.iters)
        rebuilt.append(st.amg_rebuilt)
        reused.append(eng.get_option("amg_reused") if opts.precond == 2 else 0)
        n_act.append(na)
        if na == 0:
            break
    wall = _t.perf_counter() - t0
    changed = new_set_steps(n_act, eng.n_elems)
    med = float(np.median([p for p, r in zip(per, rebuilt) if not r] or per))
    reb = [p for p, r in zip(per, rebuilt) if r]
    new_set = [p for p, c, r in zip(per, changed, rebuilt) if c and not r]
    new_idx = [k for k, (c, r) in enumerate(zip(changed, rebuilt)) if c and not r]
    return {"steps": len(per), "wall_s": wall, "step_ms": per, "cg_iters": its, "n_active": n_act,
            "displacement_max_mm": dmax,
            "new_active_set_steps": int(sum(changed)), "kept_hierarchy_steps": len(new_set),
            "kept_hierarchy_step_ms": new_set, "kept_hierarchy_step_idx": new_idx,
            "kept_hierarchy_worst_vs_median": (max(new_set) / med) if new_set else None,
            "rebuild_steps": int(sum(rebuilt)), "rebuild_step_ms": reb,
            "rebuild_overhead_ms": float(sum(p - med for p in reb)), "median_step_ms": med,
            "note": "all 40 load steps from the intact mesh, failures included; a step on a new active set "
                    "keeps the GAMG hierarchy (floating pieces masked on the device) until the time its "
                    "solves spent on extra iterations reaches the host build's time (rent or buy), then "
                    "rebuilds it (rebuild_overhead_ms = rebuild steps' time above the median step); "
                    "kept_hierarchy_step_idx = the steps that ran on a new set; no CSV IO"}


def full_run_reference(opts, fs, device):
    """The 40-step run on the reference's own network results/sim_20251117_181147
    (22,125 DOF; elements fail from step 27 on, so the GAMG hierarchy is rebuilt
    for each new active set), beside the reference's end-to-end walls for it."""
    from mfea import Engine, synth
    xyz, e2n = synth.load_mesh(synth.BASE_TILE)
    top, bot = synth.grips(xyz, 1.5)  # the reference run's grip band (results/.../fea_results)
    with Engine(device) as eng:
        eng.set_material(fs.E_mod, fs.A, fs.I)
        eng.set_mesh(xyz, e2n)
        eng.set_bc(top, bot)
        r = full_run(eng, opts, fs)
    r["reference"] = {"python_wall_s": 71.76, "python_solve_step_ms_mean": 20.4,
                      "source": "results/sim_20251117_181147/fea_results/runtime.txt:1 (whole fea_solver.py run, "
                                "PNG plots included); results/sim_20251117_181147_cpp/fea_results/"
                                "solve_runtime_1.txt (solve_system + K@U per step, 40 steps)"}
    return r


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def host_threads():
    """Threads the CPU legs may use: OMP_NUM_THREADS (the GPU box sets it to the
    job's CPU share, 16), else the process's CPU affinity."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env or len(os.sched_getaffinity(0))


def cpu_legs(a, out, xyz, e2n, top, bot, dy, n_dof):
    """CPU baselines on this host (rank 0, N = 1, after the timed region):
    (1) the "host PETSc CG" — oracle/cpu_fea.c, a C/OpenMP restatement of
        fea_petsc.cpp assembly + KSPCG/PCJACOBI (same stopping rule) — one full
        step on every thread the job may use;
    (2) the same on 1 core, a bounded sample: assembly, RHS and post run in
        full, PCG for --cpu1-its iterations, extrapolated to (1)'s count;
    (3) the reference Python's own solver class: NumPy assembly + SciPy
        spsolve (SuperLU, src/fea_solver.py:128) through oracle/fea_oracle.py."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import cpu_fea  # baseline legs only
    import fea_oracle as fo
    import fea_solver as fs
    threads = host_threads()
    host = f"{cpu_model()} ({os.cpu_count()} CPUs visible, {len(os.sched_getaffinity(0))} in affinity)"
    c = cpu_fea.CpuFea(xyz, e2n, top, bot, fs.E_mod, fs.A, fs.I)
    t = time.perf_counter()
    r = c.step(dy, -dy, rtol=a.rtol, max_it=200000, threads=threads)
    t_all = time.perf_counter() - t
    its = r["iters"]
    c.active[:] = 1
    k = max(1, min(a.cpu1_its, its))
    r1 = c.step(dy, -dy, rtol=a.rtol, max_it=k, threads=1)
    tt = r1["times"]
    t_one = tt[0] + tt[1] + tt[3] + tt[2] / k * its
    c.close()
    t = time.perf_counter()
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    t_asm = time.perf_counter() - t
    t = time.perf_counter()
    fo.solve_system(K, known, vals)
    t_sol = time.perf_counter() - t
    legs = {
        "cg_jacobi_all_threads": {
            "value": n_dof / t_all, "unit": "DOF/s", "cores": threads, "kind": "port",
            "sample": f"1 full load step of the same {a.config} mesh: C/OpenMP restatement of "
                      f"fea_petsc.cpp assembly + PETSc KSPCG/PCJACOBI to rtol {a.rtol} ({its} iters), "
                      f"{t_all:.2f} s on {threads} threads of {host}"},
        "cg_jacobi_1core": {
            "value": n_dof / t_one, "unit": "DOF/s", "cores": 1, "kind": "port",
            "sample": f"bounded: assembly + RHS + post in full, {k} of {its} PCG iterations "
                      f"({tt[2]:.2f} s) extrapolated -> {t_one:.1f} s per step, 1 thread of {host}"},
        "direct_spsolve": {
            "value": n_dof / (t_asm + t_sol), "unit": "DOF/s", "cores": 1, "kind": "port",
            "sample": f"1 step: NumPy csr assembly {t_asm:.2f} s + SciPy spsolve (SuperLU) "
                      f"{t_sol:.2f} s — the reference Python's direct solve "
                      f"(src/fea_solver.py:74-135); solve-only {n_dof / t_sol:.3g} DOF/s"},
    }
    out["cpu_baseline"] = legs["cg_jacobi_all_threads"]
    out["cpu_baselines"] = legs
    out["speedup_vs_cpu"] = out["value"] / legs["cg_jacobi_all_threads"]["value"]
    out["speedup_vs_cpu_1core"] = out["value"] / legs["cg_jacobi_1core"]["value"]
    out["speedup_vs_direct"] = out["value"] / legs["direct_spsolve"]["value"]
    if out.get("jacobi_step_ms"):
        # like for like: the same algorithm (Jacobi-PCG, same stopping rule) on
        # the GPU and on the host; speedup_vs_cpu compares the GPU's GAMG step
        # with the host's Jacobi one
        out["speedup_jacobi_vs_cpu_jacobi"] = t_all / (out["jacobi_step_ms"] * 1e-3)


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_plan(n, argv, port, env=None):
    """The N rank processes `python bench.py --gpus N` starts when no launcher
    did: (argv, env) per rank — this script with the same arguments, one
    process per GPU (LOCAL_RANK = the GPU), rendezvous on 127.0.0.1:port."""
    base = dict(os.environ if env is None else env)
    plan = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GROUP_RANK="0")
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        plan.append(([sys.executable, os.path.abspath(__file__)] + list(argv), e))
    return plan


def run_ranks(plan, poll_s=0.2):
    """Start every rank, wait; the first rank to fail ends the others (their
    process groups) and its exit code is the launcher's.  Rank 0's stdout is
    the launcher's (the JSON line); the other ranks' stdout goes to stderr."""
    import signal
    import subprocess
    procs = []
    for r, (argv, env) in enumerate(plan):
        procs.append(subprocess.Popen(argv, env=env, start_new_session=True,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in live:  # the rest would wait for the failed rank forever
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        if live:
            time.sleep(poll_s)
    for p in procs:
        p.wait()
    return rc


def world_of(a, env=None):
    """(rank, world, launch): the rank and world size of this process, and
    whether it must launch the ranks itself.  --gpus ≠ WORLD_SIZE is an error."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if a.gpus is not None and a.gpus != world:
            raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
        return int(env.get("RANK", "0")), world, False
    n = 1 if a.gpus is None else a.gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}")
    return 0, n, n > 1


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    rank, world, launch = world_of(a)
    if launch:  # no GPU call in this process: the ranks are its children
        sys.exit(run_ranks(launch_plan(world, argv, free_port())))
    local = int(os.environ.get("LOCAL_RANK", "0")) if a.device is None else a.device
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from mfea import Engine, make_opts, PC_BLOCK_JACOBI, PC_GAMG, PC_JACOBI, dist_unique_id, synth
    from mfea.synth import CONFIGS
    import fea_solver as fs

    nx0, ny = CONFIGS[a.config]
    mode = a.mode if world > 1 else ("parts" if a.parts > 1 else "1gpu")
    note = None
    dy = fs.DISPLACEMENT_MAX * a.load_step / (fs.N_STEPS - 1)
    pc = {"gamg": PC_GAMG, "jacobi": PC_JACOBI, "bjacobi": PC_BLOCK_JACOBI}[a.precond]
    opts = make_opts(rtol=a.rtol, max_it=200000, precond=pc)

    def setup(mode):
        """engine + resident mesh for one mode; returns (eng, nx, xyz, e2n, top, bot)"""
        # weak scaling: the config's tiles per GPU, side by side along x
        nx = nx0 * world if mode == "partitioned" and a.scaling == "weak" else nx0
        eng = Engine(local)
        if mode == "partitioned":
            uid = [dist_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            eng.dist_init(rank, world, uid[0])
            eng.set_partition_axis(-1)  # the min-cut px × py grid (partition.hpp)
        elif mode == "parts":
            eng.set_parts(a.parts, -1)
        if mode in ("partitioned", "parts"):
            # the global hierarchy's compact distributed cycle by default: block
            # Jacobi over partitions matches it here only because the tiled
            # network's cuts follow its weak tile seams (190-310 iterations
            # instead of 16 on the grown reference network)
            eng.set_option("amg_dist", a.amg_dist)
        xyz, e2n = synth.tiled_mesh(nx, ny, chords=a.config.startswith("C5"))
        top, bot = synth.grips(xyz)
        eng.set_material(fs.E_mod, fs.A, fs.I)
        eng.set_mesh(xyz, e2n)
        eng.set_bc(top, bot)
        eng.set_active(None)
        return eng, nx, xyz, e2n, top, bot

    def run_step(eng):
        eng.set_active(None)                       # every step starts from the intact mesh
        return eng.step(dy, -dy, opts, fs.MAX_STRAIN)

    if mode == "partitioned":
        # one probing step over RCCL with the chunks as hipGraph replays (RCCL
        # ops captured); every rank must succeed, else all retry with eager
        # launches, else fall back to independent replicas (agreed over gloo)
        # — the line reports which
        import torch

        def agree(ok):
            flag = torch.tensor([ok], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            return int(flag.item()) == 1

        eng, errs = None, []
        for graph in (1, 0):
            ok = 1
            try:
                eng, nx, xyz, e2n, top, bot = setup(mode)
                eng.set_option("dist_graph", graph)
                run_step(eng)
            except Exception as ex:  # noqa: BLE001
                ok = 0
                errs.append(str(ex))
            if agree(ok):
                if graph == 0:
                    note = f"graph-captured partitioned chunks failed ({errs[0] if errs else 'peer'}); eager launches"
                break
            if eng is not None:
                eng.close()
                eng = None
        if eng is None:
            msg = f"partitioned solve failed on some rank ({errs[-1] if errs else 'peer'})"
            if not a.allow_replicas:
                raise SystemExit(f"bench.py rank {rank}: {msg}")
            note = msg + "; replicas instead (--allow-replicas)"
            mode = "replicas"
            eng, nx, xyz, e2n, top, bot = setup(mode)
    else:
        eng, nx, xyz, e2n, top, bot = setup(mode)
    n_dof = 3 * len(xyz)
    info = eng.info()

    def one_step():
        return run_step(eng)

    def barrier_sync():
        if dist is not None:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize(local)  # the engine's device, all its streams
            dist.barrier()

    for _ in range(a.warmup):
        one_step()
    if mode in ("partitioned", "parts") and pc == PC_GAMG:
        # the automatic GAMG form (amg_dist -1) tries both forms on its first
        # two solves of an active set, building the block-Jacobi form's
        # per-partition hierarchies on the host: keep those trials out of the
        # timed steps whatever --warmup is (the choice is collective: every
        # rank sees the same value)
        for _ in range(3):
            undecided = eng.get_option("amg_dist_chosen") < 0
            if dist is not None:
                import torch
                flag = torch.tensor([1 if undecided else 0], dtype=torch.int32)
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                undecided = bool(flag.item())
            if not undecided:
                break
            one_step()
    barrier_sync()
    t0 = time.perf_counter()
    stats = []
    for _ in range(a.steps):
        stats.append(one_step())
    barrier_sync()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # DOF of the whole job: the one (partitioned) network, or N copies
    job_dof = n_dof * (world if mode == "replicas" else 1)

    force, n_active, st = stats[-1]
    # the phase split (mfea_stats t_*_ms) from one more step with the phase
    # events on (option phase_times; off in the timed steps: each event
    # between two kernels idles the GPU for several µs)
    eng.set_option("phase_times", 1)
    ph = [one_step()[2] for _ in range(5)]
    eng.set_option("phase_times", 0)
    ph_ms = {f: float(np.median([getattr(x, f) for x in ph]))
             for f in ("t_assemble_ms", "t_rhs_ms", "t_solve_ms", "t_post_ms", "t_setup_ms")}
    iters = st.iters
    # ---- roofline, live HIP events on the engine's stream, algorithmic bytes
    # per launch as in DESIGN.md §4 (partitioned: rank 0's partition, without
    # exchange).  GAMG: `roofline` = the SpMV kernel w = A_0 u (f64, with the
    # CG's four partial sums — the metric's SpMV and the iteration's longest
    # launch), `roofline_iteration` = one whole PCG iteration (every launch).
    # Jacobi: the one fused iteration kernel.
    nf = info["n_free_nodes"]
    tj = {}
    a.traffic = a.traffic or os.path.join(REPO, "profiles", f"traffic_{a.config}.json")
    if os.path.exists(a.traffic) and mode == "1gpu":
        try:
            tj = json.load(open(a.traffic))
            if tj.get("config") != a.config:  # only a profile of the same config
                tj = {}
        except Exception:
            tj = {}
    # partitioned GAMG: the whole iteration interleaves exchanges, so only the
    # SpMV of rank 0's rows is profiled (its bytes: rank 0's share of A_0 by rows)
    split = mode in ("partitioned", "parts") and pc == PC_GAMG
    iter_ms = None if split else eng.profile_iteration(pc, reps=200 if pc != PC_GAMG else 50)
    if pc == PC_GAMG:
        ai = eng.amg_info()
        iter_bytes = amg_iteration_bytes(ai)
        nl = ai["levels"]
        if ai.get("cycle", 0) == 1:  # compact cycle: two sweeps per level
            kc = ai.get("collapse_level", 0)
            launches = 2 + (2 * kc + 1 if kc else 2 * (nl - 1))
            form = f"compact, collapsed below level {kc}" if kc else "compact"
            if kc == 2 and ai.get("merged"):
                launches = 5
                form = "compact, levels 0-1 merged, collapsed below level 2"
        else:
            # levels from the first one of ≤ 2048 rows (above the coarsest) run
            # in one single-workgroup launch (the engine's default amg_tail_rows)
            tail = next((l for l in range(1, nl - 1) if ai["rows"][l] <= 2048), 0)
            launches = 2 + (4 * tail + 1 if tail else 4 * (nl - 1))
            form = "four-step"
        iter_kernel = (f"GAMG-PCG iteration ({launches} launches: update + "
                       f"{nl}-level {form} V-cycle + w = A u)")
        spmv_ms = eng.profile_spmv(reps=100)
        nd = ai["nd"]
        spmv_bytes = amg_spmv_bytes(ai)
        if split:
            spmv_bytes = int(spmv_bytes * nf / max(ai["rows"][0], 1))
        kernel = f"k_amg_cg_w (SpMV w = A_0 u, f64 symmetric {nd}x{nd} blocks, + CG partial sums)"
        kernel_ms, kernel_bytes = spmv_ms, spmv_bytes
        traffic = tj.get("spmv_bytes_per_launch") if tj.get("spmv_kernel") == "k_amg_cg_w" else None
        iter_traffic = tj.get("iteration_bytes") if tj.get("iter_kernel", "").startswith("GAMG") else None
    else:
        iter_bytes, iter_kernel = iteration_bytes(info, pc == PC_BLOCK_JACOBI)
        kernel, kernel_ms, kernel_bytes = iter_kernel, iter_ms, iter_bytes
        traffic = tj.get("bytes_per_launch") if iter_kernel.split()[0] in tj.get("iter_kernel", "") else None
        iter_traffic = None
    achieved = kernel_bytes / (kernel_ms * 1e-3) / 1e9

    parallelism = {"1gpu": "1gpu", "parts": f"parts{a.parts}@1gpu",
                   "partitioned": f"partitioned{world} (RCCL)", "replicas": f"replicas{world}"}[mode]
    workload = (f"{a.config}: {nx}x{ny} tiles, {n_dof} DOF, {st.n_free} free DOF, {len(e2n)} elements, "
                f"load step {a.load_step}/40")
    if mode == "partitioned":
        workload += f", cut into {world} strips (min-cut grid, one per GPU; {a.scaling} scaling)"
    elif mode == "parts":
        workload += f", {a.parts} partitions on 1 GPU"
    elif mode == "replicas":
        workload += f", one copy per GPU ({world} GPUs)"
    out = {
        "metric": "DOF solved/sec + CG iters to 1e-8; SpMV achieved HBM GB/s vs roofline",
        "value": job_dof * a.steps / dt,
        "unit": "DOF/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * dt / a.steps,
        "higher_is_better": True,
        "scaling": a.scaling if mode == "partitioned" else "weak",
        "vs_baseline": None,
        "dtype": "f64" if pc != PC_GAMG else "f64 (CG; f32 AMG V-cycle)",
        "data": "synthetic (tiled copies of results/sim_20251117_181147; no RNG)",
        "config": {
            "workload": workload,
            "n_dof": n_dof, "n_free_dof": st.n_free, "n_elems": len(e2n),
            "precond": a.precond, "rtol": a.rtol, "parallelism": parallelism,
            "cg_kernel": "lanes" if info["cg_lanes"] else "sell", "n_lanes": info["n_lanes"],
            "lane_geometry": {"block": info["block_size"], "grid": info["grid"], "halo_records": "compact" if info["halo_compact"] else "per lane"},
            "rank0_part": {"free_dof": 3 * nf, "n_pairs": info["n_pairs"], "n_ghost": info["n_ghost"]},
        },
        "cg_iters": iters,
        "relres": st.relres,
        "step_breakdown_ms": {"assemble": ph_ms["t_assemble_ms"], "rhs": ph_ms["t_rhs_ms"],
                              "pcg": ph_ms["t_solve_ms"], "post": ph_ms["t_post_ms"],
                              "amg_setup (inside pcg)": ph_ms["t_setup_ms"],
                              "note": "medians of 5 untimed steps with the phase events on"},
        "roofline": {
            "kernel": kernel,
            "bound": "hbm",
            "achieved": achieved,
            "peak": PEAK_HBM_GBPS,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBPS,
            "traffic": traffic,
            "alg_bytes_per_launch": kernel_bytes,
            "avg_launch_us": kernel_ms * 1e3,
        },
    }
    if split:
        out["roofline"]["note"] = ("rank 0's w = A_0 u over its own rows; bytes = the whole A_0's scaled by "
                                   "its share of the rows")
    if pc == PC_GAMG and not split:
        ia = iter_bytes / (iter_ms * 1e-3) / 1e9
        out["roofline_iteration"] = {
            "kernel": iter_kernel, "bound": "hbm", "achieved": ia, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": ia / PEAK_HBM_GBPS, "traffic": iter_traffic, "alg_bytes_per_iteration": iter_bytes,
            "avg_iteration_us": iter_ms * 1e3}
    if pc == PC_GAMG:
        out["amg"] = {"levels": ai["levels"], "rows": ai["rows"], "blocks": ai["blocks"],
                      "setup_pair_items": ai["pair_items"], "split_levels": ai["n_dist"]}
    if mode in ("partitioned", "parts") and pc == PC_GAMG:
        ch = eng.get_option("amg_dist_chosen")
        how = ("option amg_dist -1: the faster of the two, measured in warmup" if a.amg_dist < 0
               else f"--amg-dist {a.amg_dist}")
        out["config"]["amg_partitions"] = {
            0: "block Jacobi over per-partition hierarchies",
            1: "distributed V-cycle of one global hierarchy (compact: level 0 split, levels below replicated)",
            -1: "undecided"}[ch] + f" ({how})"
    if note:
        out["note"] = note

    # ---- legs after the timed region (not part of `value`)
    if not a.no_jacobi and pc == PC_GAMG:
        # SURVEY §8(d)'s iteration metric: Jacobi-PCG to rtol 1e-8 on the same step
        eng.set_active(None)
        eng.set_option("phase_times", 1)  # (its step time is the phase sum)
        fj, nj, sj = eng.step(dy, -dy, make_opts(rtol=a.rtol, max_it=200000, precond=PC_JACOBI), fs.MAX_STRAIN)
        eng.set_option("phase_times", 0)
        out["jacobi_iters_1e8"] = sj.iters
        out["jacobi_step_ms"] = sj.t_assemble_ms + sj.t_rhs_ms + sj.t_solve_ms + sj.t_post_ms
    if not a.no_full_run:
        out["full_run"] = full_run(eng, opts, fs)
        if world == 1 and mode == "1gpu":
            out["full_run_reference_network"] = full_run_reference(opts, fs, local)
            # the failure path at scale: the tiled network strains far less than
            # the reference network at the same grip displacement, so the leg
            # pulls until its peak strain at the last step is the reference
            # network's (2.1 x the failure strain: first failures mid-run)
            eng.set_active(None)
            eng.step(fs.DISPLACEMENT_MAX, -fs.DISPLACEMENT_MAX, opts, 1e30)  # intact, nothing fails
            peak = float(np.abs(eng.stress()).max()) / fs.E_mod
            scale = 2.1 * fs.MAX_STRAIN / peak
            fr = full_run(eng, opts, fs, dmax=fs.DISPLACEMENT_MAX * scale)
            fr["note"] = (f"the {a.config} network pulled to DISPLACEMENT_MAX x {scale:.0f}, where its peak "
                          f"strain at the last step is 2.1 x MAX_STRAIN as on the reference network: elements "
                          f"fail from mid-run on. ") + fr["note"]
            out["full_run_failures"] = fr

    if not a.no_jacobi and pc == PC_GAMG and mode == "1gpu":
        # the reference sweep's other preconditioners on the same step
        # (src/fea_petsc_solverAndPC.cpp:331): SSOR and the source default's
        # ICC, whole-matrix factorisations in the chain-piece multicolour
        # order (csrc/sweep.hip)
        from mfea import PC_ICC, PC_SOR
        eng.set_option("phase_times", 1)  # (their step times are phase sums)
        for name, code in (("sor", PC_SOR), ("icc", PC_ICC)):
            eng.set_active(None)
            eng.step(dy, -dy, make_opts(rtol=a.rtol, max_it=200000, precond=code), fs.MAX_STRAIN)  # plan build
            eng.set_active(None)
            _, _, sk = eng.step(dy, -dy, make_opts(rtol=a.rtol, max_it=200000, precond=code), fs.MAX_STRAIN)
            out[f"{name}_iters_1e8"] = sk.iters
            out[f"{name}_step_ms"] = sk.t_assemble_ms + sk.t_rhs_ms + sk.t_solve_ms + sk.t_post_ms
            out[f"{name}_plan"] = {"colours": eng.get_option("sweep_colors"),
                                   "pieces": eng.get_option("sweep_pieces"),
                                   "iteration_us": 1e3 * eng.profile_iteration(code, reps=50)}

    if rank == 0 and not a.no_cpu and world == 1:
        cpu_legs(a, out, xyz, e2n, top, bot, dy, n_dof)

    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
