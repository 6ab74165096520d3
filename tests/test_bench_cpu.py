"""bench.py's algorithmic byte accounting, no GPU: the GAMG
iteration bytes summed launch by launch from the formula of each kernel, on a
small hand-checkable hierarchy, and the SpMV kernel's bytes as the roofline
uses them."""
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_amg_iteration_bytes_by_hand(bench):
    # two levels, planar (ND = 2): level 0 with n rows / nb blocks of A_0 /
    # pb blocks of P_0, then the coarsest level with nn rows
    n, nb, pb, nn = 10, 30, 20, 4
    ai = {"nd": 2, "levels": 2, "rows": [n, nn], "blocks": [nb, nn], "pblocks": [pb, 0]}
    B, V, V8, Bs, Bs8 = 16, 8, 16, 12, 24   # f32 block, f32 row, f64 row, symmetric f32 / f64 block
    resid = nb * (Bs + 4) + (2 * V + V8) * n
    restrict = pb * (B + 4) + V * n + (2 * V + B) * nn
    prolong = pb * (B + 4) + 2 * V * n + V * nn
    post = nb * (Bs + 4) + (2 * V + B + V8) * n
    update = (9 * V8 + V + B + V) * n
    w = nb * (Bs8 + 4) + (2 * V8 + V) * n
    assert bench.amg_iteration_bytes(ai) == resid + restrict + prolong + post + update + w


def test_spmv_bytes_are_the_w_kernels_share(bench):
    """amg_spmv_bytes (the roofline's) equals what amg_iteration_bytes charges
    to the w kernel: the part of the iteration linear in blocks₀ that is not
    resid's or post's, plus the w kernel's vector terms."""
    n, nb = 1000, 3100
    ai = {"nd": 2, "levels": 2, "rows": [n, 1], "blocks": [nb, 1], "pblocks": [1, 0]}
    assert bench.amg_spmv_bytes(ai) == nb * (24 + 4) + (2 * 16 + 8) * n
    ai0 = dict(ai, blocks=[0, 1])
    delta = bench.amg_iteration_bytes(ai) - bench.amg_iteration_bytes(ai0)
    assert delta == nb * ((12 + 4) * 2 + (24 + 4))  # resid + post (f32 sym) + w (f64 sym)
    # 3-D: 6 stored values per symmetric block
    ai3 = {"nd": 3, "levels": 2, "rows": [n, 1], "blocks": [nb, 1], "pblocks": [1, 0]}
    assert bench.amg_spmv_bytes(ai3) == nb * (48 + 4) + 60 * n


def test_amg_iteration_bytes_compact_by_hand(bench):
    """The compact cycle (two sweeps per level on the f32 iterate x, with P̃ /
    R̂ of tb blocks and Ã as full f32 blocks), and the cycle collapsed below
    level kc (one sweep of V's vb blocks there)."""
    n, nn, nb, tb = 1000, 300, 4000, 2500
    ai = {"nd": 2, "levels": 2, "rows": [n, nn], "blocks": [nb, nn], "pblocks": [1800, 0],
          "ptblocks": [tb, 0], "cycle": 1}
    B, V, V8, Bs, Bs8 = 16, 8, 16, 12, 24
    down = tb * (B + 4) + nb * (B + 4) + 2 * V * n + V * nn
    up = tb * (B + 4) + 2 * V * n + V * nn
    update = (9 * V8 + V + B + V) * n
    w = nb * (Bs8 + 4) + (2 * V8 + V) * n
    assert bench.amg_iteration_bytes(ai) == down + up + update + w
    assert bench.amg_iteration_bytes(ai, compact=False) == bench.amg_iteration_bytes(dict(ai, cycle=0))
    # three levels collapsed below level 1: level 0's sweeps, then V at level 1
    n2, nb1, tb1, vb = 40, 1500, 900, 2700
    ai3 = {"nd": 2, "levels": 3, "rows": [n, nn, n2], "blocks": [nb, nb1, n2], "pblocks": [1800, 600, 0],
           "ptblocks": [tb, tb1, 0], "cycle": 1, "collapse_level": 1, "collapse_blocks": vb}
    vapply = vb * (B + 4) + 2 * V * nn
    assert bench.amg_iteration_bytes(ai3) == down + up + vapply + update + w
    # not collapsed: level 1's two sweeps instead
    down1 = tb1 * (B + 4) + nb1 * (B + 4) + 2 * V * nn + V * n2
    up1 = tb1 * (B + 4) + 2 * V * nn + V * n2
    assert bench.amg_iteration_bytes(dict(ai3, collapse_level=0)) == down + up + down1 + up1 + update + w
    # levels 0 and 1 merged around a level-2 collapse: one down sweep (DQ and
    # Ã_0 rows), V at level 2, one up sweep (U rows)
    n3, dqb, ub = 10, 7000, 5000
    ai4 = {"nd": 2, "levels": 4, "rows": [n, nn, n2, n3], "blocks": [nb, nb1, 300, n3],
           "pblocks": [1800, 600, 50, 0], "ptblocks": [tb, tb1, 80, 0], "cycle": 1, "collapse_level": 2,
           "collapse_blocks": vb, "merged": 1, "merge_dq_blocks": dqb, "merge_u_blocks": ub}
    mdown = dqb * (B + 4) + nb * (B + 4) + 2 * V * n + V * (nn + n2)
    mv = vb * (B + 4) + 2 * V * n2
    mup = ub * (B + 4) + 2 * V * n + V * (nn + n2)
    assert bench.amg_iteration_bytes(ai4) == mdown + mv + mup + update + w


# ---- the multi-GPU launcher (bench.py --gpus N), no GPU -----------------------

def test_launch_plan_one_process_per_rank(bench):
    argv = ["--gpus", "4", "--steps", "3"]
    plan = bench.launch_plan(4, argv, 29517, env={"PATH": "/usr/bin"})
    assert len(plan) == 4
    for r, (cmd, env) in enumerate(plan):
        assert cmd[1].endswith("bench.py") and cmd[2:] == argv
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert (env["MASTER_ADDR"], env["MASTER_PORT"]) == ("127.0.0.1", "29517")
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/usr/bin"


def test_world_of(bench):
    a = bench.parse(["--gpus", "8"])
    assert bench.world_of(a, env={}) == (0, 8, True)          # launches its 8 ranks
    assert bench.world_of(a, env={"WORLD_SIZE": "8", "RANK": "3"}) == (3, 8, False)
    with pytest.raises(SystemExit):                            # --gpus disagrees with the launcher
        bench.world_of(a, env={"WORLD_SIZE": "4", "RANK": "0"})
    assert bench.world_of(bench.parse([]), env={}) == (0, 1, False)
    assert bench.world_of(bench.parse([]), env={"WORLD_SIZE": "2", "RANK": "1"}) == (1, 2, False)
    assert bench.world_of(bench.parse(["--gpus", "1"]), env={}) == (0, 1, False)
    assert not bench.parse([]).allow_replicas                   # the replica fallback is opt-in


def test_run_ranks_first_failure_ends_the_rest(bench):
    import sys
    import time
    ok = [sys.executable, "-c", "print('rank0 line')"]
    bad = [sys.executable, "-c", "import sys; sys.exit(3)"]
    hang = [sys.executable, "-c", "import time; time.sleep(600)"]
    env = dict(os.environ)
    t = time.time()
    assert bench.run_ranks([(ok, env), (bad, env), (hang, env)], poll_s=0.05) == 3
    assert time.time() - t < 60
    assert bench.run_ranks([(ok, env), (ok, env)], poll_s=0.05) == 0


@pytest.mark.timeout(300)
def test_bench_gpus2_without_gpu_exits_nonzero():
    """`python bench.py --gpus 2` with no GPU: both ranks start (gloo), the
    engine cannot be created, and with no --allow-replicas the launcher exits
    non-zero instead of reporting a number."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu"], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode != 0
    assert '"metric"' not in r.stdout
    assert "partitioned solve failed" in r.stderr


def test_new_set_steps_label_the_step_after_the_failures(bench):
    """eng.step reports the active count after its own failure update, so the
    step that RUNS on a new set is the one after the count moved (round-5's
    labelling marked the failing step itself)."""
    E = 10
    # steps 0-2 intact; step 3 fails 2 elements, step 4 none, step 5 one, step 6 one
    n_act = [10, 10, 10, 8, 8, 7, 6, 6]
    assert bench.new_set_steps(n_act, E) == [0, 0, 0, 0, 1, 0, 1, 1]
    # a failure in step 0 (b = 0: cannot happen in the reference loop) → step 1
    assert bench.new_set_steps([9, 9], E) == [0, 1]
    assert bench.new_set_steps([], E) == []
    assert bench.new_set_steps([10], E) == [0]
