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
    """The compact cycle (two sweeps per level with P̃ / R̃ of tb blocks)."""
    n, nn, nb, tb = 1000, 300, 4000, 2500
    ai = {"nd": 2, "levels": 2, "rows": [n, nn], "blocks": [nb, nn], "pblocks": [1800, 0],
          "ptblocks": [tb, 0], "cycle": 1}
    B, V, V8, Bs, Bs8 = 16, 8, 16, 12, 24
    down = tb * (B + 4) + nb * (Bs + 4) + (V8 + 2 * V + B) * n + (B + 2 * V) * nn
    up = tb * (B + 4) + 2 * V * n + V * nn
    update = (9 * V8 + V + B + V) * n
    w = nb * (Bs8 + 4) + (2 * V8 + V) * n
    assert bench.amg_iteration_bytes(ai) == down + up + update + w
    assert bench.amg_iteration_bytes(ai, compact=False) == bench.amg_iteration_bytes(dict(ai, cycle=0))
