"""Synthetic mycelium meshes for benchmarking (SURVEY §8d recipe).

Base tile = ``results/sim_20251117_181147`` (7,375 nodes, 7,504 elements, z = 0),
committed as data under tests/golden/meshes/.  ``tiled_mesh(nx, ny)`` copies it
on an nx × ny grid with 0.04 mm gaps and stitches nodes of *different* tiles
closer than 0.1 mm with extra bar elements (KD-tree pairs, sorted), so the
network stays one connected, grip-to-grip load path.  ``chords`` adds
intra-tile chords between not-yet-joined nodes 0.04–0.053 mm apart (the
"dense-filament" C5 variant, mean degree ≈ 4).  Deterministic: no RNG anywhere.
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd
from scipy.spatial import cKDTree

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BASE_TILE = os.path.join(_REPO, "tests", "golden", "meshes", "sim_20251117_181147")


def load_mesh(d):
    """nodes.csv / elements.csv as the reference reads them (pd.read_csv defaults)."""
    nodes = pd.read_csv(os.path.join(d, "nodes.csv"))
    elems = pd.read_csv(os.path.join(d, "elements.csv"))
    return nodes[["x", "y", "z"]].values.astype(np.float64), elems[["n1", "n2"]].values.astype(np.int64)


CHORD_MIN, CHORD_MAX = 0.04, 0.053  # mm, the C5 "dense-filament" chord window


def tiled_mesh(nx=1, ny=1, gap=0.04, stitch=0.1, chords=False, base=BASE_TILE):
    xyz0, e0 = load_mesh(base)
    n0 = xyz0.shape[0]
    lo, hi = xyz0.min(axis=0), xyz0.max(axis=0)
    wx, wy = hi[0] - lo[0] + gap, hi[1] - lo[1] + gap
    xyz, e2n, tile = [], [], []
    t = 0
    for iy in range(ny):
        for ix in range(nx):
            off = np.array([ix * wx, iy * wy, 0.0])
            xyz.append(xyz0 + off)
            e2n.append(e0 + t * n0)
            tile.append(np.full(n0, t))
            t += 1
    xyz = np.concatenate(xyz)
    e2n = np.concatenate(e2n)
    tile = np.concatenate(tile)
    extra = []
    if nx * ny > 1:
        pairs = cKDTree(xyz[:, :2]).query_pairs(stitch, output_type="ndarray")
        pairs = pairs[tile[pairs[:, 0]] != tile[pairs[:, 1]]]
        extra.append(pairs)
    if chords:
        # intra-tile chords between nodes CHORD_MIN..CHORD_MAX apart that no
        # element joins yet (the base tile's segments are 0.05 mm long, so a
        # plain distance window would mostly double existing elements);
        # mean degree ≈ 4.1 ("about 4"; the base tile is 2.0)
        tr = cKDTree(xyz[:, :2])
        pairs = tr.query_pairs(CHORD_MAX, output_type="ndarray")
        dd = np.linalg.norm(xyz[pairs[:, 0]] - xyz[pairs[:, 1]], axis=1)
        pairs = pairs[(dd >= CHORD_MIN) & (tile[pairs[:, 0]] == tile[pairs[:, 1]])]
        pairs = np.sort(pairs, axis=1)
        ek = np.sort(e2n, axis=1)
        n_all = np.int64(len(xyz))
        joined = np.isin(pairs[:, 0] * n_all + pairs[:, 1], ek[:, 0] * n_all + ek[:, 1])
        extra.append(pairs[~joined])
    if extra:
        ex = np.concatenate(extra)
        ex = np.sort(ex, axis=1)
        ex = ex[np.lexsort((ex[:, 1], ex[:, 0]))]
        e2n = np.concatenate([e2n, ex.astype(np.int64)])
    return xyz, e2n


def grips(xyz, tol=1.5):
    """Top/bottom grip bands (src/fea_solver.py:207-210, node_id == row)."""
    y = xyz[:, 1]
    top = np.flatnonzero(np.abs(y - y.max()) < tol)
    bot = np.flatnonzero(np.abs(y - y.min()) < tol)
    return top, bot


# benchmark configurations of BASELINE.json (tiles nx × ny)
CONFIGS = {
    "C1_test_I": None,
    "C2_100k": (1, 5),
    "C3_1M": (6, 8),
    "C5_10M_dense": (20, 23),
}


def write_mesh(d, xyz, e2n):
    os.makedirs(d, exist_ok=True)
    pd.DataFrame({"node_id": np.arange(len(xyz)), "x": xyz[:, 0], "y": xyz[:, 1], "z": xyz[:, 2]}) \
        .to_csv(os.path.join(d, "nodes.csv"), index=False)
    pd.DataFrame({"elem_id": np.arange(len(e2n)), "n1": e2n[:, 0], "n2": e2n[:, 1]}) \
        .to_csv(os.path.join(d, "elements.csv"), index=False)
