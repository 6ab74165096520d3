"""World-size-2 CPU coverage of the multi-GPU path, over gloo.

Every process of the RCCL path builds its own partition plan from the whole
mesh (mfea_dist_init → mfea_set_mesh → partition.cpp build_partition), with no
negotiation: the plans must agree by construction.  Here two gloo ranks each
build their plan through the test shim and check, with collectives, that they
do — node ownership is a partition, every element is reported by exactly one
rank, the cut-element pair lists name the same elements in the same order on
both sides, and each rank's displacement-halo send list is its peer's receive
list.  Then the ranks run a distributed Jacobi-PCG on the CPU with the GPU
path's decomposition — owner-computes assembly of the local mesh (no
communication), one halo exchange of the cut free rows per operator
application, one all-reduce of the partial sums per iteration, the reaction
summed across ranks — and check it against the direct solve of the whole
system (src/fea_solver.py:112-135 via the oracle) and the reference's
iteration count (golden sys_sim_20251117_181147_step20.npz).

Replaces what src/fea_petsc_parallel.cpp does with PETSc's row-block
ownership (:234-268), MatMult ghost scatters and KSP dot-product allreduces
(:351), and its reaction gather (:400-428)."""
import ctypes as C
import os
import socket

import numpy as np
import pytest

from conftest import GOLDEN, build_host_shim, load_mesh

P = C.c_void_p
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shim():
    lib = C.CDLL(build_host_shim())
    lib.shim_part.restype = C.c_int
    lib.shim_part.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int64, P, C.c_int64, P, C.c_int,
                              C.c_int, C.c_int, P, C.c_char_p, C.c_int, C.c_double]
    lib.shim_part_arrays.argtypes = [P] * 12
    return lib


def _ptr(a):
    return a.ctypes.data_as(P)


def build_plan(xyz, e2n, top, bot, world, rank, axis=-1, slack=0.2):
    lib = _shim()
    xyz = np.ascontiguousarray(xyz, np.float64)
    e2n = np.ascontiguousarray(e2n, np.int64)
    top = np.ascontiguousarray(top, np.int64)
    bot = np.ascontiguousarray(bot, np.int64)
    sz = np.zeros(8, np.int64)
    err = C.create_string_buffer(256)
    rc = lib.shim_part(len(xyz), _ptr(xyz), len(e2n), _ptr(e2n), len(top), _ptr(top), len(bot),
                       _ptr(bot), world, rank, axis, _ptr(sz), err, 256, slack)
    assert rc == 0, err.value
    nl, el, npair, npeer, nx, nxs, nxr, _ = (int(v) for v in sz)
    p = {"node_g": np.empty(nl, np.int64), "ghost": np.empty(nl, np.uint8),
         "elem_g": np.empty(el, np.int64), "elem_own": np.empty(el, np.uint8),
         "elem_pair": np.empty(el, np.int32), "peers": np.empty(npeer, np.int32),
         "peer_cnt": np.empty(npeer, np.int64), "xpeers": np.empty(nx, np.int32),
         "xsend_cnt": np.empty(nx, np.int64), "xrecv_cnt": np.empty(nx, np.int64),
         "xsend_node": np.empty(nxs, np.int64), "xrecv_node": np.empty(nxr, np.int64)}
    lib.shim_part_arrays(*(_ptr(p[k]) for k in ("node_g", "ghost", "elem_g", "elem_own", "elem_pair",
                                                 "peers", "peer_cnt", "xpeers", "xsend_cnt",
                                                 "xrecv_cnt", "xsend_node", "xrecv_node")))
    p["n_pairs"] = npair
    p["axis"] = int(sz[7])
    return p


def test_partition_boundaries_follow_sparse_gaps():
    """Strip boundaries move (≤ 20 % of a strip) to the fewest crossing
    elements: on a tiled network they land in the gaps between tiles."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mycelium-fea-project_amd"))
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(6, 2)
    top, bot = synth.grips(xyz)
    known = np.zeros(len(xyz), bool)
    known[top] = known[bot] = True
    for world, sl in ((3, 0.2), (6, 0.2), (4, 0.4)):
        cuts = {}
        for slack in (0.0, sl):
            owned = [build_plan(xyz, e2n, top, bot, world, r, axis=0, slack=slack) for r in range(world)]
            own = np.full(len(xyz), -1)
            for r, p in enumerate(owned):
                own[p["node_g"][p["ghost"] == 0]] = r
            assert np.all(own >= 0)
            nfree = np.bincount(own[~known], minlength=world)
            if slack == 0:
                assert nfree.max() - nfree.min() <= 1
            else:
                assert np.all(np.abs(nfree - (~known).sum() / world) <= slack * (~known).sum() / world + 1)
            cuts[slack] = int(np.sum(own[e2n[:, 0]] != own[e2n[:, 1]]))
        print(world, cuts)
        assert cuts[sl] < cuts[0.0] / 3, (world, cuts)


def _split(arr, cnts):
    return np.split(arr, np.cumsum(cnts)[:-1]) if len(cnts) else []


# ---------------------------------------------------------------------------
def _worker(rank, world, port):
    import torch
    import torch.distributed as dist
    import fea_oracle as fo

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        _check_rank(rank, world, dist, torch, fo)
    finally:
        dist.destroy_process_group()


def _check_rank(rank, world, dist, torch, fo):
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    e2n = elems[["n1", "n2"]].values.astype(np.int64)
    N, E = len(xyz), len(e2n)
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    p = build_plan(xyz, e2n, top, bot, world, rank)

    # ---- plans agree across ranks (each rank built its own, no negotiation)
    allp = [None] * world
    dist.all_gather_object(allp, {k: (v.tolist() if isinstance(v, np.ndarray) else v)
                                  for k, v in p.items()})
    owned = np.zeros(N, np.int64)
    reported = np.zeros(E, np.int64)
    for q in allp:
        ng, gh = np.array(q["node_g"]), np.array(q["ghost"], bool)
        owned[ng[~gh]] += 1
        reported[np.array(q["elem_g"])[np.array(q["elem_own"], bool)]] += 1
    assert np.all(owned == 1), "node ownership must partition the nodes"
    assert np.all(reported == 1), "every element is reported by exactly one rank"
    me = allp[rank]
    eg = np.array(me["elem_g"])
    pairs = np.full(me["n_pairs"], -1, np.int64)
    ep = np.array(me["elem_pair"])
    pairs[ep[ep >= 0]] = eg[ep >= 0]
    for i, (peer, cnt) in enumerate(zip(me["peers"], me["peer_cnt"])):
        off = int(np.sum(me["peer_cnt"][:i]))
        mine = pairs[off: off + cnt]
        q = allp[peer]
        j = q["peers"].index(rank)
        qoff = int(np.sum(q["peer_cnt"][:j]))
        qpairs = np.full(q["n_pairs"], -1, np.int64)
        qep, qeg = np.array(q["elem_pair"]), np.array(q["elem_g"])
        qpairs[qep[qep >= 0]] = qeg[qep >= 0]
        assert np.array_equal(mine, qpairs[qoff: qoff + q["peer_cnt"][j]]), "pair lists differ"
    ng = np.array(me["node_g"])
    for i, peer in enumerate(me["xpeers"]):
        sends = _split(np.array(me["xsend_node"]), me["xsend_cnt"])[i]
        q = allp[peer]
        j = q["xpeers"].index(rank)
        recvs = _split(np.array(q["xrecv_node"]), q["xrecv_cnt"])[j]
        assert np.array_equal(ng[sends], np.array(q["node_g"])[recvs]), "halo lists differ"

    # ---- distributed Jacobi-PCG with the GPU path's exchange pattern
    z = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(z["dy"])
    nl = len(ng)
    g2l = np.full(N, -1, np.int64)
    g2l[ng] = np.arange(nl)
    le2n = g2l[e2n[eg]]
    assert np.all(le2n >= 0)
    # owner-computes assembly of the local mesh: rows of owned nodes are complete
    K = fo.assemble_global_stiffness(xyz[ng], le2n, np.ones(len(eg), bool)).tocsr()
    known_g = np.zeros(N, bool)
    known_g[top] = known_g[bot] = True
    val_g = np.zeros(N)
    val_g[top] = dy
    val_g[bot] = -dy  # bottom overrides top (src/fea_solver.py:226-242)
    gh = np.array(me["ghost"], bool)
    kn = known_g[ng]
    dof = lambda nodes_: (3 * nodes_[:, None] + np.arange(3)).ravel()  # noqa: E731
    own_free = np.flatnonzero(~gh & ~kn)
    loc_free = np.flatnonzero(~kn)            # owned + ghost free nodes
    loc_known = np.flatnonzero(kn)
    rows = dof(own_free)
    A = K[rows][:, dof(loc_free)].tocsr()
    A = A + 1e-12 * _embed_identity(own_free, loc_free)   # K_ff + reg·I (py:125)
    xk = np.zeros(3 * len(loc_known))
    xk[1::3] = val_g[ng[loc_known]]
    b = -(K[rows][:, dof(loc_known)] @ xk)
    pos = np.full(nl, -1, np.int64)
    pos[loc_free] = np.arange(len(loc_free))
    own_pos = dof(pos[own_free])
    dinv = 1.0 / A[:, own_pos].diagonal()

    xs = _split(np.array(me["xsend_node"]), me["xsend_cnt"])
    xr = _split(np.array(me["xrecv_node"]), me["xrecv_cnt"])

    def halo(v_own):
        """full local free vector: owned part + ghost rows from their owners."""
        full = np.zeros(3 * len(loc_free))
        full[own_pos] = v_own
        reqs, bufs = [], []
        for i, peer in enumerate(me["xpeers"]):
            out = torch.from_numpy(np.ascontiguousarray(full[dof(pos[xs[i]])]))
            inb = torch.empty(3 * len(xr[i]), dtype=torch.float64)
            reqs.append(dist.isend(out, peer))
            reqs.append(dist.irecv(inb, peer))
            bufs.append((i, inb))
        for r in reqs:
            r.wait()
        for i, inb in bufs:
            full[dof(pos[xr[i]])] = inb.numpy()
        return full

    def allsum(*vals):
        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t)
        return t.numpy()

    def pcg(rtol):
        x = np.zeros(len(rows))
        r = b.copy()
        zv = dinv * r
        pv = zv.copy()
        rho, rr, bb = allsum(r @ zv, r @ r, b @ b)
        it = 0
        while np.sqrt(rr) > rtol * np.sqrt(bb):
            q = A @ halo(pv)
            (pq,) = allsum(pv @ q)
            alpha = rho / pq
            x += alpha * pv
            r -= alpha * q
            zv = dinv * r
            rho_new, rr = allsum(r @ zv, r @ r)
            pv = zv + (rho_new / rho) * pv
            rho = rho_new
            it += 1
        return x, it

    _, it8 = pcg(1e-8)
    assert abs(it8 - int(z["pcg_iters_1e8"])) <= 3
    x, _ = pcg(1e-13)
    U_own = np.zeros(3 * N)
    rows_g = dof(ng[own_free])
    U_own[rows_g] = x
    Ut = torch.from_numpy(U_own)
    dist.all_reduce(Ut)                      # disjoint owned slices: a gather
    U = Ut.numpy()
    U[1::3][known_g] = val_g[known_g]
    assert np.linalg.norm(U - z["U"]) / np.linalg.norm(z["U"]) <= 1e-10
    # reaction: each rank sums K·U over its owned top rows; one scalar all-reduce
    own_top = np.flatnonzero(~gh & np.isin(ng, top))
    Ul = U[dof(ng)]
    (F,) = allsum(float(np.sum((K[3 * own_top + 1] @ Ul))))
    Kg = fo.assemble_global_stiffness(xyz, e2n, np.ones(E, bool))
    Fr = float(np.sum((Kg @ z["U"])[3 * top + 1]))
    assert abs(F - Fr) <= 1e-8 * abs(Fr)
    assert len(rows_g) == len(rows)


def _embed_identity(own_free, loc_free):
    import scipy.sparse as sp
    pos = {int(n): i for i, n in enumerate(loc_free)}
    cols = np.array([3 * pos[int(n)] + c for n in own_free for c in range(3)])
    return sp.csr_matrix((np.ones(len(cols)), (np.arange(len(cols)), cols)),
                         shape=(len(cols), 3 * len(loc_free)))


def test_partition_plans_agree_and_distributed_pcg_matches_direct():
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    assert torch.distributed.is_gloo_available()
    mp.spawn(_worker, args=(WORLD, _free_port()), nprocs=WORLD, join=True)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_plans_are_consistent_without_processes(world):
    """The same agreement checks for more ranks, plans built in one process."""
    import fea_oracle as fo
    nodes, elems = load_mesh("sim_20251117_175809")
    xyz = nodes[["x", "y", "z"]].values
    e2n = elems[["n1", "n2"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    plans = [build_plan(xyz, e2n, top, bot, world, r) for r in range(world)]
    owned = np.zeros(len(xyz), int)
    rep = np.zeros(len(e2n), int)
    for p in plans:
        owned[p["node_g"][p["ghost"] == 0]] += 1
        rep[p["elem_g"][p["elem_own"] == 1]] += 1
    assert np.all(owned == 1) and np.all(rep == 1)
    for r, p in enumerate(plans):
        for i, peer in enumerate(p["xpeers"]):
            q = plans[peer]
            j = list(q["xpeers"]).index(r)
            snd = _split(p["xsend_node"], p["xsend_cnt"])[i]
            rcv = _split(q["xrecv_node"], q["xrecv_cnt"])[j]
            assert np.array_equal(p["node_g"][snd], q["node_g"][rcv])
        # every ghost free node of a rank is received from its owner
        known = np.zeros(len(xyz), bool)
        known[top] = known[bot] = True
        ghost_free = p["node_g"][(p["ghost"] == 1) & ~known[p["node_g"]]]
        got = np.concatenate([p["node_g"][x] for x in _split(p["xrecv_node"], p["xrecv_cnt"])]) \
            if len(p["xrecv_cnt"]) else np.zeros(0, int)
        assert set(ghost_free.tolist()) == set(got.tolist())


# ---------------------------------------------------------------------------
# The multi-process drop-in's record gather (fea_solver.gather_records): rank 0
# receives every node's U and every element's stress / activity from its owner
# ---------------------------------------------------------------------------
def _gather_worker(rank, world, port, out_q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import fea_solver as fs
        N, E = 11, 7
        node_owner = np.arange(N) % world
        elem_owner = (np.arange(E) * 5) % world
        U = np.full(3 * N, np.nan)          # what a partitioned handle leaves in foreign entries
        S = np.full(E, np.nan)
        A = np.zeros(E, dtype=bool)
        mine_n, mine_e = node_owner == rank, elem_owner == rank
        ref_U = np.arange(3 * N, dtype=float) * 0.25 - 2.0
        ref_U[1::3] = -0.0                  # signed zeros must survive the gather
        ref_S = np.linspace(-1.0, 1.0, E)
        ref_A = np.arange(E) % 2 == 0
        U.reshape(-1, 3)[mine_n] = ref_U.reshape(-1, 3)[mine_n]
        S[mine_e] = ref_S[mine_e]
        A[mine_e] = ref_A[mine_e]
        rec = fs.gather_records(mine_n, mine_e, U, S, A, rank, world)
        if rank == 0:
            Ug, Sg, Ag = rec
            ok = (np.array_equal(Ug, ref_U) and np.array_equal(np.signbit(Ug), np.signbit(ref_U))
                  and np.array_equal(Sg, ref_S) and np.array_equal(Ag, ref_A))
            out_q.put(ok)
        else:
            out_q.put(rec is None)
    finally:
        dist.destroy_process_group()


def test_dropin_record_gather_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert all(q.get(timeout=10) for _ in range(WORLD))


def _sums_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rng = np.random.default_rng(100 + rank)
    mine = rng.standard_normal(4) * 10.0 ** rng.integers(-20, 20, 4)
    # capi.hip xchg_sums (dist_sums 1): every rank's [world][4] buffer zero but
    # its own row (k_amg_gsum zero_w), one all-reduce sum
    buf = torch.zeros(world, 4, dtype=torch.float64)
    buf[rank] = torch.from_numpy(mine)
    dist.all_reduce(buf)
    # ... equals the all-gather of the rows (the p2p form, dist_sums 0) bit for bit
    rows = [torch.zeros(4, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(rows, torch.from_numpy(mine))
    ok = bool(torch.equal(buf, torch.stack(rows)))
    # and every rank then sums the rows in rank order to the same bits
    s = np.zeros(4)
    for r in range(world):
        s = s + buf[r].numpy()
    allsum = [torch.zeros(4, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(allsum, torch.from_numpy(s))
    ok = ok and all(torch.equal(a, allsum[0]) for a in allsum)
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_cg_sums_allreduce_equals_rank_gather(world):
    """The GAMG CG's per-rank partial sums as one all-reduce of a zero-padded
    [world][4] buffer (capi.hip xchg_sums, option dist_sums 1) carry exactly
    the rows the send / receive pairs carried (x + 0 + … + 0 = x), so every
    rank forms bitwise the same α, β and stopping test as before."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_sums_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get() for _ in range(world))
    assert all(res[r] for r in range(world)), res
