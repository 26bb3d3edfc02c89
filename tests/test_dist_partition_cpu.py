"""CPU: partitioning one given graph across ranks (gala/dist.py row partitions
with a p2p or dense halo, gala/vertex_cut.py column ownership + reduce-scatter).

* Layout invariants on one process: vertex ranges balanced by edges, every own row keeps
  its global CSR edge order under the column remap, own/halo groups, halo bookkeeping;
  the vertex cut holds every edge of the graph exactly once across ranks.
* gloo world 2 and 3: the ranks aggregate with the host-CPU backend (libgala_cpu.so, the
  same per-row order and rounding as the HIP kernels).  Row-partition `exact` mode (p2p
  or dense halo) must be BIT-identical to the one-process aggregation of the whole graph;
  overlap / chunked modes and the vertex cut agree to fp32 rounding.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gala import dist as gdist, layout, vertex_cut as vc
from gala.backend import CpuBackend
from gala.comm import Comm
from _graphs import banded, cora_like, features, powerlaw, with_empty_rows

F = 12
GRAPHS = {"cora": cora_like, "powerlaw": powerlaw, "empty_rows": with_empty_rows, "banded": banded}


def _one_process(g, X, layers=2):
    be = CpuBackend()
    cg = be.graph(g)
    norm = be.degree(cg)
    H = torch.from_numpy(X)
    outs = []
    for _ in range(layers):
        Xs = be.row_broadcast(norm, H, torch.empty_like(H))
        H = be.spmm(cg, Xs, torch.empty_like(H), norm, False)
        outs.append(H.numpy().copy())
    return outs


# ---- layout invariants ---------------------------------------------------------------------
@pytest.mark.parametrize("name", list(GRAPHS))
@pytest.mark.parametrize("world", [1, 2, 3, 4])
@pytest.mark.parametrize("mode,chunks", [("p2p", 1), ("dense", 1), ("dense", 3)])
def test_partition_layout(name, world, mode, chunks):
    g = GRAPHS[name]()
    b = gdist.row_bounds(g.rowptr, world)
    assert b[0] == 0 and b[-1] == g.n_rows and np.all(np.diff(b) >= 0)
    w = g.rowptr.astype(np.int64) + np.arange(g.n_rows + 1)
    heaviest = int(np.diff(w).max())
    for p in range(world):
        assert abs(int(w[b[p + 1]] - w[b[p]]) - w[-1] / world) <= heaviest + 1
    halo_total = 0
    for p in range(world):
        pt = gdist.partition_graph(g, p, world, halo_mode=mode, chunks=chunks)
        assert pt.halo_mode == mode
        r0, r1 = pt.r0, pt.r0 + pt.n
        x2g = pt.xs_to_global()
        assert x2g.shape[0] == pt.n_cols
        # own rows are written where own_blocks says
        for j0, j1, x0 in pt.own_blocks():
            np.testing.assert_array_equal(x2g[x0:x0 + j1 - j0], np.arange(r0 + j0, r0 + j1))
        if mode == "p2p":
            assert np.all(np.diff(x2g) > 0)                       # monotone remap
            assert np.all((pt.halo < r0) | (pt.halo >= r1))
            assert pt.lo == int(np.sum(pt.halo < r0))
            assert int(pt.recv_counts.sum()) == pt.halo.shape[0] and pt.recv_counts[p] == 0
            owner = np.searchsorted(pt.bounds, pt.halo, side="right") - 1
            np.testing.assert_array_equal(np.bincount(owner, minlength=world), pt.recv_counts)
            off = pt.recv_offsets()
            for q in range(world):
                if q != p and pt.recv_counts[q]:
                    blk = x2g[off[q]:off[q] + pt.recv_counts[q]]
                    assert np.all((blk >= pt.bounds[q]) & (blk < pt.bounds[q + 1]))
            halo_total += pt.halo.shape[0]
        else:
            # every vertex has exactly one table row; the gather blocks are the owners'
            real = x2g[x2g >= 0]
            np.testing.assert_array_equal(np.sort(real), np.arange(g.n_rows))
            for t, own in pt.gather_slices():
                blk = x2g[own]
                blk = blk[blk >= 0]
                assert np.all((blk >= r0) & (blk < r1))
        # every own row keeps exactly its global edges, in CSR order
        e0, e1 = int(g.rowptr[r0]), int(g.rowptr[r1])
        np.testing.assert_array_equal(pt.graph.rowptr, g.rowptr[r0:r1 + 1] - e0)
        np.testing.assert_array_equal(x2g[pt.graph.col], g.col[e0:e1])
        # groups: a partition of the row's edges, own columns first, order kept per group
        assert len(pt.groups) == 1 + chunks
        assert sum(h.nnz for h in pt.groups) == pt.graph.nnz
        np.testing.assert_array_equal(sum(np.diff(h.rowptr) for h in pt.groups), np.diff(pt.graph.rowptr))
        og = pt.groups[0]
        assert np.all((x2g[og.col] >= r0) & (x2g[og.col] < r1))
        for h in pt.groups[1:]:
            assert np.all((x2g[h.col] < r0) | (x2g[h.col] >= r1))
    if world == 1 and mode == "p2p":
        assert halo_total == 0


def test_partition_rejects_tiled_or_rectangular():
    g = cora_like()
    with pytest.raises(ValueError):
        gdist.partition_graph(layout.HostGraph(g.n_rows, g.n_cols + 1, g.rowptr, g.col), 0, 2)
    with pytest.raises(ValueError):
        gdist.partition_graph(layout.col_tile(g, 1000), 0, 2)
    with pytest.raises(ValueError):
        gdist.partition_graph(g, 0, 2, halo_mode="p2p", chunks=2)
    with pytest.raises(ValueError):
        vc.vertex_cut_partition(layout.col_tile(g, 1000), 0, 2)


def test_dense_auto_mode_on_uniform_graph():
    # a uniform graph's halo is nearly every other vertex: auto picks the all-gather table
    g = cora_like()
    assert gdist.partition_graph(g, 0, 2).halo_mode == "dense"
    # a graph without cut edges has an empty halo: p2p
    blocks = layout.csr_build(100, 100, np.arange(100, dtype=np.int32), np.arange(100, dtype=np.int32))
    assert gdist.partition_graph(blocks, 0, 2).halo_mode == "p2p"


@pytest.mark.parametrize("name", list(GRAPHS))
@pytest.mark.parametrize("world,chunks", [(1, 1), (2, 1), (3, 2), (4, 3)])
def test_vertex_cut_layout(name, world, chunks):
    g = GRAPHS[name]()
    seen = []
    for p in range(world):
        pt = vc.vertex_cut_partition(g, p, world, chunks=chunks)
        c, P = pt.block, world
        assert pt.chunks == chunks and len(pt.chunk_graphs) == chunks and pt.exchange == "dense"
        assert c * chunks >= int(np.diff(pt.bounds).max())
        # degree graph: the own rows' full CSR (rowptr and col of matching length)
        dg = pt.deg_graph
        np.testing.assert_array_equal(np.diff(dg.rowptr), np.diff(g.rowptr)[pt.r0:pt.r0 + pt.n])
        assert int(dg.rowptr[-1]) == dg.nnz
        total = 0
        for k, h in enumerate(pt.chunk_graphs):
            assert h.n_rows == P * c and h.n_cols == pt.n
            assert h.nnz == 0 or (h.col.min() >= 0 and h.col.max() < pt.n)
            rows = np.repeat(np.arange(h.n_rows), np.diff(h.rowptr))
            q, jj = rows // c, rows % c
            j = k * c + jj
            assert np.all(j < np.diff(pt.bounds)[q])                 # padding rows stay empty
            grow = pt.bounds[q] + j
            seen.append(np.stack([grow, h.col.astype(np.int64) + pt.r0]))
            total += h.nnz
        assert total == pt.nnz
    allp = np.concatenate(seen, axis=1)
    rows = np.repeat(np.arange(g.n_rows), np.diff(g.rowptr))
    ref = np.stack([rows, g.col.astype(np.int64)])
    # every edge exactly once; and per row the held edges keep the CSR order
    key = lambda a: np.lexsort((a[1], a[0]))  # noqa: E731
    np.testing.assert_array_equal(allp[:, key(allp)], ref[:, key(ref)])


@pytest.mark.parametrize("name", list(GRAPHS))
@pytest.mark.parametrize("world,chunks", [(1, 1), (2, 1), (3, 2), (4, 3)])
def test_vertex_cut_sparse_layout(name, world, chunks):
    """DCSR send rows + receive CSR: a rank sends exactly the destination rows it holds
    edges of and its own rows (owner-major, ascending), every edge is held once, and what
    each owner's receive CSR expects from source q in chunk k is what q sends it, row for
    row."""
    g = GRAPHS[name]()
    parts = [vc.vertex_cut_partition(g, p, world, chunks=chunks, exchange="sparse") for p in range(world)]
    rows_all = np.repeat(np.arange(g.n_rows), np.diff(g.rowptr))
    seen = []
    sent = {}                                     # (src, dst, k) -> global rows sent, in order
    for pt in parts:
        sp, p = pt.sparse, pt.rank
        assert pt.exchange == "sparse" and len(sp.send_graphs) == chunks
        for k, h in enumerate(sp.send_graphs):
            rows = np.flatnonzero(np.repeat(True, h.n_rows))
            # recover the compact rows' global ids from their dense-layout positions
            d = sp.send_dense_rows[k] - k * world * pt.block
            q, j = d // pt.block, k * pt.block + d % pt.block
            grow = pt.bounds[q] + j
            assert np.all(np.diff(grow) > 0)                          # owner-major, ascending
            # only rows with a held edge, plus the rank's own rows (their own-vertex logits)
            assert np.all((np.diff(h.rowptr) > 0) | (q == p))
            np.testing.assert_array_equal(sp.send_self_cols[k], np.where(q == p, grow - pt.r0, -1))
            np.testing.assert_array_equal(np.bincount(q, minlength=world), sp.send_counts[k])
            er = np.repeat(grow, np.diff(h.rowptr))
            seen.append(np.stack([er, h.col.astype(np.int64) + pt.r0]))
            for qq in range(world):
                sent[(p, qq, k)] = grow[q == qq]
        assert sum(h.nnz for h in sp.send_graphs) == pt.nnz
    allp = np.concatenate(seen, axis=1)
    ref = np.stack([rows_all, g.col.astype(np.int64)])
    key = lambda a: np.lexsort((a[1], a[0]))  # noqa: E731
    np.testing.assert_array_equal(allp[:, key(allp)], ref[:, key(ref)])
    for pt in parts:                              # the receive side matches the senders
        sp, p = pt.sparse, pt.rank
        base = 0
        slot_row = {}
        for k in range(chunks):
            for q in range(world):
                blk = sent[(q, p, k)]
                assert blk.shape[0] == sp.recv_counts[k, q]
                for i, r in enumerate(blk):
                    slot_row[base + i] = (int(r), q)
                base += blk.shape[0]
        rg = sp.recv_graph
        assert rg.n_rows == pt.n
        for r in range(pt.n):
            ent = [slot_row[int(x)] for x in rg.col[rg.rowptr[r]:rg.rowptr[r + 1]]]
            assert all(gr == pt.r0 + r for gr, _ in ent)
            srcs = [q for _, q in ent]
            assert srcs == sorted(set(srcs))                          # source-rank order, once each


def test_touched_fraction_counts_pairs_whatever_the_column_order():
    """touched_fraction counts distinct remote (row, owner) pairs: the same on a graph whose
    rows hold their columns in any order, and equal to a direct count."""
    g = layout.gen_graph("rmat", 5000, 40000)
    rng = np.random.default_rng(1)
    col = g.col.copy()
    for r in range(0, g.n_rows, 3):
        a, b = int(g.rowptr[r]), int(g.rowptr[r + 1])
        col[a:b] = rng.permutation(col[a:b])
    shuffled = layout.HostGraph(g.n_rows, g.n_cols, g.rowptr, col)
    for P in (2, 3, 5):
        bnd = gdist.row_bounds(g.rowptr, P)
        rows = np.repeat(np.arange(g.n_rows), np.diff(g.rowptr.astype(np.int64)))
        ow = np.searchsorted(bnd, g.col, side="right") - 1
        far = ow != np.searchsorted(bnd, rows, side="right") - 1
        want = np.unique(rows[far] * P + ow[far]).shape[0] / (g.n_rows * (P - 1))
        assert vc.touched_fraction(g, bnd) == want
        assert vc.touched_fraction(shuffled, bnd) == want


def test_touched_fraction_and_auto_exchange():
    g = banded()
    b = gdist.row_bounds(g.rowptr, 4)
    f = vc.touched_fraction(g, b)
    assert 0 < f < 0.1                                  # locality: few remote (row, rank) pairs
    assert vc.vertex_cut_partition(g, 0, 4, exchange="auto").exchange == "sparse"
    u = cora_like()
    assert vc.touched_fraction(u, gdist.row_bounds(u.rowptr, 2)) > 0.5
    assert vc.vertex_cut_partition(u, 0, 2, exchange="auto").exchange == "dense"
    pt = vc.vertex_cut_partition(g, 1, 4, exchange="sparse")
    assert pt.comm_bytes(F) < vc.vertex_cut_partition(g, 1, 4).comm_bytes(F) / 5


# ---- gloo ranks -----------------------------------------------------------------------------
MODES = [("p2p", 1, True), ("p2p", 1, False), ("dense", 1, True), ("dense", 1, False),
         ("dense", 3, False), ("vcut", 1, None), ("vcut", 3, None), ("vcut-sparse", 1, None),
         ("vcut-sparse", 3, None)]


def _worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = GRAPHS[name]()
        X = features(g.n_rows, F, seed=11)
        be, comm = CpuBackend(), Comm()
        res = {}
        for mode, chunks, exact in MODES:
            if mode.startswith("vcut"):
                ex = "sparse" if mode == "vcut-sparse" else "dense"
                pt = vc.vertex_cut_partition(g, rank, world, chunks=chunks, exchange=ex)
                agg = vc.VertexCutAggregator(pt, F, be, comm)
            else:
                pt = gdist.partition_graph(g, rank, world, halo_mode=mode, chunks=chunks)
                agg = gdist.DistAggregator(pt, F, be, comm, exact=exact)
            H = torch.from_numpy(X[pt.r0:pt.r0 + pt.n].copy())
            outs = []
            for _ in range(2):                          # two layers reuse the halo buffers
                Y = torch.empty((pt.n, F))
                agg(H, Y)
                outs.append(Y)
                H = Y
            gathered = []
            sizes = [int(pt.bounds[r + 1] - pt.bounds[r]) for r in range(world)]
            for Y in outs:                              # gloo all_gather: equal sizes, so pad
                pad = torch.full((max(sizes), F), float("nan"))
                pad[:pt.n] = Y
                ys = [torch.empty_like(pad) for _ in sizes]
                dist.all_gather(ys, pad)
                gathered.append(torch.cat([y[:s] for y, s in zip(ys, sizes)]).numpy())
            res[(mode, chunks, exact)] = (gathered, agg.halo_bytes())
        if rank == 0:
            q.put(res)
        dist.barrier()      # every rank tears down together (gloo)
    finally:
        dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)   # skip library destructors: a gloo rank can abort in one at interpreter exit


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,name", [(2, "powerlaw"), (3, "cora"), (3, "empty_rows"), (3, "banded")])
def test_distributed_aggregation_matches_one_process(world, name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = GRAPHS[name]()
    ref = _one_process(g, features(g.n_rows, F, seed=11))
    for key, (got, hb) in res.items():
        mode, chunks, exact = key
        assert hb > 0 or (mode == "vcut-sparse" and name == "banded"), key
        for layer in range(2):
            if exact:
                np.testing.assert_array_equal(got[layer], ref[layer], err_msg=str(key))  # bit-identical
            else:
                np.testing.assert_allclose(got[layer], ref[layer], rtol=1e-5, atol=1e-6, err_msg=str(key))


# ---- vertex-cut GAT forward: softmax row statistics reduce-scattered -----------------------
H_GAT, F_GAT = 2, 8


def _gat_inputs(g):
    rng = np.random.default_rng(21)
    aL = rng.uniform(-1, 1, (g.n_rows, H_GAT)).astype(np.float32)
    aR = rng.uniform(-1, 1, (g.n_rows, H_GAT)).astype(np.float32)
    X = rng.uniform(-1, 1, (g.n_rows, F_GAT)).astype(np.float32)
    return aL, aR, X


def _gat_one_process(g):
    from gala import _abi
    aL, aR, X = _gat_inputs(g)
    be = CpuBackend()
    Y = torch.empty((g.n_rows, F_GAT))
    _abi.call_cpu("gala_gat_fwd_f32", be.graph(g).csr(), aL.ctypes.data, aR.ctypes.data, X.ctypes.data, F_GAT,
                  F_GAT, H_GAT, 0.2, _abi.GALA_SOFTMAX_REF, Y.data_ptr(), F_GAT, None, None)
    return Y.numpy()


def _gat_worker(rank, world, port, name, chunks, q, exchange="dense"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = GRAPHS[name]()
        aL, aR, X = _gat_inputs(g)
        pt = vc.vertex_cut_partition(g, rank, world, chunks=chunks, exchange=exchange)
        own = slice(pt.r0, pt.r0 + pt.n)
        gat = vc.VertexCutGat(pt, F_GAT, H_GAT, CpuBackend(), Comm())
        Y = gat(torch.from_numpy(aL[own].copy()), torch.from_numpy(aR[own].copy()), torch.from_numpy(X[own].copy()))
        sizes = [int(pt.bounds[r + 1] - pt.bounds[r]) for r in range(world)]
        pad = torch.full((max(sizes), F_GAT), float("nan"))
        pad[:pt.n] = Y
        ys = [torch.empty_like(pad) for _ in sizes]
        dist.all_gather(ys, pad)
        if rank == 0:
            q.put(torch.cat([y[:s] for y, s in zip(ys, sizes)]).numpy())
        dist.barrier()      # every rank tears down together (gloo)
    finally:
        dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)   # skip library destructors: a gloo rank can abort in one at interpreter exit


@pytest.mark.parametrize("world,name,chunks,exchange", [(2, "powerlaw", 1, "dense"), (3, "cora", 2, "dense"),
                                                        (3, "empty_rows", 1, "dense"), (2, "powerlaw", 2, "sparse"),
                                                        (3, "banded", 2, "sparse")])
def test_vertex_cut_gat_matches_one_process(world, name, chunks, exchange):
    """REF GAT forward with column ownership (VertexCutGat): per-rank unnormalised partial
    rows and softmax sums (GALA_GAT_PARTIAL on the host-CPU backend), reduce-scattered to
    the row owners, equal the one-process fused forward within fp32 rounding."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gat_worker, args=(r, world, port, name, chunks, q, exchange)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _gat_one_process(GRAPHS[name]())
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


# ---- vertex-cut GAT training: row statistics forward + REF backward -------------------------
def _gat_attn_weights():
    rng = np.random.default_rng(23)
    return rng.uniform(-0.5, 0.5, F_GAT).astype(np.float32), rng.uniform(-0.5, 0.5, H_GAT).astype(np.float32)


def _check_gat_against_oracle(g, got):
    """A distributed REF layer with the attention Linear (Y, dX, d_aL gathered over the
    ranks) against the oracle's pass-by-pass REF layer (orc_gat_ref_layer: edge sum,
    LeakyReLU, REF softmax, aggregation, and the REF backward chain), whose dX gets the
    attention Linear's term d_aL * wR, at 1e-4."""
    import oracle as orc
    aL, _, X = _gat_inputs(g)
    wR, bR = _gat_attn_weights()
    dY = np.random.default_rng(22).uniform(-1, 1, (g.n_rows, F_GAT)).astype(np.float32)
    lay = orc.GatRefLayer(g.rowptr, g.col, g.n_rows, X, dY, aL, wR, bR, H_GAT).run()
    D = F_GAT // H_GAT
    dX = lay.dX.astype(np.float64) + np.repeat(lay.daL.astype(np.float64), D, 1) * wR.astype(np.float64)
    for a, b, what in ((got[0], lay.Y, "Y"), (got[1], dX, "dX"), (got[2], lay.daL, "d_aL")):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-4, err_msg=what)


def _gat_train_one_process(g, rc=False):
    """Y, dX, d_aL of the REF layer on one process (gala_cpu_gat_{fwd,bwd}_stats_f32); rc:
    the source logits recomputed from X (wR, bR), dX then including the path through aR
    (d_aR = d_aL in REF mode), plus the Linear's gradients dwR, dbR."""
    from gala import _abi
    aL, aR, X = _gat_inputs(g)
    wR, bR = _gat_attn_weights()
    dY = np.random.default_rng(22).uniform(-1, 1, (g.n_rows, F_GAT)).astype(np.float32)
    be = CpuBackend()
    cg = be.graph(g)
    n = g.n_rows
    Y, Ym = torch.empty((n, F_GAT)), torch.empty((n, F_GAT))
    q, sma, aRo = torch.empty(n * H_GAT), torch.empty(n * H_GAT), torch.empty(n * H_GAT)
    _abi.call_cpu("gala_gat_fwd_stats_f32", cg.csr(), aL.ctypes.data, None if rc else aR.ctypes.data,
                  wR.ctypes.data if rc else None, bR.ctypes.data if rc else None, X.ctypes.data,
                  F_GAT, F_GAT, H_GAT, 0.2, Y.data_ptr(), F_GAT, q.data_ptr(), Ym.data_ptr(), F_GAT, sma.data_ptr(),
                  aRo.data_ptr() if rc else None, None, None)
    aR_b = aRo.view(n, H_GAT) if rc else torch.from_numpy(aR)
    dX, d_aL = be.gat_bwd_stats(cg, torch.from_numpy(aL), aR_b, torch.from_numpy(dY), q, Y, Ym,
                                sma, H_GAT, 0.2)
    d_aL = d_aL.view(n, H_GAT).numpy()
    out = [Y.numpy(), dX.numpy(), d_aL]
    if rc:   # float64 restatement of the Linear's backward over all rows
        D = F_GAT // H_GAT
        g64 = d_aL.astype(np.float64)
        dX = dX.numpy().astype(np.float64) + np.repeat(g64, D, 1) * np.tile(wR.astype(np.float64), 1)
        out[1] = dX
        dW = (np.repeat(g64, D, 1) * X.astype(np.float64)).sum(0)
        out += [dW, g64.sum(0)]
    return out


def _gat_train_worker(rank, world, port, name, chunks, q, rc=False, exchange="dense"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = GRAPHS[name]()
        aL, aR, X = _gat_inputs(g)
        dY = np.random.default_rng(22).uniform(-1, 1, (g.n_rows, F_GAT)).astype(np.float32)
        pt = vc.vertex_cut_partition(g, rank, world, chunks=chunks, exchange=exchange)
        own = slice(pt.r0, pt.r0 + pt.n)
        gat = vc.VertexCutGat(pt, F_GAT, H_GAT, CpuBackend(), Comm())
        t = lambda a: torch.from_numpy(a[own].copy())  # noqa: E731
        grads = []
        if rc:
            wR, bR = _gat_attn_weights()
            Y = gat.forward_train(t(aL), None, t(X), torch.from_numpy(wR), torch.from_numpy(bR))
            dX, d_aL, dW, db = gat.backward(t(dY))
            for G in (dW, db):                  # the caller's all-reduce of the Linear's grads
                dist.all_reduce(G)
                grads.append(G.numpy().copy())
        else:
            Y = gat.forward_train(t(aL), t(aR), t(X))
            dX, d_aL = gat.backward(t(dY))
        sizes = [int(pt.bounds[r + 1] - pt.bounds[r]) for r in range(world)]
        out = []
        for T in (Y, dX, d_aL):
            pad = torch.full((max(sizes), T.shape[1]), float("nan"))
            pad[:pt.n] = T
            ts = [torch.empty_like(pad) for _ in sizes]
            dist.all_gather(ts, pad)
            out.append(torch.cat([x[:s] for x, s in zip(ts, sizes)]).numpy())
        if rank == 0:
            q.put(out + grads)
        dist.barrier()      # every rank tears down together (gloo)
    finally:
        dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)   # skip library destructors: a gloo rank can abort in one at interpreter exit


@pytest.mark.parametrize("world,name,chunks,rc,exchange",
                         [(1, "cora", 2, False, "dense"), (2, "powerlaw", 1, False, "dense"),
                          (3, "cora", 2, False, "dense"), (3, "empty_rows", 1, False, "dense"),
                          (2, "cora", 1, True, "dense"), (3, "powerlaw", 2, True, "dense"),
                          (2, "powerlaw", 2, False, "sparse"), (3, "banded", 2, True, "sparse")])
def test_vertex_cut_gat_training_matches_one_process(world, name, chunks, rc, exchange):
    """VertexCutGat.forward_train / backward (gala_gat_fwd_partial_stats_f32 partials, one
    exchange per direction, d_aL from the owner's row statistics) against the one-process
    row-statistics pair: Y, dX and d_aL within fp32 rounding; with the source logits
    recomputed, dX includes the path through aR and the Linear's gradients match, and Y, dX,
    d_aL are within 1e-4 of the oracle's REF layer."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gat_train_worker, args=(r, world, port, name, chunks, q, rc, exchange))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _gat_train_one_process(GRAPHS[name](), rc)
    for a, b, what in zip(got, ref, ("Y", "dX", "d_aL", "dwR", "dbR")):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-4, err_msg=what)
    if rc:
        _check_gat_against_oracle(GRAPHS[name](), got)


def test_auto_halo_mode_is_one_choice_for_all_ranks():
    """The halo layout choice is made from every rank's halo share, so all ranks agree
    (their collectives must match) even on a skewed graph whose ranks' halos differ."""
    g = powerlaw()
    for world in (2, 3, 4):
        modes = {gdist.partition_graph(g, p, world).halo_mode for p in range(world)}
        assert len(modes) == 1
        fr = gdist.halo_fractions(g, gdist.row_bounds(g.rowptr, world))
        assert modes == {"dense" if fr.max() > 0.5 else "p2p"}


# ---- halo GAT: the one-GPU statistics kernels over a gathered table ----------------------------
def _halo_gat_worker(rank, world, port, name, rc, halo_mode, q, cls="HaloGat", chunks=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = GRAPHS[name]()
        aL, aR, X = _gat_inputs(g)
        dY = np.random.default_rng(22).uniform(-1, 1, (g.n_rows, F_GAT)).astype(np.float32)
        pt = gdist.partition_graph(g, rank, world, halo_mode=halo_mode, chunks=chunks)
        own = slice(pt.r0, pt.r0 + pt.n)
        gat = getattr(gdist, cls)(pt, F_GAT, H_GAT, CpuBackend(), Comm())
        t = lambda a: torch.from_numpy(a[own].copy())  # noqa: E731
        grads = []
        if rc:
            wR, bR = _gat_attn_weights()
            Xo = gat.own_rows("X") if chunks == 1 else t(X)
            Xo.copy_(t(X))                              # written in place: no copy in forward_train
            Y = gat.forward_train(t(aL), None, Xo, torch.from_numpy(wR), torch.from_numpy(bR))
            dX, d_aL, dW, db = gat.backward(t(dY))
            for G in (dW, db):
                dist.all_reduce(G)
                grads.append(G.numpy().copy())
        else:
            Y = gat.forward_train(t(aL), t(aR), t(X))
            dX, d_aL = gat.backward(t(dY))
        sizes = [int(pt.bounds[r + 1] - pt.bounds[r]) for r in range(world)]
        out = []
        for T in (Y, dX, d_aL):
            pad = torch.full((max(sizes), T.shape[1]), float("nan"))
            pad[:pt.n] = T
            ts = [torch.empty_like(pad) for _ in sizes]
            dist.all_gather(ts, pad)
            out.append(torch.cat([x[:s] for x, s in zip(ts, sizes)]).numpy())
        if rank == 0:
            q.put(out + grads)
        dist.barrier()      # every rank tears down together (gloo)
    finally:
        dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)   # skip library destructors: a gloo rank can abort in one at interpreter exit


@pytest.mark.parametrize("world,name,rc,halo_mode", [(2, "powerlaw", False, "p2p"), (3, "cora", True, "dense"),
                                                     (3, "banded", True, "p2p"), (2, "empty_rows", False, "dense")])
def test_halo_gat_bit_identical_to_one_process(world, name, rc, halo_mode):
    """HaloGat (gala/dist.py): each rank runs the one-process statistics kernels over its rows
    with the pattern's columns in the gathered table (gala_cpu_gat_{fwd,bwd}_stats_ex_f32):
    Y, dX and d_aL are bit-identical to the one-process pair, the Linear's gradients within
    fp32 rounding (summed over ranks); with the attention Linear, Y, dX and d_aL are also
    within 1e-4 of the oracle's REF layer (the reference's pass sequence)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_gat_worker, args=(r, world, port, name, rc, halo_mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = GRAPHS[name]()
    ref = _gat_train_one_process(g, rc)
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[2], ref[2])
    if rc:     # the one-process reference adds the Linear path in float64
        np.testing.assert_allclose(got[1], ref[1], rtol=1e-5, atol=1e-6)
        for a, b in zip(got[3:], ref[3:]):
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-4)
        _check_gat_against_oracle(g, got)
    else:
        np.testing.assert_array_equal(got[1], ref[1])


@pytest.mark.parametrize("world,name,rc,halo_mode,chunks", [(2, "powerlaw", False, "p2p", 1),
                                                            (3, "cora", True, "dense", 1),
                                                            (3, "banded", True, "p2p", 1),
                                                            (2, "empty_rows", False, "dense", 1),
                                                            (3, "cora", True, "dense", 3),
                                                            (2, "powerlaw", False, "dense", 2)])
def test_halo_gat_overlap_matches_one_process(world, name, rc, halo_mode, chunks):
    """HaloGatOverlap (gala/dist.py): the own-column partial statistics overlap the exchange and
    every halo chunk continues them as it lands (a dense table gathered in 1-3 row chunks) --
    each row's sums grouped per range, so Y, dX and d_aL agree with the one-process pair to
    fp32 rounding (not bit for bit)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_gat_worker, args=(r, world, port, name, rc, halo_mode, q, "HaloGatOverlap",
                                                        chunks))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _gat_train_one_process(GRAPHS[name](), rc)
    for a, b in zip(got, ref):
        assert np.isfinite(a).all()
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5 * max(1.0, float(np.abs(b).max())))
