"""CPU: partitioning a given graph across ranks (gala/dist.py partition_graph / HaloExchange /
DistAggregator, SURVEY §8(e) for whole datasets such as config 5's Papers100M).

* Layout invariants on one process: vertex ranges balanced by edges, the monotone
  global -> Xs remap (every row keeps its CSR edge order), own/halo edge split, halo
  bookkeeping.
* gloo world 2 and 3: each rank fetches exactly its halo rows with grouped send/recv and
  aggregates with the host-CPU backend (libgala_cpu.so, the same per-row order and
  rounding as the HIP kernels).  exact mode must be BIT-identical to the one-process
  aggregation of the whole graph; overlap mode (own edges first, halo edges accumulated
  after) within fp32 rounding.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gala import _abi, dist as gdist, layout
from _graphs import cora_like, features, powerlaw, with_empty_rows

F = 12
GRAPHS = {"cora": cora_like, "powerlaw": powerlaw, "empty_rows": with_empty_rows}


# ---- host-CPU backend ops over torch CPU tensors (the injected local kernels) -----------
class _Csr:
    def __init__(self, g):
        self.g = g
        c = _abi.gala_csr_t()
        c.n_rows, c.n_cols, c.nnz = g.n_rows, g.n_cols, g.nnz
        c.rowptr, c.col, c.val = g.rowptr.ctypes.data, g.col.ctypes.data, None
        c.val_heads, c.n_seg, c.seg_bounds, c.split = 1, 1, None, None
        self.c = c


def _spmm(g, X, out, dst_scale, accum):
    import ctypes
    A = _Csr(g)
    flags = _abi.GALA_SPMM_ACCUM if accum else 0
    _abi.call_cpu("gala_spmm_f32", ctypes.byref(A.c), X.data_ptr(), X.stride(0), out.data_ptr(),
                  out.stride(0), X.shape[1], None, dst_scale.data_ptr(), flags, 0, 5, 7, None)
    return out


def _rb(s, X, out):
    _abi.call_cpu("gala_row_broadcast_f32", X.shape[0], X.shape[1], s.data_ptr(), X.data_ptr(),
                  X.stride(0), out.data_ptr(), out.stride(0), None)
    return out


def _degree(g):
    import ctypes
    out = torch.empty(g.n_rows)
    _abi.call_cpu("gala_degree_f32", ctypes.byref(_Csr(g).c), out.data_ptr(), -0.5, 0, 0, None)
    return out


def _one_process(g, X, layers=2):
    norm = _degree(g)
    H = torch.from_numpy(X)
    outs = []
    for _ in range(layers):
        Xs = _rb(norm, H, torch.empty_like(H))
        H = _spmm(g, Xs, torch.empty_like(H), norm, False)
        outs.append(H.numpy().copy())
    return outs


# ---- layout invariants ---------------------------------------------------------------------
@pytest.mark.parametrize("name", list(GRAPHS))
@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_partition_layout(name, world):
    g = GRAPHS[name]()
    b = gdist.row_bounds(g.rowptr, world)
    assert b[0] == 0 and b[-1] == g.n_rows and np.all(np.diff(b) >= 0)
    w = g.rowptr.astype(np.int64) + np.arange(g.n_rows + 1)
    heaviest = int(np.diff(w).max())
    for p in range(world):
        assert abs(int(w[b[p + 1]] - w[b[p]]) - w[-1] / world) <= heaviest + 1
    halo_total = 0
    for p in range(world):
        pt = gdist.partition_graph(g, p, world)
        r0, r1 = pt.r0, pt.r0 + pt.n
        x2g = pt.xs_to_global()
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
        # every own row keeps exactly its global edges, in CSR order
        e0, e1 = int(g.rowptr[r0]), int(g.rowptr[r1])
        np.testing.assert_array_equal(pt.graph.rowptr, g.rowptr[r0:r1 + 1] - e0)
        np.testing.assert_array_equal(x2g[pt.graph.col], g.col[e0:e1])
        # own + halo split: same edges, own columns inside the own slice
        og, hg = pt.own_graph, pt.halo_graph
        assert og.nnz + hg.nnz == pt.graph.nnz
        np.testing.assert_array_equal(np.diff(og.rowptr) + np.diff(hg.rowptr), np.diff(pt.graph.rowptr))
        assert np.all((og.col >= pt.lo) & (og.col < pt.lo + pt.n))
        assert np.all((hg.col < pt.lo) | (hg.col >= pt.lo + pt.n))
        halo_total += pt.halo.shape[0]
    if world == 1:
        assert halo_total == 0


def test_partition_rejects_tiled_or_rectangular():
    g = cora_like()
    with pytest.raises(ValueError):
        gdist.partition_graph(layout.HostGraph(g.n_rows, g.n_cols + 1, g.rowptr, g.col), 0, 2)
    with pytest.raises(ValueError):
        gdist.partition_graph(layout.col_tile(g, 1000), 0, 2)


# ---- gloo ranks -----------------------------------------------------------------------------
def _worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = GRAPHS[name]()
        X = features(g.n_rows, F, seed=11)
        pt = gdist.partition_graph(g, rank, world)
        res = {}
        for exact in (True, False):
            agg = gdist.DistAggregator(pt, F, "cpu", exact=exact, spmm=_spmm, row_broadcast=_rb,
                                       degree=_degree)
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
            res[exact] = gathered
        if rank == 0:
            q.put((res, [int(gdist.partition_graph(g, r, world).halo.shape[0]) for r in range(world)]))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,name", [(2, "powerlaw"), (3, "cora"), (3, "empty_rows")])
def test_distributed_aggregation_matches_one_process(world, name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, halos = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(halos) > 0
    g = GRAPHS[name]()
    ref = _one_process(g, features(g.n_rows, F, seed=11))
    for layer in range(2):
        np.testing.assert_array_equal(res[True][layer], ref[layer])     # bit-identical
        np.testing.assert_allclose(res[False][layer], ref[layer], rtol=1e-5, atol=1e-6)
