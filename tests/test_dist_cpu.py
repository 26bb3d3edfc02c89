"""CPU, world_size 2 (gloo): the vertex-partitioned aggregation (gala/dist.py).

Each rank builds its partition, exchanges boundary rows with all_gather_into_tensor and
aggregates local + cut edges; the gathered result must equal norm * A (norm * X) on the
assembled global graph.  The test exercises the partitioning, the halo column mapping,
the collective and the two-segment accumulation order of the distributed path.  The
local kernels run on the host-CPU backend (libgala_cpu.so).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gala import dist as gdist
from gala import layout
from gala.backend import CpuBackend
from gala.comm import Comm

N_LOCAL, EDGES, F = 600, 7000, 8


def _csr_mm(hg: layout.HostGraph, X: torch.Tensor) -> torch.Tensor:
    rows = np.repeat(np.arange(hg.n_rows), np.diff(hg.rowptr))
    out = torch.zeros((hg.n_rows, X.shape[1]), dtype=torch.float64)
    out.index_add_(0, torch.from_numpy(rows), X.double()[torch.from_numpy(hg.col.astype(np.int64))])
    return out


def _features(world):
    rng = np.random.default_rng(5)
    return rng.uniform(-1, 1, (world * N_LOCAL, F)).astype(np.float32)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        part = gdist.make_partition(rank, world, N_LOCAL, EDGES, cut_frac=0.2, boundary_frac=0.1, seed=9)
        agg = gdist.DistGCNAggregator(part, F, CpuBackend(), Comm())
        Xg = _features(world)
        H = torch.from_numpy(Xg[rank * N_LOCAL:(rank + 1) * N_LOCAL])
        Y = torch.empty((N_LOCAL, F))
        agg(H, Y)
        Y2 = torch.empty_like(Y)
        agg(Y, Y2)  # second layer reuses the halo buffer
        ys = [torch.empty_like(Y) for _ in range(world)]
        dist.all_gather(ys, Y)
        ys2 = [torch.empty_like(Y2) for _ in range(world)]
        dist.all_gather(ys2, Y2)
        if rank == 0:
            q.put((torch.cat(ys).numpy(), torch.cat(ys2).numpy(), part.n_cut_edges))
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


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_aggregation_matches_global(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    Y, Y2, ncut = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ncut > 0
    parts = [gdist.make_partition(r, world, N_LOCAL, EDGES, cut_frac=0.2, boundary_frac=0.1, seed=9)
             for r in range(world)]
    G = gdist.global_reference_graph(parts)
    t, _ = layout.transpose(G)      # the generator keeps the global graph symmetric
    np.testing.assert_array_equal(t.rowptr, G.rowptr)
    np.testing.assert_array_equal(t.col, G.col)
    norm = torch.from_numpy(G.degrees().astype(np.float64) ** -0.5)
    X = torch.from_numpy(_features(world)).double()
    ref = norm[:, None] * _csr_mm(G, norm[:, None] * X)
    np.testing.assert_allclose(Y, ref.numpy(), atol=1e-5, rtol=1e-5)
    ref2 = norm[:, None] * _csr_mm(G, norm[:, None] * torch.from_numpy(Y).double())
    np.testing.assert_allclose(Y2, ref2.numpy(), atol=1e-5, rtol=1e-5)


def test_partition_shapes_and_cut_fraction():
    parts = [gdist.make_partition(r, 4, 1000, 20000, cut_frac=0.1, boundary_frac=0.1, seed=1) for r in range(4)]
    for p in parts:
        g = p.graph
        assert g.n_seg == 2 and g.n_rows == 1000 and g.n_cols == 1000 + 4 * 100
        assert abs(g.nnz - 20000) < 20
        halo = g.bounds[3] - g.bounds[2]
        assert halo == p.n_cut_edges and abs(halo / g.nnz - 0.1) < 0.01
        seg1 = gdist.segment_view(g, 1)
        assert seg1.col.min() >= 1000
        own = (seg1.col >= 1000 + p.rank * 100) & (seg1.col < 1000 + (p.rank + 1) * 100)
        assert not own.any()  # no cut edge points into the own boundary block


def test_single_rank_partition_is_the_headline_graph():
    p = gdist.make_partition(0, 1, 2000, 2000 + 2 * 7000, seed=42)
    g = layout.gen_graph("uniform", 2000, 7000, seed=42)
    np.testing.assert_array_equal(p.graph.rowptr, g.rowptr)
    np.testing.assert_array_equal(p.graph.col, g.col)
