"""Vertex-partitioned multi-GPU aggregation (one process per GPU, RCCL over xGMI).

SURVEY §8(e): graphs that shard naturally are cut into per-GPU partitions; a GPU owns
its vertices' feature rows and all edges whose destination it owns.  Edges whose source
lives on another GPU ("cut" edges) read that source's feature row from a halo buffer
filled by one RCCL all-gather of every partition's boundary rows per aggregation.

Per-rank layout (the reference's own column-tiled layout, src/ops/tiling.h:222-283, with
two segments):
    columns [0, n)            local vertices                       -> segment 0
    columns [n, n + P*b)      all partitions' boundary rows, rank q's  -> segment 1
                              block at n + q*b (the all-gather output)
Boundary vertices of a partition are its first b vertices, so the send buffer is a
contiguous slice of the (norm-prescaled) feature matrix: no pack kernel.

One aggregation  Y = norm * A (norm * H):
    Xs[0:n] = norm * H                         (gala_row_broadcast_f32)
    all_gather(Xs[n:], Xs[0:b])                 comm stream (RCCL)      } overlapped
    Y  = norm * A_local (Xs)                    compute stream, seg 0   }
    Y += norm * A_halo  (Xs)                    after the all-gather, seg 1 (ACCUM)

The synthetic partition generator (weak scaling: every rank owns an ogbn-products-sized
partition) draws local edges uniformly inside the partition and cut edges between the
boundary sets of two partitions; both endpoints' ranks derive the same cut edges from a
counter-based hash, so the global graph is symmetric.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import layout

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return x ^ (x >> np.uint64(31))


def _bounded(h: np.ndarray, n: int) -> np.ndarray:
    # high 32 bits * n >> 32 (n < 2^31): unbiased enough, deterministic, vectorised
    return ((h >> np.uint64(32)) * np.uint64(n)) >> np.uint64(32)


def cut_edges(p: int, q: int, count: int, b: int, seed: int):
    """The `count` cut edges between boundary sets of partitions p < q (u in B_p, v in B_q)."""
    assert p < q
    k = np.arange(count, dtype=np.uint64)
    base = np.uint64((seed * 1_000_003 + p * 4099 + q) & 0xFFFFFFFF) << np.uint64(32)
    u = _bounded(_splitmix64(base ^ (k * np.uint64(2))), b).astype(np.int32)
    v = _bounded(_splitmix64(base ^ (k * np.uint64(2) + np.uint64(1))), b).astype(np.int32)
    return u, v


@dataclass
class Partition:
    rank: int
    world: int
    n: int                   # local vertices
    b: int                   # boundary vertices per partition (first b local vertices)
    graph: layout.HostGraph  # n rows, n + world*b columns, 2 segments (local, halo)
    n_local_edges: int
    n_cut_edges: int

    @property
    def n_cols(self) -> int:
        return self.n + self.world * self.b


def make_partition(rank: int, world: int, n: int, edges_per_rank: int, cut_frac: float = 0.1,
                   boundary_frac: float = 0.1, seed: int = 42) -> Partition:
    """Rank `rank`'s partition: ~edges_per_rank stored edges incl. n self loops, of which
    ~cut_frac are cut edges to the other partitions' boundary vertices."""
    b = max(1, int(round(boundary_frac * n))) if world > 1 else 0
    cut_half = int(round(cut_frac * edges_per_rank)) if world > 1 else 0
    per_pair = cut_half // max(world - 1, 1)
    cut_half = per_pair * (world - 1)
    u_local = (edges_per_rank - n - cut_half) // 2
    hg = layout.gen_graph("uniform", n, u_local, seed=seed + 7919 * rank)
    rows = np.repeat(np.arange(n, dtype=np.int32), np.diff(hg.rowptr))
    src = [rows]
    dst = [hg.col]
    for q in range(world):
        if q == rank:
            continue
        p0, q0 = min(rank, q), max(rank, q)
        u, v = cut_edges(p0, q0, per_pair, b, seed)
        mine, theirs = (u, v) if rank == p0 else (v, u)
        src.append(mine)
        dst.append((n + q * b + theirs).astype(np.int32))
    src = np.concatenate(src)
    dst = np.concatenate(dst)
    n_cols = n + world * b
    g = layout.csr_build(n, n_cols, src, dst)
    if world > 1:
        bp = np.array([0, n, n_cols], np.int32)
        g = _tile(g, bp)
    return Partition(rank, world, n, b, g, int(hg.nnz), int(src.shape[0] - hg.nnz))


def _tile(g: layout.HostGraph, bp: np.ndarray) -> layout.HostGraph:
    from . import _abi
    S = bp.shape[0] - 1
    rp = np.empty((g.n_rows + 1) * S, np.int32)
    col = np.empty(g.nnz, np.int32)
    bounds = np.empty(2 * S, np.int32)
    _abi.call("gala_host_col_tile", g.n_rows, g.rowptr.ctypes.data, g.col.ctypes.data, None, S,
              bp.ctypes.data, rp.ctypes.data, col.ctypes.data, None, bounds.ctypes.data)
    return layout.HostGraph(g.n_rows, g.n_cols, rp, col, None, S, bounds)


def segment_view(g: layout.HostGraph, s: int) -> layout.HostGraph:
    """Segment s of a tiled graph as a stand-alone CSR (relative offsets, sliced cols)."""
    n = g.n_rows
    rp = g.rowptr[s * (n + 1):(s + 1) * (n + 1)]
    b0, b1 = int(g.bounds[2 * s]), int(g.bounds[2 * s + 1])
    return layout.HostGraph(n, g.n_cols, rp, g.col[b0:b1])


def global_reference_graph(parts: list[Partition]) -> layout.HostGraph:
    """Assemble the global graph (global vertex id = rank*n + local) for checking."""
    n, b, P = parts[0].n, parts[0].b, parts[0].world
    src, dst = [], []
    for pt in parts:
        g = pt.graph
        for s in range(g.n_seg):
            sg = segment_view(g, s)
            rows = np.repeat(np.arange(n), np.diff(sg.rowptr))
            cols = sg.col.astype(np.int64)
            gc = np.where(cols < n, pt.rank * n + cols, 0)
            halo = cols >= n
            q = (cols[halo] - n) // b
            gc[halo] = q * n + (cols[halo] - n - q * b)
            src.append(pt.rank * n + rows)
            dst.append(gc)
    src = np.concatenate(src).astype(np.int32)
    dst = np.concatenate(dst).astype(np.int32)
    return layout.csr_build(P * n, P * n, src, dst)


class DistGCNAggregator:
    """norm * A (norm * H) over a vertex-partitioned graph (see module docstring).

    spmm(g, X, out, dst_scale, accum) and row_broadcast(scale, X, out) are the local
    device ops (gala.ops on the GPU).  The CPU gloo test injects equivalent torch ops to
    exercise the partitioning, the halo indexing and the exchange without a GPU."""

    def __init__(self, part: Partition, F: int, device, spmm=None, row_broadcast=None,
                 degree=None, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.part, self.F, self.group = part, F, group
        if spmm is None:
            from . import ops
            spmm = lambda g, X, out, dst_scale, accum: ops.spmm(g, X, out=out, dst_scale=dst_scale, accum=accum)  # noqa: E731
            row_broadcast = lambda s, X, out: ops.row_broadcast(s, X, out=out)  # noqa: E731
            degree = lambda g: ops.degree(g, power=-0.5)  # noqa: E731
            mk = lambda hg: ops.DeviceGraph.from_host(hg, device)  # noqa: E731
        else:
            mk = lambda hg: hg  # noqa: E731
        self._spmm, self._rb = spmm, row_broadcast
        g = part.graph
        self.full = mk(g)
        self.segs = [mk(segment_view(g, s)) for s in range(g.n_seg)] if g.n_seg > 1 else [self.full]
        self.norm = degree(self.full)
        self.Xs = torch.empty((part.n_cols, F), device=device, dtype=torch.float32)
        self.is_cuda = torch.device(device).type == "cuda"
        self.comm_stream = torch.cuda.Stream(device=device) if self.is_cuda else None

    def __call__(self, H, out):
        torch, p = self.torch, self.part
        n, b = p.n, p.b
        self._rb(self.norm, H, self.Xs[:n])                         # Xs = norm * H
        if p.world == 1:
            return self._spmm(self.segs[0], self.Xs, out, self.norm, False)
        send = self.Xs[:b]
        recv = self.Xs[n:]
        if self.is_cuda:
            ready = torch.cuda.Event()
            ready.record()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ready)
                work = self.dist.all_gather_into_tensor(recv, send, group=self.group, async_op=True)
            self._spmm(self.segs[0], self.Xs, out, self.norm, False)     # local edges
            work.wait()                                                    # current stream waits
        else:
            self.dist.all_gather_into_tensor(recv, send, group=self.group)
            self._spmm(self.segs[0], self.Xs, out, self.norm, False)
        return self._spmm(self.segs[1], self.Xs, out, self.norm, True)  # cut edges, ACCUM
