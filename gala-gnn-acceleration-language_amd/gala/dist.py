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


# ---- partitioning a given graph ----------------------------------------------------------
# SURVEY §8(e) for graphs that arrive whole (the reference's npy datasets, config 5): rank p
# owns the contiguous vertex range [bounds[p], bounds[p+1)) -- cut where the stored-edge
# count (plus one per row) crosses p/P of the total -- with all edges into those rows.
# Each rank's feature buffer Xs holds, in GLOBAL id order,
#     [ halo rows owned by ranks < p | own rows | halo rows owned by ranks > p ]
# so the remap global id -> Xs row is monotone and a row's edges keep their CSR order:
# one SpMM over `graph` sums every row in exactly the single-GPU (and reference) order,
# which makes the distributed result bit-identical to the one-GPU result.  The halo rows
# are fetched once per aggregation by point-to-point sends/receives straight into their
# Xs slices (RCCL grouped send/recv: only the rows a peer actually needs cross xGMI).
# Overlap mode instead runs the own-column edges (`own_graph`) while the halo is in
# flight and accumulates the halo edges (`halo_graph`) afterwards: faster, but a row's
# sum is then (own part) + (halo part), exact to fp32 rounding only.


def row_bounds(rowptr: np.ndarray, world: int) -> np.ndarray:
    """[world+1] vertex-range cuts balancing stored edges + rows per rank (deterministic:
    every rank computes the same cuts from the same rowptr)."""
    n = rowptr.shape[0] - 1
    w = rowptr.astype(np.int64) + np.arange(n + 1, dtype=np.int64)
    targets = (np.arange(1, world, dtype=np.int64) * int(w[-1])) // world
    cuts = np.searchsorted(w, targets, side="left")
    return np.concatenate([[0], cuts, [n]]).astype(np.int64)


def _csr_select(rowptr: np.ndarray, col: np.ndarray, keep: np.ndarray, n_cols: int) -> layout.HostGraph:
    """The rows' edges with keep[e] set, CSR order preserved."""
    n = rowptr.shape[0] - 1
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rowptr))
    rp = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(rows[keep], minlength=n), out=rp[1:])
    return layout.HostGraph(n, n_cols, rp.astype(np.int32), np.ascontiguousarray(col[keep], np.int32))


@dataclass
class GraphPartition:
    rank: int
    world: int
    bounds: np.ndarray          # int64 [world+1] global vertex ranges
    lo: int                     # halo rows owned by lower ranks: Xs[0:lo]
    halo: np.ndarray            # int64 global ids of all halo rows, ascending
    recv_counts: np.ndarray     # int64 [world] halo rows owned by each rank (0 for self)
    graph: layout.HostGraph     # own rows over the Xs columns, global edge order (exact)
    own_graph: layout.HostGraph   # the edges into own columns (overlap mode, first)
    halo_graph: layout.HostGraph  # the edges into halo columns (overlap mode, second)
    split_threshold: int = 0      # the WHOLE graph's hub-row threshold (ops.DeviceGraph.from_host):
                                  # the same rows split into the same chunks as on one GPU

    @property
    def r0(self) -> int:
        return int(self.bounds[self.rank])

    @property
    def n(self) -> int:
        return int(self.bounds[self.rank + 1] - self.bounds[self.rank])

    @property
    def n_cols(self) -> int:
        return self.n + int(self.halo.shape[0])

    @property
    def own_slice(self) -> slice:
        return slice(self.lo, self.lo + self.n)

    def recv_offsets(self) -> np.ndarray:
        """Xs row where the block received from rank q starts ([world])."""
        off = np.zeros(self.world, np.int64)
        pos = 0
        for q in range(self.world):
            if q == self.rank:
                pos = self.lo + self.n
                continue
            off[q] = pos
            pos += int(self.recv_counts[q])
        return off

    def xs_to_global(self) -> np.ndarray:
        """Global vertex id of every Xs row (int64 [n_cols])."""
        own = np.arange(self.r0, self.r0 + self.n, dtype=np.int64)
        return np.concatenate([self.halo[:self.lo], own, self.halo[self.lo:]])


def partition_graph(g: layout.HostGraph, rank: int, world: int,
                    bounds: np.ndarray | None = None) -> GraphPartition:
    """Rank `rank`'s share of the square one-segment graph `g` (rows = destinations)."""
    if g.n_rows != g.n_cols or g.n_seg != 1:
        raise ValueError("partition_graph needs a square, one-segment CSR")
    b = row_bounds(g.rowptr, world) if bounds is None else np.asarray(bounds, np.int64)
    r0, r1 = int(b[rank]), int(b[rank + 1])
    e0, e1 = int(g.rowptr[r0]), int(g.rowptr[r1])
    rp = (g.rowptr[r0:r1 + 1].astype(np.int64) - e0)
    cols = g.col[e0:e1].astype(np.int64)
    own = (cols >= r0) & (cols < r1)
    halo = np.unique(cols[~own])
    lo = int(np.searchsorted(halo, r0))
    n = r1 - r0
    xs_col = np.where(own, lo + (cols - r0), 0)
    hidx = np.searchsorted(halo, cols[~own])
    xs_col[~own] = np.where(hidx < lo, hidx, hidx + n)
    xs_col = xs_col.astype(np.int32)
    n_cols = n + int(halo.shape[0])
    owner = np.searchsorted(b, halo, side="right") - 1
    recv_counts = np.bincount(owner, minlength=world).astype(np.int64)
    graph = layout.HostGraph(n, n_cols, rp.astype(np.int32), xs_col)
    thr = max(1024, 8 * int(np.ceil(g.nnz / max(g.n_rows, 1))))
    return GraphPartition(rank, world, b, lo, halo, recv_counts, graph,
                          _csr_select(rp, xs_col, own, n_cols), _csr_select(rp, xs_col, ~own, n_cols), thr)


class HaloExchange:
    """Per-aggregation halo fetch for a GraphPartition: rank p sends every peer exactly
    the own rows that peer's edges read, received straight into the peer's Xs slices.

    Setup exchanges the request lists once (counts by all_to_all_single, ids by grouped
    send/recv); each call packs the rows to send with one index_select and issues one
    grouped batch of sends/receives (RCCL on the GPU, gloo on the CPU tests)."""

    def __init__(self, part: GraphPartition, device, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.part, self.group = torch, dist, part, group
        self.device = torch.device(device)
        P, p = part.world, part.rank
        recv = torch.from_numpy(part.recv_counts.copy()).to(self.device)
        send = torch.empty_like(recv)
        dist.all_to_all_single(send, recv, group=group)
        self.send_counts = send.cpu().numpy().astype(np.int64)
        self.recv_counts = part.recv_counts
        # my requests to q, as q-local row ids; q's requests to me -> my send rows
        owner = np.searchsorted(part.bounds, part.halo, side="right") - 1
        req = {q: torch.from_numpy((part.halo[owner == q] - part.bounds[q]).astype(np.int64)).to(self.device)
               for q in range(P) if q != p and self.recv_counts[q] > 0}
        got = {q: torch.empty(int(self.send_counts[q]), dtype=torch.int64, device=self.device)
               for q in range(P) if q != p and self.send_counts[q] > 0}
        ops = [dist.P2POp(dist.isend, req[q], q, group) for q in sorted(req)]
        ops += [dist.P2POp(dist.irecv, got[q], q, group) for q in sorted(got)]
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        self.send_peers = sorted(got)
        self.recv_peers = sorted(req)
        self.send_idx = (torch.cat([got[q] for q in self.send_peers]) if got
                         else torch.empty(0, dtype=torch.int64, device=self.device))
        self.send_off = np.concatenate([[0], np.cumsum([self.send_counts[q] for q in self.send_peers])]).astype(np.int64)
        self.recv_off = part.recv_offsets()
        self.sendbuf = None

    def start(self, Xs):
        """Pack and post the exchange for Xs (own rows already written); returns works."""
        torch, dist, part = self.torch, self.dist, self.part
        F = Xs.shape[1]
        if self.sendbuf is None or self.sendbuf.shape[1] != F:
            self.sendbuf = torch.empty((self.send_idx.shape[0], F), dtype=Xs.dtype, device=Xs.device)
        if self.send_idx.shape[0]:
            torch.index_select(Xs[part.own_slice], 0, self.send_idx, out=self.sendbuf)
        ops = [dist.P2POp(dist.isend, self.sendbuf[self.send_off[i]:self.send_off[i + 1]], q, self.group)
               for i, q in enumerate(self.send_peers)]
        ops += [dist.P2POp(dist.irecv, Xs[self.recv_off[q]:self.recv_off[q] + self.recv_counts[q]], q, self.group)
                for q in self.recv_peers]
        return dist.batch_isend_irecv(ops) if ops else []


class DistAggregator:
    """norm * A (norm * H) over a GraphPartition of a given graph (see the block comment
    above partition_graph).  exact=True: one SpMM after the halo arrives, bit-identical
    to the one-GPU aggregation; exact=False: own-column edges overlap the exchange.
    spmm / row_broadcast / degree default to the HIP ops (injectable for CPU tests)."""

    def __init__(self, part: GraphPartition, F: int, device, exact: bool = True, spmm=None,
                 row_broadcast=None, degree=None, group=None):
        import torch
        self.torch, self.part, self.F, self.exact = torch, part, F, exact
        if spmm is None:
            from . import ops
            spmm = lambda g, X, out, dst_scale, accum: ops.spmm(g, X, out=out, dst_scale=dst_scale, accum=accum)  # noqa: E731
            row_broadcast = lambda s, X, out: ops.row_broadcast(s, X, out=out)  # noqa: E731
            degree = lambda g: ops.degree(g, power=-0.5)  # noqa: E731
            mk = lambda hg: ops.DeviceGraph.from_host(hg, device, split=part.split_threshold)  # noqa: E731
        else:
            mk = lambda hg: hg  # noqa: E731
        self._spmm, self._rb = spmm, row_broadcast
        self.graph = mk(part.graph)
        self.own_graph = None if exact else mk(part.own_graph)
        self.halo_graph = None if exact else mk(part.halo_graph)
        self.norm = degree(self.graph)          # own rows' full degrees
        self.Xs = torch.empty((part.n_cols, F), device=device, dtype=torch.float32)
        self.exchange = HaloExchange(part, device, group) if part.world > 1 else None

    def __call__(self, H, out):
        p = self.part
        self._rb(self.norm, H, self.Xs[p.own_slice])                 # own rows of Xs = norm * H
        works = self.exchange.start(self.Xs) if self.exchange else []
        if self.exact:
            for w in works:
                w.wait()
            return self._spmm(self.graph, self.Xs, out, self.norm, False)
        self._spmm(self.own_graph, self.Xs, out, self.norm, False)   # overlaps the exchange
        for w in works:
            w.wait()
        return self._spmm(self.halo_graph, self.Xs, out, self.norm, True)
