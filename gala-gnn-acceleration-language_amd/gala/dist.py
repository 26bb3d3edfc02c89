"""Multi-GPU aggregation by vertex partitions (one process per GPU, RCCL over xGMI).

The reference is single-GPU (no collectives anywhere); this is new work
scoped by SURVEY §8(e).  Two families live in this package:

* **Row partitions with a halo** (this module).  Rank p owns the vertex range
  [bounds[p], bounds[p+1)) -- its rows of A (the destinations) and their feature rows.
  The columns an own row reads from other ranks (the halo) are fetched once per
  aggregation, then the rank runs the SpMM over its rows.  The halo arrives either
    - "p2p":   each peer sends exactly the rows this rank's edges read (grouped RCCL
               send/recv, request lists exchanged once at setup), or
    - "dense": one RCCL all-gather of every rank's rows into a padded table (used when
               the halo is most of the graph -- a uniform graph at any P -- where the
               all-gather moves the same bytes with RCCL's best algorithm).  The table
               may be gathered in K row chunks so SpMM work overlaps the transfer.
  `exact` mode runs ONE SpMM over the rank's rows once the halo is complete.  Its column
  ids are remapped but every row keeps its CSR edge order, so the result is bit-identical
  to the one-GPU (and reference) aggregation.  Overlap mode runs the own-column edges
  while the halo is in flight and accumulates each halo chunk's edges when it lands
  (exact to fp32 rounding only: a row's sum is split into per-chunk partial sums).
* **Vertex cut** (gala/vertex_cut.py): rank p owns the columns of its range; partial
  rows are summed into their owners by RCCL reduce-scatter.

Layouts follow the reference's column-tiled CSR (src/ops/tiling.h:222-283): a group of
edges selected by column range, relative row offsets, rows in global order.

The weak-scaling generator at the top (make_partition / DistGCNAggregator) builds one
ogbn-products-sized partition per rank with synthetic cut edges; bench.py reports it as
the secondary weak-scaling number next to the strong-scaling run of one graph.
"""
from __future__ import annotations

from dataclasses import dataclass, field

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


# ---- weak scaling: one synthetic partition per rank ---------------------------------------
# Per-rank layout (two column segments of the tiled layout):
#     columns [0, n)            local vertices                        -> segment 0
#     columns [n, n + P*b)      every partition's boundary rows, rank q's block at n + q*b
#                               (the all-gather output)               -> segment 1
# Boundary vertices of a partition are its first b vertices, so the all-gather's send
# buffer is a contiguous slice of the (norm-prescaled) features: no pack kernel.

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
    """norm * A (norm * H) over a synthetic weak-scaling Partition: the local-edge SpMM
    (segment 0) overlaps the all-gather of the boundary rows, the cut edges (segment 1)
    accumulate after it.  `backend` is gala.backend.HipBackend / CpuBackend."""

    def __init__(self, part: Partition, F: int, backend, comm=None):
        self.part, self.F, self.be = part, F, backend
        self.comm = comm
        g = part.graph
        self.full = backend.graph(g)
        self.segs = [backend.graph(segment_view(g, s)) for s in range(g.n_seg)] if g.n_seg > 1 else [self.full]
        self.norm = backend.degree(self.full)
        self.Xs = backend.empty(part.n_cols, F)

    def refresh_norm(self):
        """Recompute the degree norm (the generated forward does, gala.cu:433-440)."""
        self.norm = self.be.degree(self.full)

    def __call__(self, H, out):
        be, p = self.be, self.part
        n, b = p.n, p.b
        be.row_broadcast(self.norm, H, self.Xs[:n])                       # Xs = norm * H
        if p.world == 1:
            return be.spmm(self.segs[0], self.Xs, out, self.norm, False)
        work = self.comm.all_gather(self.Xs[n:], self.Xs[:b])
        be.spmm(self.segs[0], self.Xs, out, self.norm, False)             # local edges, overlapped
        self.comm.wait([work])
        return be.spmm(self.segs[1], self.Xs, out, self.norm, True)       # cut edges, ACCUM

    def halo_bytes(self) -> int:
        return 4 * self.F * self.part.b * (self.part.world - 1)


# ---- strong scaling: partitioning one given graph -----------------------------------------

def row_bounds(rowptr: np.ndarray, world: int) -> np.ndarray:
    """[world+1] vertex-range cuts balancing stored edges + rows per rank (deterministic:
    every rank computes the same cuts from the same rowptr)."""
    n = rowptr.shape[0] - 1
    w = rowptr.astype(np.int64) + np.arange(n + 1, dtype=np.int64)
    targets = (np.arange(1, world, dtype=np.int64) * int(w[-1])) // world
    cuts = np.searchsorted(w, targets, side="left")
    return np.concatenate([[0], cuts, [n]]).astype(np.int64)


def _rowptr_of_selected(rowptr: np.ndarray, keep: np.ndarray) -> np.ndarray:
    """Row offsets of the CSR restricted to the edges with keep[e] (CSR order kept)."""
    cs = np.zeros(keep.shape[0] + 1, np.int64)
    np.cumsum(keep, out=cs[1:])
    return (cs[rowptr.astype(np.int64)] - cs[int(rowptr[0])]).astype(np.int32)


@dataclass
class GraphPartition:
    """Rank `rank`'s rows of one graph and the column layout of its feature buffer Xs.

    halo_mode "p2p":   Xs = [halo rows of lower ranks | own rows | halo rows of higher
                       ranks], in global id order (only the rows this rank reads).
    halo_mode "dense": Xs = a padded table of ALL rows, gathered in `chunks` row chunks;
                       owner q's local row j sits at k*P*c + q*c + (j - k*c), k = j // c,
                       c = `block` rows per (rank, chunk).
    `graph` has the rank's rows with every edge (global CSR order, remapped columns);
    `groups[0]` its own-column edges and `groups[1 + k]` the edges into halo chunk k."""
    rank: int
    world: int
    bounds: np.ndarray          # int64 [world+1] global vertex ranges
    halo_mode: str
    chunks: int
    block: int                  # dense: rows per (rank, chunk) block
    lo: int                     # p2p: Xs row of own row 0
    halo: np.ndarray            # p2p: int64 global ids of all halo rows, ascending
    recv_counts: np.ndarray     # p2p: int64 [world] halo rows owned by each rank (0 for self)
    n_cols: int                 # rows of Xs
    graph: layout.HostGraph
    groups: list = field(default_factory=list)
    split_threshold: int = 0      # the WHOLE graph's hub-row threshold: the same rows split
                                  # into the same chunks as on one GPU
    n_halo_rows: int = 0          # distinct non-own rows this rank's edges read

    @property
    def r0(self) -> int:
        return int(self.bounds[self.rank])

    @property
    def n(self) -> int:
        return int(self.bounds[self.rank + 1] - self.bounds[self.rank])

    @property
    def own_graph(self) -> layout.HostGraph:
        return self.groups[0]

    @property
    def halo_graph(self) -> layout.HostGraph:
        if len(self.groups) != 2:
            raise ValueError("halo_graph: one halo chunk only")
        return self.groups[1]

    def own_blocks(self):
        """[(first own row, end own row, Xs row)] where the own rows are written."""
        if self.halo_mode == "p2p":
            return [(0, self.n, self.lo)]
        c, P, p = self.block, self.world, self.rank
        out = []
        for k in range(self.chunks):
            j0, j1 = k * c, min((k + 1) * c, self.n)
            if j1 > j0:
                out.append((j0, j1, k * P * c + p * c))
        return out

    def own_offset(self) -> int:
        """Table row of own row 0 when the own rows are one block (p2p, or dense with one
        chunk); defined for a rank without rows too."""
        if self.halo_mode == "p2p":
            return self.lo
        if self.chunks != 1:
            raise ValueError("own rows are one block only with one chunk")
        return self.rank * self.block

    def gather_slices(self):
        """dense: [(table rows of chunk k, this rank's block in it)] for the all-gathers."""
        c, P, p = self.block, self.world, self.rank
        return [(slice(k * P * c, (k + 1) * P * c), slice(k * P * c + p * c, k * P * c + (p + 1) * c))
                for k in range(self.chunks)]

    @property
    def own_slice(self) -> slice:
        if self.halo_mode != "p2p":
            raise ValueError("own rows are not contiguous in a dense table")
        return slice(self.lo, self.lo + self.n)

    def recv_offsets(self) -> np.ndarray:
        """p2p: Xs row where the block received from rank q starts ([world])."""
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
        """Global vertex id held by every Xs row (int64 [n_cols]; -1 for padding)."""
        if self.halo_mode == "p2p":
            own = np.arange(self.r0, self.r0 + self.n, dtype=np.int64)
            return np.concatenate([self.halo[:self.lo], own, self.halo[self.lo:]])
        out = np.full(self.n_cols, -1, np.int64)
        N = int(self.bounds[-1])
        out[_dense_map(self.bounds, self.block, self.world, N)] = np.arange(N, dtype=np.int64)
        return out

    def halo_bytes(self, F: int) -> int:
        """Bytes this rank receives per aggregation."""
        if self.halo_mode == "p2p":
            return 4 * F * int(self.recv_counts.sum())
        return 4 * F * self.block * self.chunks * (self.world - 1)


def _dense_map(bounds: np.ndarray, c: int, P: int, N: int) -> np.ndarray:
    """Global id -> dense-table row (int64 [N])."""
    out = np.empty(N, np.int64)
    for q in range(P):
        j = np.arange(int(bounds[q + 1] - bounds[q]), dtype=np.int64)
        k = j // c
        out[int(bounds[q]):int(bounds[q + 1])] = k * P * c + q * c + (j - k * c)
    return out


def halo_fractions(g: layout.HostGraph, bounds: np.ndarray) -> np.ndarray:
    """Per rank: distinct non-own rows its edges read / the other ranks' rows.  Every rank
    computes the same array from the same graph, so choices made from it agree."""
    N, P = g.n_rows, bounds.shape[0] - 1
    out = np.zeros(P)
    used = np.zeros(N, bool)
    for q in range(P):
        r0, r1 = int(bounds[q]), int(bounds[q + 1])
        used[:] = False
        used[g.col[int(g.rowptr[r0]):int(g.rowptr[r1])]] = True
        used[r0:r1] = False
        out[q] = used.sum() / max(N - (r1 - r0), 1)
    return out


def partition_graph(g: layout.HostGraph, rank: int, world: int, bounds: np.ndarray | None = None,
                    halo_mode: str = "auto", chunks: int = 1, dense_frac: float = 0.5) -> GraphPartition:
    """Rank `rank`'s share of the square one-segment graph `g` (rows = destinations).
    halo_mode "auto" picks "dense" when the halo exceeds dense_frac of the other ranks'
    rows (then an all-gather moves no more than point-to-point would); chunks > 1 needs
    the dense table (the p2p layout has one halo group)."""
    if g.n_rows != g.n_cols or g.n_seg != 1:
        raise ValueError("partition_graph needs a square, one-segment CSR")
    N = g.n_rows
    b = row_bounds(g.rowptr, world) if bounds is None else np.asarray(bounds, np.int64)
    r0, r1 = int(b[rank]), int(b[rank + 1])
    n = r1 - r0
    e0, e1 = int(g.rowptr[r0]), int(g.rowptr[r1])
    rp = (g.rowptr[r0:r1 + 1].astype(np.int64) - e0).astype(np.int32)
    cols = g.col[e0:e1]
    own = (cols >= r0) & (cols < r1)
    used = np.zeros(N, bool)
    used[cols] = True
    used[r0:r1] = False
    n_halo = int(used.sum())
    if halo_mode == "auto":
        # one decision for all ranks (their collectives must match): the largest halo share
        halo_mode = "dense" if (chunks > 1 or halo_fractions(g, b).max() > dense_frac) else "p2p"
    if halo_mode == "p2p" and chunks != 1:
        raise ValueError("the p2p halo has one chunk")
    thr = layout.split_threshold(g.n_rows, g.nnz)
    if halo_mode == "p2p":
        halo = np.flatnonzero(used).astype(np.int64)
        lo = int(np.searchsorted(halo, r0))
        xmap = np.full(N, -1, np.int64)
        xmap[halo[:lo]] = np.arange(lo)
        xmap[r0:r1] = lo + np.arange(n)
        xmap[halo[lo:]] = lo + n + np.arange(halo.shape[0] - lo)
        n_cols = n + halo.shape[0]
        owner = np.searchsorted(b, halo, side="right") - 1
        recv_counts = np.bincount(owner, minlength=world).astype(np.int64)
        block, K = 0, 1
    else:
        K = max(int(chunks), 1)
        m = int(np.diff(b).max(initial=0))
        block = max((m + K - 1) // K, 1)
        xmap = _dense_map(b, block, world, N)
        n_cols = K * world * block
        halo, lo, recv_counts = np.zeros(0, np.int64), 0, np.zeros(world, np.int64)
    xs_col = xmap[cols].astype(np.int32)
    graph = layout.HostGraph(n, n_cols, rp, xs_col)
    groups = [layout.HostGraph(n, n_cols, _rowptr_of_selected(rp, own), xs_col[own])]
    if halo_mode == "p2p":
        groups.append(layout.HostGraph(n, n_cols, _rowptr_of_selected(rp, ~own), xs_col[~own]))
    else:
        kcol = (xs_col // (world * block)).astype(np.int32)
        for k in range(K):
            sel = ~own & (kcol == k)
            groups.append(layout.HostGraph(n, n_cols, _rowptr_of_selected(rp, sel), xs_col[sel]))
    return GraphPartition(rank, world, b, halo_mode, K, block, lo, halo, recv_counts, n_cols, graph,
                          groups, thr, n_halo)


class HaloExchange:
    """p2p halo of a GraphPartition: rank p sends every peer exactly the own rows that
    peer's edges read, received straight into the peer's Xs slices.  Setup exchanges the
    request lists once (counts by all_to_all_single, ids by grouped send/recv); each call
    packs the rows to send with one index_select and posts one grouped send/recv batch."""

    def __init__(self, part: GraphPartition, comm, device):
        import torch
        self.torch, self.part, self.comm = torch, part, comm
        self.device = torch.device(device)
        P, p = part.world, part.rank
        recv = torch.from_numpy(part.recv_counts.copy()).to(self.device)
        send = torch.empty_like(recv)
        comm.all_to_all_single(send, recv)
        self.send_counts = send.cpu().numpy().astype(np.int64)
        self.recv_counts = part.recv_counts
        # my requests to q, as q-local row ids; q's requests to me -> my send rows
        owner = np.searchsorted(part.bounds, part.halo, side="right") - 1
        req = {q: torch.from_numpy((part.halo[owner == q] - part.bounds[q]).astype(np.int64)).to(self.device)
               for q in range(P) if q != p and self.recv_counts[q] > 0}
        got = {q: torch.empty(int(self.send_counts[q]), dtype=torch.int64, device=self.device)
               for q in range(P) if q != p and self.send_counts[q] > 0}
        comm.wait(comm.exchange([(req[q], q) for q in sorted(req)], [(got[q], q) for q in sorted(got)]))
        self.send_peers = sorted(got)
        self.recv_peers = sorted(req)
        self.send_idx = (torch.cat([got[q] for q in self.send_peers]) if got
                         else torch.empty(0, dtype=torch.int64, device=self.device))
        self.send_off = np.concatenate([[0], np.cumsum([self.send_counts[q] for q in self.send_peers])]).astype(np.int64)
        self.recv_off = part.recv_offsets()
        self.sendbuf = None

    def start(self, Xs):
        """Pack and post the exchange (own rows of Xs already written); [[works]]."""
        torch, part = self.torch, self.part
        F = Xs.shape[1]
        if self.sendbuf is None or self.sendbuf.shape[1] != F:
            self.sendbuf = torch.empty((self.send_idx.shape[0], F), dtype=Xs.dtype, device=Xs.device)
        if self.send_idx.shape[0]:
            torch.index_select(Xs[part.own_slice], 0, self.send_idx, out=self.sendbuf)
        sends = [(self.sendbuf[self.send_off[i]:self.send_off[i + 1]], q) for i, q in enumerate(self.send_peers)]
        recvs = [(Xs[self.recv_off[q]:self.recv_off[q] + self.recv_counts[q]], q) for q in self.recv_peers]
        return [self.comm.exchange(sends, recvs)]


class DenseHalo:
    """dense halo: one all-gather per row chunk of the padded table (in place: each
    rank's block of chunk k is already written where the gather puts it)."""

    def __init__(self, part: GraphPartition, comm):
        self.part, self.comm = part, comm
        self.slices = part.gather_slices()

    def start(self, Xs):
        return [[self.comm.all_gather(Xs[t], Xs[own])] for t, own in self.slices]


class DistAggregator:
    """norm * A (norm * H) over a GraphPartition of one graph (see the module docstring).
    exact=True: one SpMM after the whole halo arrived, bit-identical to one GPU.
    exact=False: own-column edges overlap the exchange; halo chunk k's edges accumulate
    as soon as chunk k has landed.  `backend`: gala.backend.HipBackend / CpuBackend."""

    def __init__(self, part: GraphPartition, F: int, backend, comm=None, exact: bool = True):
        self.part, self.F, self.exact, self.be, self.comm = part, F, exact, backend, comm
        thr = part.split_threshold
        self.graph = backend.graph(part.graph, split=thr)
        self.groups = None if exact else [backend.graph(h, split=thr) for h in part.groups]
        self.norm = backend.degree(self.graph)          # own rows' full degrees
        self._xs = {}
        self.Xs = self._table(F)
        if part.world == 1:
            self.exchange = None
        elif part.halo_mode == "p2p":
            self.exchange = HaloExchange(part, comm, backend.device)
        else:
            self.exchange = DenseHalo(part, comm)
        self._blocks = part.own_blocks()

    def _table(self, F):
        """The feature buffer Xs of width F (one per width: a program's layers differ)."""
        if F not in self._xs:
            t = self.be.empty(self.part.n_cols, F)
            if self.part.halo_mode == "dense" and self.part.world > 1:
                t.zero_()  # padding rows are never read; keep the table finite
            self._xs[F] = t
        return self._xs[F]

    def refresh_norm(self):
        self.norm = self.be.degree(self.graph)

    def __call__(self, H, out):
        """out = norm * A (norm * H) (the GCN aggregation with the graph's own norm)."""
        return self.apply(H, out, self.norm, self.norm)

    def apply(self, H, out, pre=None, post=None, relu=False, act=None, samp=None):
        """out = post * A (pre * H) over the own rows (pre / post: [n] vectors or None), the
        generated programs' GCN_AGGREGATE (codegen/gala.cu:442-456) on a partition.  relu:
        the ReLU prologue, pre * relu(act * H) in the same pass.  samp (nsamp, ra, rb): the
        kernel-sampled aggregation (cuda.h:313-321), exact mode only -- a row's samples are
        picked by position among all its edges, which the exact layout keeps in CSR order, so
        it samples the same edges as one GPU."""
        if samp is not None and not self.exact:
            raise ValueError("DistAggregator: kernel sampling needs exact mode (one SpMM over the rows' edges)")
        be = self.be
        Xs = self._table(H.shape[1])
        sl = lambda v, a, b: None if v is None else v[a:b]  # noqa: E731
        for j0, j1, x0 in self._blocks:                               # own rows of Xs = pre * H
            if relu:
                be.row_scale_relu(sl(act, j0, j1), sl(pre, j0, j1), H[j0:j1], Xs[x0:x0 + (j1 - j0)])
            elif pre is None:
                Xs[x0:x0 + (j1 - j0)].copy_(H[j0:j1])
            else:
                be.row_broadcast(pre[j0:j1], H[j0:j1], Xs[x0:x0 + (j1 - j0)])
        chunks = self.exchange.start(Xs) if self.exchange else []
        if self.exact:
            for works in chunks:
                self.comm.wait(works)
            return be.spmm(self.graph, Xs, out, post, False, samp)
        be.spmm(self.groups[0], Xs, out, post, False)                # overlaps the exchange
        for k, works in enumerate(chunks):
            self.comm.wait(works)
            be.spmm(self.groups[1 + k], Xs, out, post, True)
        return out

    def halo_bytes(self) -> int:
        return self.part.halo_bytes(self.F) if self.part.world > 1 else 0


class HaloGat:
    """The REF GAT layer's training pair over a row partition with a halo, computed exactly as
    one GPU computes it.  Rank p gathers the feature rows its edges read (the halo: the
    all-gather table or the p2p rows of a GraphPartition), then runs the one-GPU statistics
    kernels over its own rows with the pattern's columns indexing the gathered table
    (gala_gat_{fwd,bwd}_stats_ex_f32: self_col maps each row to its own table column, the
    backward reads the rows' own dY apart from the table).  Every row keeps its CSR edge
    order and the whole graph's hub-row chunks, so Y, dX and d_aL are BIT-identical to the
    one-GPU pair.  Per layer it moves F + H floats per halo row forward (X, and the source
    logits the forward recomputed for the backward) and F backward (dY); the vertex cut
    (gala/vertex_cut.py VertexCutGat) moves 2F + 2H partial floats per row forward.

      forward_train(aL, aR, X[, wR, bR]) -> Y      (aR None: recomputed from X per head)
      backward(dY[, linear]) -> (dX, d_aL[, dwR, dbR])
    X may already be written into `own_rows(F)` (the own block of the table) to skip a copy."""

    _chunked = False      # HaloGatOverlap takes a table gathered in row chunks

    def __init__(self, part: GraphPartition, F: int, heads: int, backend, comm=None, slope: float = 0.2):
        import torch
        if part.chunks != 1 and not self._chunked:
            raise ValueError("HaloGat: one halo chunk (the kernels read the whole table)")
        self.part, self.F, self.H, self.be, self.comm, self.slope = part, F, heads, backend, comm, slope
        self.graph = backend.graph(part.graph, split=part.split_threshold)
        self.x0 = part.own_offset() if part.chunks == 1 else None
        dev = getattr(backend, "device", torch.device("cpu"))
        # the table row of every own row (one block unless the table is gathered in chunks)
        sc = np.concatenate([np.arange(x, x + j1 - j0) for j0, j1, x in part.own_blocks()] or [np.zeros(0)])
        self.self_col = torch.from_numpy(sc.astype(np.int32)).to(dev)
        if comm is None:
            self.exchange = None
        elif part.halo_mode == "p2p":
            self.exchange = HaloExchange(part, comm, backend.device)
        else:
            self.exchange = DenseHalo(part, comm)
        zero = part.halo_mode == "dense" and part.world > 1   # padding rows: keep the table finite
        self.Xs, self.dYs, self.As = (backend.empty(part.n_cols, w) for w in (F, F, heads))
        if zero:
            for t in (self.Xs, self.dYs, self.As):
                t.zero_()
        self.saved = None

    def own_rows(self, which="X"):
        """The own block of the X (or dY) table: write the layer input there to skip a copy."""
        t = self.Xs if which == "X" else self.dYs
        return t[self.x0:self.x0 + self.part.n]

    def _gather(self, table, rows):
        own = table[self.x0:self.x0 + self.part.n]
        if rows is not None and rows.data_ptr() != own.data_ptr():
            own.copy_(rows)
        return [w for works in (self.exchange.start(table) if self.exchange else []) for w in works]

    @staticmethod
    def _wait(works):
        for w in works:
            if w is not None:
                w.wait()

    def forward_train(self, aL, aR, X, wR=None, bR=None):
        n, H = self.part.n, self.H
        if self.saved is not None:   # a previous forward's logits exchange may still read As
            self._wait(self.saved[-1])
        self._wait(self._gather(self.Xs, X))
        if aR is not None:                   # a given source logit: its table too
            self._wait(self._gather(self.As, aR.reshape(n, H)))
            ar_works = []
            Y, q, Ym, sma = self.be.gat_stats_table(self.graph, aL, self.As, self.Xs, H, self.slope, self.self_col,
                                                    None)
        else:                                # recomputed in the kernel; the own logits written out
            Y, q, Ym, sma = self.be.gat_stats_table(self.graph, aL, None, self.Xs, H, self.slope, self.self_col,
                                                    self.As, wR=wR, bR=bR)
            ar_works = self._gather(self.As, None)   # the backward's logits of the halo rows
        self.saved = (aL, q, Y, Ym, sma, wR, ar_works)
        return Y

    def backward(self, dY, linear=True):
        if self.saved is None:
            raise RuntimeError("HaloGat.backward: no forward_train to take the row statistics from")
        aL, q, Y, Ym, sma, wR, ar_works = self.saved
        n, H = self.part.n, self.H
        works = self._gather(self.dYs, dY)
        self._wait(ar_works)
        self._wait(works)
        linear = linear and wR is not None
        # with the Linear: dX += d_aR wR in the kernel's store (REF: d_aR = d_aL)
        dX, d_aL = self.be.gat_bwd_stats_table(self.graph, aL, self.As, self.dYs, self.own_rows("dY"), q, Y, Ym,
                                               sma, H, self.slope, wR=wR if linear else None)
        d_aL = d_aL.view(n, H)
        if not linear:
            return dX, d_aL
        dW, db = self.be.head_linear_grads(self.own_rows("X"), d_aL, H)
        return dX, d_aL, dW, db

    def halo_bytes(self) -> int:
        """Bytes this rank receives per forward + backward (X and dY rows, the logits)."""
        return self.part.halo_bytes(2 * self.F + self.H) if self.part.world > 1 else 0


class HaloGatOverlap(HaloGat):
    """HaloGat with the halo exchange hidden behind the edges already computable.  The
    forward runs the unnormalised row statistics of the edges into the rank's own columns
    (gala_gat_fwd_partial_stats_ex_f32 over part.groups[0], which also writes the own
    vertices' logits) while the X rows are in flight, then continues every row from those
    partials over each halo chunk as it lands (gala_gat_fwd_continue_f32, in place:
    unnormalised for all but the last chunk, normalised after it; GAT REF subtracts no row
    maximum, common.h:760-773, so the sums simply continue).  With a dense table gathered in
    K row chunks (partition_graph(..., chunks=K)) the all-gathers pipeline against the
    chunks' edges.  The backward likewise: sum_e p_e dY[c] over the own columns and the
    row-local d_aL overlap the dY exchange, each halo chunk continues it, dX = q (P_own +
    P_halo).  Each row's sums are grouped per column range, so results agree with one GPU to
    fp32 rounding, not bit for bit.

    Unlike HaloGat, this backward keeps the two-pass attention-Linear backward (a separate
    gala_head_attn_bwd_f32 pass adds d_aL wR to dX after the last chunk), and its row-local
    d_aL comes from gala_gat_bwd_stats_f32 over an edgeless own-row graph, which also writes
    an [n, F] dX of zeros that is dropped: two dX-sized passes per step that HaloGat does not
    pay.  It is a layout for links slower than its own-column passes; bench.py
    times it as a candidate and at one rank it is never chosen."""
    _chunked = True

    def __init__(self, part: GraphPartition, F: int, heads: int, backend, comm=None, slope: float = 0.2):
        super().__init__(part, F, heads, backend, comm, slope)
        self.groups = [backend.graph(h, split=part.split_threshold) for h in part.groups]
        n = part.n
        self.own_graph = backend.graph(layout.HostGraph(n, n, np.zeros(n + 1, np.int32), np.zeros(0, np.int32)),
                                       split=False)
        self.Ssc = backend.empty(n, heads)
        self.blocks = part.own_blocks()

    def own_rows(self, which="X"):
        if self.part.chunks != 1:
            raise ValueError("HaloGatOverlap: the own rows are not one block of a chunked table")
        return super().own_rows(which)

    def _start(self, table, rows):
        """Own rows written into the table, the exchange started: one work list per halo chunk."""
        if rows is not None:
            for j0, j1, x in self.blocks:
                dst = table[x:x + j1 - j0]
                if dst.data_ptr() != rows[j0:j1].data_ptr():
                    dst.copy_(rows[j0:j1])
        chunks = self.exchange.start(table) if self.exchange else []
        return [chunks[k] if k < len(chunks) else [] for k in range(len(self.groups) - 1)]

    def forward_train(self, aL, aR, X, wR=None, bR=None):
        n, H, F, be = self.part.n, self.H, self.F, self.be
        if self.saved is not None:
            self._wait(self.saved[-1])
        chunks = self._start(self.Xs, X)
        if aR is not None:                   # given source logits: their (small) table first
            for works in self._start(self.As, aR.reshape(n, H)):
                self._wait(works)
            kw = {}
        else:
            kw = {"wR": wR, "bR": bR}
        At = self.As if aR is not None else None
        Y, Ym, q, sma = be.empty(n, F), be.empty(n, F), be.empty(n, H), be.empty(n, H)
        be.gat_partial_stats(self.groups[0], aL, At, self.Xs, H, self.slope, Y, q, Ym, sma,
                             self_col=None if aR is not None else self.self_col,
                             aR_out=None if aR is not None else self.As, **kw)
        last = len(chunks) - 1
        for k, works in enumerate(chunks):
            self._wait(works)
            be.gat_continue(self.groups[1 + k], aL, At, self.Xs, H, self.slope, Y, q, Ym, sma, partial=k < last,
                            **kw)
        ar_works = [w for works in self._start(self.As, None) for w in works] if aR is None else []
        self.saved = (aL, q, Y, Ym, sma, wR, X, ar_works)
        return Y

    def backward(self, dY, linear=True):
        if self.saved is None:
            raise RuntimeError("HaloGatOverlap.backward: no forward_train to take the row statistics from")
        aL, q, Y, Ym, sma, wR, X, ar_works = self.saved
        n, H, be = self.part.n, self.H, self.be
        chunks = self._start(self.dYs, dY)
        # the own columns' logits were written by this rank's forward; the halo's may still be in flight
        dX = be.empty(n, self.F)
        be.gat_partial(self.groups[0], aL, self.As, self.dYs, H, self.slope, dX, self.Ssc)
        _, d_aL = be.gat_bwd_stats(self.own_graph, aL, self.As, dY, q, Y, Ym, sma, H, self.slope)
        self._wait(ar_works)
        last = len(chunks) - 1
        for k, works in enumerate(chunks):
            self._wait(works)
            be.gat_continue(self.groups[1 + k], aL, self.As, self.dYs, H, self.slope, dX, self.Ssc,
                            partial=k < last)
        d_aL = d_aL.view(n, H)
        if not (linear and wR is not None):
            return dX, d_aL
        dW, db = be.head_linear_grads(X, d_aL, H)
        be.head_attn_bwd(d_aL, wR, H, dX)
        return dX, d_aL, dW, db
