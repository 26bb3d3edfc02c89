"""Vertex-cut aggregation: column ownership + RCCL reduce-scatter of partial rows.

SURVEY §8(e) / BASELINE north_star ("vertex-cut graph partitioning across the GPUs of one
node with RCCL all-reduce of halo feature rows").  The reference's own column-tiled layout
is the anchor: ord_col_tiling_torch (src/ops/tiling.h:222-283) cuts A by column ranges
into segments with relative row offsets, and the DCSR variant ord_col_tiling_torch_dcsr
(tiling.h:285-387) keeps only the rows with edges in a segment.  Here one segment is one
rank:

* rank p owns the vertex range V_p = [bounds[p], bounds[p+1)) -- the feature rows X[V_p]
  (so no input halo at all) and every edge whose SOURCE (column) lies in V_p;
* it computes partial sums  Y_p = A[:, V_p] (norm * H)[V_p]  for every row;
* one reduce-scatter sums the partials into each row's owner: rank p receives
  sum_q Y_q[V_p], which is exactly the next layer's input rows -- the layout is closed
  under aggregation, nothing else moves.

Partial rows are laid out in K row chunks so the reduce-scatter of chunk k overlaps the
SpMM of chunk k+1: chunk k holds, for every owner q, the c = ceil(max|V_q| / K) rows
j in [k*c, (k+1)*c) of V_q (padded), owner-major -- exactly the block layout
reduce_scatter_tensor expects.  Every chunk is an ordinary CSR (rows in global order,
columns local to V_p), so the SpMM kernel is the one-GPU kernel.

The sparse exchange (exchange="sparse", the DCSR variant): a rank computes partial rows
only for the destination rows it holds edges of (plus its own rows), sends each owner its
block with one uneven all_to_all_single per chunk, and the owner sums what it receives
with an SpMM over a receive CSR (each row's partials in source-rank order).  "auto" picks
it when the graph's touched fraction is low (banded / skewed graphs); a uniform graph
touches every (row, rank) pair and keeps the dense reduce-scatter.

Numerics: a row's sum is split into per-rank partial sums (each in CSR order) added by
RCCL (or by the receive SpMM), so results agree with the one-GPU aggregation to fp32
rounding, not bit for bit (the row-partition `exact` mode in gala/dist.py is the bit-exact
one).

Degrees need no collective: the owned rows' full CSR (a slice of the whole graph) is
partition metadata.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import layout
from .dist import row_bounds


@dataclass
class SparseExchange:
    """DCSR partial rows + the sparse exchange of one rank (the ord_col_tiling_torch_dcsr
    idea, src/ops/tiling.h:285-387: a column segment keeps only the rows it has edges in).

    send_graphs[k]  compact CSR of chunk k: only the destination rows this rank holds an
                    edge of, owner-major and ascending (the order all_to_all_single sends
                    them in), columns local to V_p
    send_counts     int64 [K, P] rows sent to each owner per chunk
    recv_counts     int64 [K, P] rows received from each source rank per chunk
    recv_graph      CSR [n own rows, sum(recv_counts)]: row r lists the received partial rows
                    of r in source-rank order, so an unweighted SpMM over it sums them in a
                    fixed order (deterministic; the post scale fuses in as its dst scale)."""
    send_graphs: list
    send_counts: np.ndarray
    recv_counts: np.ndarray
    recv_graph: layout.HostGraph
    send_dense_rows: list       # per chunk: int64 row of every compact row in the dense layout
    send_self_cols: list        # per chunk: int32 own-vertex column of every compact row (-1: none)


@dataclass
class VertexCutPartition:
    rank: int
    world: int
    bounds: np.ndarray          # int64 [world+1] vertex ranges (rows owned = columns held)
    chunks: int                 # K
    block: int                  # c: rows per (owner, chunk)
    chunk_graphs: list = field(default_factory=list)  # dense: K x CSR [world*c rows, n local cols]
    deg_graph: layout.HostGraph | None = None          # the own rows' full CSR (degree pass)
    split_threshold: int = 0
    nnz: int = 0                # edges held by this rank
    exchange: str = "dense"     # "dense" (reduce-scatter) | "sparse" (DCSR rows, all-to-all)
    sparse: SparseExchange | None = None
    touched_frac: float = 1.0   # remote (row, source rank) pairs / (N * (P-1)), whole graph

    @property
    def n(self) -> int:
        return int(self.bounds[self.rank + 1] - self.bounds[self.rank])

    @property
    def r0(self) -> int:
        return int(self.bounds[self.rank])

    def partial_rows(self) -> int:
        if self.exchange == "sparse":
            return int(self.sparse.send_counts.sum())
        return self.chunks * self.world * self.block

    def comm_bytes(self, F: int) -> int:
        """Bytes this rank sends per aggregation (dense: the reduce-scatter's share; sparse:
        the partial rows for the other owners)."""
        if self.exchange == "sparse":
            sc = self.sparse.send_counts.copy()
            sc[:, self.rank] = 0
            return 4 * F * int(sc.sum())
        return 4 * F * self.chunks * self.block * (self.world - 1)

    def self_cols(self, k: int) -> np.ndarray:
        """int32 [rows of chunk k]: the local column of each partial row's own vertex, -1
        for rows of other owners (the own-vertex map of gala_gat_fwd_partial_stats_ex_f32)."""
        if self.exchange == "sparse":
            return self.sparse.send_self_cols[k]
        P, c, p = self.world, self.block, self.rank
        out = np.full(P * c, -1, np.int32)
        j = np.arange(k * c, min((k + 1) * c, self.n), dtype=np.int32)
        out[p * c + (j - k * c)] = j
        return out

    def chunk_nnz(self) -> int:
        gs = self.sparse.send_graphs if self.exchange == "sparse" else self.chunk_graphs
        return sum(h.nnz for h in gs)


def touched_fraction(g: layout.HostGraph, bounds: np.ndarray) -> float:
    """Remote (destination row, source rank) pairs of the whole graph over N * (P-1): the
    share of the dense reduce-scatter's rows that carry a partial sum.  Every rank computes
    the same number from the same graph, so the exchange choice agrees across ranks."""
    P = bounds.shape[0] - 1
    N = g.n_rows
    if P == 1 or g.nnz == 0:
        return 0.0
    rp = g.rowptr.astype(np.int64)
    if P > 64:   # distinct (row, owner) pairs by sorting
        rows = np.repeat(np.arange(N, dtype=np.int64), np.diff(rp))
        ow = np.searchsorted(bounds, g.col, side="right") - 1
        far = ow != np.searchsorted(bounds, rows, side="right") - 1
        return np.unique(rows[far] * P + ow[far]).shape[0] / float(N * (P - 1))
    # distinct remote (row, owner) pairs, whatever the column order inside a row: an owner
    # bit mask per row (OR over the row's edges), the row's own owner cleared, popcount
    bit = np.left_shift(np.uint64(1), (np.searchsorted(bounds, g.col, side="right") - 1).astype(np.uint64))
    full = np.flatnonzero(np.diff(rp) > 0)
    mask = np.bitwise_or.reduceat(bit, rp[full]) if full.size else np.zeros(0, np.uint64)
    own = np.left_shift(np.uint64(1), (np.searchsorted(bounds, full, side="right") - 1).astype(np.uint64))
    remote = int(np.bitwise_count(mask & ~own).sum())
    return remote / float(N * (P - 1))


def vertex_cut_partition(g: layout.HostGraph, rank: int, world: int, chunks: int = 1,
                         bounds: np.ndarray | None = None, exchange: str = "dense",
                         sparse_frac: float = 0.5) -> VertexCutPartition:
    """Rank `rank`'s column share of the square one-segment graph `g`.  The vertex ranges
    balance stored edges + rows like row_bounds (for a symmetric graph the column counts
    equal the row counts).  exchange "dense": partial rows for every destination, summed by
    reduce-scatter; "sparse": only the rows the rank holds edges of (DCSR), sent with
    all_to_all_single and summed by the owner in rank order; "auto": sparse when the graph's
    touched fraction (touched_fraction) is below sparse_frac."""
    if g.n_rows != g.n_cols or g.n_seg != 1:
        raise ValueError("vertex_cut_partition needs a square, one-segment CSR")
    N, P = g.n_rows, world
    b = row_bounds(g.rowptr, world) if bounds is None else np.asarray(bounds, np.int64)
    c0, c1 = int(b[rank]), int(b[rank + 1])
    K = max(int(chunks), 1)
    m = int(np.diff(b).max(initial=0))
    c = max((m + K - 1) // K, 1)
    rp = g.rowptr.astype(np.int64)
    deg = np.diff(rp)
    frac = touched_fraction(g, b) if (exchange == "auto" or exchange == "sparse") else 1.0
    if exchange == "auto":
        exchange = "sparse" if (P > 1 and frac < sparse_frac) else "dense"
    if exchange not in ("dense", "sparse"):
        raise ValueError(f"vertex_cut_partition: exchange {exchange!r} (dense | sparse | auto)")
    sel = (g.col >= c0) & (g.col < c1)
    cs = np.zeros(g.nnz + 1, np.int64)
    np.cumsum(sel, out=cs[1:])
    cnt = cs[rp[1:]] - cs[rp[:-1]]                       # held edges per row
    # chunk index and chunk-local row of every global row
    rk = np.empty(N, np.int64)
    pos = np.empty(N, np.int64)
    for q in range(P):
        j = np.arange(int(b[q + 1] - b[q]), dtype=np.int64)
        rk[int(b[q]):int(b[q + 1])] = j // c
        pos[int(b[q]):int(b[q + 1])] = q * c + j % c
    edge_k = np.repeat(rk.astype(np.int32), deg) if K > 1 else None
    graphs, sparse = [], None
    if exchange == "dense":
        for k in range(K):
            rows_k = rk == k
            counts = np.zeros(P * c, np.int64)
            counts[pos[rows_k]] = cnt[rows_k]
            rowptr = np.zeros(P * c + 1, np.int64)
            np.cumsum(counts, out=rowptr[1:])
            keep = sel if K == 1 else (sel & (edge_k == k))
            cols = (g.col[keep] - c0).astype(np.int32)
            graphs.append(layout.HostGraph(P * c, c1 - c0, rowptr.astype(np.int32), cols))
    else:
        sparse = _sparse_exchange(g, b, rank, K, c, sel, cnt, rk, pos, edge_k)
    drp = (rp[c0:c1 + 1] - rp[c0]).astype(np.int32)
    dg = layout.HostGraph(c1 - c0, N, drp, g.col[int(rp[c0]):int(rp[c1])])
    return VertexCutPartition(rank, world, b, K, c, graphs, dg, layout.split_threshold(g.n_rows, g.nnz),
                              int(cs[-1]), exchange, sparse, frac)


def _sparse_exchange(g, b, rank, K, c, sel, cnt, rk, pos, edge_k) -> SparseExchange:
    P = b.shape[0] - 1
    c0, c1 = int(b[rank]), int(b[rank + 1])
    owner_of = lambda r: np.searchsorted(b, r, side="right") - 1  # noqa: E731
    # the rows a rank holds edges of, and always its own rows: each own vertex then has a
    # compact row for its own source logit (VertexCutGat's aR_out), at the cost of a local copy
    touched = cnt > 0
    touched[c0:c1] = True
    send_graphs, dense_rows, self_rows = [], [], []
    send_counts = np.zeros((K, P), np.int64)
    for k in range(K):
        rows = np.flatnonzero(touched & (rk == k))              # owner-major, ascending
        send_counts[k] = np.bincount(owner_of(rows), minlength=P)[:P]
        self_rows.append(np.where((rows >= c0) & (rows < c1), rows - c0, -1).astype(np.int32))
        rowptr = np.zeros(rows.shape[0] + 1, np.int64)
        np.cumsum(cnt[rows], out=rowptr[1:])
        keep = sel if K == 1 else (sel & (edge_k == k))
        cols = (g.col[keep] - c0).astype(np.int32)
        assert cols.shape[0] == rowptr[-1]
        send_graphs.append(layout.HostGraph(rows.shape[0], c1 - c0, rowptr.astype(np.int32), cols))
        dense_rows.append(k * P * c + pos[rows])
    # receive side: which source ranks hold edges of each own row (its columns' owners)
    n = c1 - c0
    e0, e1 = int(g.rowptr[c0]), int(g.rowptr[c1])
    lrow = np.repeat(np.arange(n, dtype=np.int64), np.diff(g.rowptr[c0:c1 + 1].astype(np.int64)))
    T = np.zeros((n, P), bool)
    T[lrow, owner_of(g.col[e0:e1])] = True
    T[:, rank] = True                                           # the own rows always come back
    recv_counts = np.zeros((K, P), np.int64)
    cols = []
    base = 0
    for k in range(K):
        Tk = T[k * c:(k + 1) * c]
        recv_counts[k] = Tk.sum(0)
        qoff = np.concatenate([[0], np.cumsum(recv_counts[k])[:-1]])
        idx = base + qoff[None, :] + np.cumsum(Tk, 0) - 1
        cols.append(idx[Tk])                                   # row-major: row, then source rank
        base += int(recv_counts[k].sum())
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(T.sum(1), out=rowptr[1:])
    col = np.concatenate(cols).astype(np.int32) if cols else np.zeros(0, np.int32)
    recv = layout.HostGraph(n, max(base, 1), rowptr.astype(np.int32), col)
    return SparseExchange(send_graphs, send_counts, recv_counts, recv, dense_rows, self_rows)


class _PartialRows:
    """The partial-row plumbing both vertex-cut operators share.  Per chunk k: the rows this
    rank computes (its send rows), their collective, and where the summed rows land:
      dense   send [K*P*c, W] (every destination row), recv [K*c, W] by reduce-scatter; the
              own rows are recv[:n]
      sparse  send [sum send_counts, W] (DCSR: rows with a held edge), recv [sum recv_counts,
              W] by all_to_all_single; the own rows are an SpMM over the receive CSR (each
              row's partials summed in source-rank order; a post scale fuses in)."""

    def __init__(self, part: VertexCutPartition, backend, comm=None):
        self.part, self.be, self.comm = part, backend, comm
        thr = part.split_threshold
        self.sparse = part.exchange == "sparse"
        P, c, K = part.world, part.block, part.chunks
        if self.sparse:
            sp = part.sparse
            self.graphs = [backend.graph(h, split=thr) for h in sp.send_graphs]
            self.recv_graph = backend.graph(sp.recv_graph, split=False)
            so = np.concatenate([[0], np.cumsum(sp.send_counts.sum(1))]).astype(np.int64)
            ro = np.concatenate([[0], np.cumsum(sp.recv_counts.sum(1))]).astype(np.int64)
            self._send = [(int(so[k]), int(so[k + 1])) for k in range(K)]
            self._recv = [(int(ro[k]), int(ro[k + 1])) for k in range(K)]
            self._ss = [sp.send_counts[k].tolist() for k in range(K)]
            self._rs = [sp.recv_counts[k].tolist() for k in range(K)]
            self.n_send, self.n_recv = max(int(so[-1]), 1), max(int(ro[-1]), 1)
            if comm is not None:  # every rank agrees that no block passes the cut's bound
                biggest = max([int(v) for k in range(K) for v in self._ss[k] + self._rs[k]] + [0])
                comm.check_block_bound(biggest, c)
        else:
            self.graphs = [backend.graph(h, split=thr) for h in part.chunk_graphs]
            self._send = [(k * P * c, (k + 1) * P * c) for k in range(K)]
            self._recv = [(k * c, (k + 1) * c) for k in range(K)]
            self._ss = self._rs = [None] * K
            self.n_send, self.n_recv = K * P * c, K * c

    def alloc(self, W):
        """(send, recv) buffers of W columns."""
        return self.be.empty(self.n_send, W), self.be.empty(self.n_recv, W)

    def send_rows(self, buf, k):
        a, b = self._send[k]
        return buf[a:b]

    def post(self, send, recv, k):
        """Chunk k's collective (async on RCCL; None when done in place)."""
        a, b = self._send[k]
        c, d = self._recv[k]
        if self.comm is None:       # one rank without collectives
            recv[c:d].copy_(send[a:b])
            return None
        if self.sparse:   # every (chunk, owner) block has at most `block` rows, on every rank
            return self.comm.all_to_all(recv[c:d], send[a:b], self._rs[k], self._ss[k], max_rows=self.part.block)
        return self.comm.reduce_scatter(recv[c:d], send[a:b])

    @staticmethod
    def wait(works):
        for w in works:
            if w is not None:
                w.wait()

    def own_rows(self, recv, out, post=None, view_ok=False):
        """out [n, W] = post * (the summed partial rows of the own vertices).  view_ok: the
        dense exchange without a post scale may hand back recv[:n] itself (the own rows are
        its first n rows), saving a copy; the caller then reads it before the next exchange."""
        n = self.part.n
        if self.sparse:
            return self.be.spmm(self.recv_graph, recv, out, post, False)
        if post is None:
            return recv[:n] if view_ok else out.copy_(recv[:n])
        return self.be.row_broadcast(post, recv[:n], out)


class VertexCutAggregator(_PartialRows):
    """norm * A (norm * H) with column ownership (see the module docstring):
        Xs        = norm[V_p] * H                            (ROW_BROADCAST)
        Y_p^k     = A_k[:, V_p] Xs          k = 0..K-1      (SpMM, chunk k's rows)
      dense exchange:
        S[k-th c] = reduce_scatter(Y^k)     overlapped with the next chunk's SpMM
        out       = norm[V_p] * S[:n]                        (ROW_BROADCAST)
      sparse exchange (DCSR: Y^k holds only the rows this rank has edges of):
        R^k       = all_to_all(Y^k)         overlapped with the next chunk's SpMM
        out       = norm[V_p] * (R_graph R) (SpMM over the receive CSR: the partials of a
                                             row summed in source-rank order, norm fused)
    `backend`: gala.backend.HipBackend / CpuBackend; `comm`: gala.comm.Comm."""

    def __init__(self, part: VertexCutPartition, F: int, backend, comm=None):
        super().__init__(part, backend, comm)
        self.F = F
        self.deg_graph = backend.graph(part.deg_graph, split=False)
        self.norm = backend.degree(self.deg_graph)
        self._bufs = {}
        self.Xs, self.partial, self.S = self._buffers(F)

    def _buffers(self, F):
        """(Xs [n, F], send rows, received / owner rows) of width F (a program's layers
        differ in width)."""
        if F not in self._bufs:
            self._bufs[F] = (self.be.empty(self.part.n, F),) + self.alloc(F)
        return self._bufs[F]

    def refresh_norm(self):
        self.norm = self.be.degree(self.deg_graph)

    def __call__(self, H, out):
        """out = norm * A (norm * H) with the graph's own norm (the GCN aggregation)."""
        return self.apply(H, out, self.norm, self.norm)

    def local_spmm(self, F=None):
        """The partial-row SpMMs alone (bench: the rank's kernel time)."""
        Xs, partial, _ = self._buffers(F or self.F)
        for k, gk in enumerate(self.graphs):
            self.be.spmm(gk, Xs, self.send_rows(partial, k), None, False)

    def exchange_only(self, F=None):
        """The collectives of one aggregation alone (bench: the exchange time)."""
        _, partial, S = self._buffers(F or self.F)
        self.wait([self.post(partial, S, k) for k in range(len(self.graphs))])

    def apply(self, H, out, pre=None, post=None, relu=False, act=None, samp=None):
        """out = post * A (pre * H) over the own rows (pre / post: [n] vectors or None): the
        generated programs' GCN_AGGREGATE (codegen/gala.cu:442-456) with column ownership.
        relu: the ReLU prologue, out = post * A (pre * relu(act * H)) (one elementwise pass).
        Kernel sampling is refused: a row's samples are picked by position among ALL its
        edges (cuda.h:313-321), which the cut splits by owner."""
        if samp is not None:
            raise NotImplementedError("VertexCutAggregator: kernel sampling (use the row partition)")
        be = self.be
        Xs, partial, S = self._buffers(H.shape[1])
        if relu:
            be.row_scale_relu(act, pre, H, Xs)
        elif pre is None:
            Xs.copy_(H)
        else:
            be.row_broadcast(pre, H, Xs)
        works = []
        for k, gk in enumerate(self.graphs):
            be.spmm(gk, Xs, self.send_rows(partial, k), None, False)
            works.append(self.post(partial, S, k))
        self.wait(works)
        return self.own_rows(S, out, post)

    def halo_bytes(self) -> int:
        return self.part.comm_bytes(self.F) if self.part.world > 1 else 0


class VertexCutGat(_PartialRows):
    """The REF-mode GAT layer (edge softmax + attention-weighted aggregation) with column
    ownership.  The softmax of a row spans every column range, so each rank computes for its
    edges the UNNORMALISED partial rows and softmax sums (GALA_GAT_PARTIAL):
        U_p[r] = sum_{e in row r, col in V_p} p_e X[col],   S_p[r, h] = sum p_e,
        p_e = min(exp(LeakyReLU(aL[r] + aR[col])), 1e12)           (common.h:760-773)
    and the exchange (dense reduce-scatter, or the sparse DCSR all-to-all) hands each owner
    Y[r] = (sum_p U_p[r]) / (1e-12 + sum_p S_p[r])  -- REF has no max subtraction, so
    partial sums simply add.  aL of every destination row arrives by all-gathers of the
    owners' [n, H] blocks, one per chunk, all posted up front (each chunk's kernel waits for
    its own); aR and X of the own columns are local.

    Training (`forward_train` + `backward`, the REF layer of the generated programs with the
    row statistics of gala_gat_{fwd,bwd}_stats_f32):
      forward   gala_gat_fwd_partial_stats_f32 adds  Um_p[r] = sum m_e p_e X[col] and
                M_p[r, h] = sum m_e p_e (m_e the LeakyReLU factor) to U_p and S_p; the packed
                [U | Um] rows and the two [rows, H] sums are exchanged, and the owner forms
                q = 1/(S + 1e-12), Y = q U, Ym = q Um, sma = q M.
      backward  the REF dX[r] = sum_e alpha_e dY[col_e] (A, not A^T: common.h:835-894) only
                reads dY of the columns a rank holds -- its own rows -- so each rank runs the
                same partial forward kernel with dY in place of X (P_p[r] = sum p_e dY[col])
                and the exchange hands the owner dX = q P.  d_aL of a row needs no edge:
                <dY, Ym> - (<dY, Y> + 1e-12) sma (+1e-12) per head, from the owner's rows
                (gala_gat_bwd_stats_f32 on the owner's rows without edges).
                With the source logits recomputed (aR = the per-head Linear wR, bR of X), the
                REF d_aR equals d_aL (common.h:622-675), so the owner also adds
                dX[:, head h] += d_aL[:, h] wR_h and returns the Linear's gradients over its
                rows (dwR, dbR; the caller all-reduces them), as GatAggregateFfn does on one GPU
                (host/gala_torch.cpp).
    No dY or X row crosses the links; per layer the collectives move (2F + 2H) floats per
    (sent) row forward and F backward.  Results agree with one GPU to fp32 rounding (each
    row's sums are regrouped by column range, and dX is q * sum p dY instead of sum fl(p q) dY)."""

    def __init__(self, part: VertexCutPartition, F: int, heads: int, backend, comm=None, slope: float = 0.2):
        super().__init__(part, backend, comm)
        self.F, self.H, self.slope = F, heads, slope
        P, c, K = part.world, part.block, part.chunks
        self.aLpad = backend.empty(K * c, heads)
        self.aLall = backend.empty(K * P * c, heads)
        import torch
        dev = getattr(backend, "device", torch.device("cpu"))
        if self.sparse:
            self._al_idx = [torch.from_numpy(np.ascontiguousarray(r, np.int64)).to(dev)
                            for r in part.sparse.send_dense_rows]
            self.aLsend = backend.empty(self.n_send, heads)
        # each own vertex's row in some chunk: the partial forward writes its source logit
        self._self_col = [torch.from_numpy(np.ascontiguousarray(part.self_cols(k))).to(dev) for k in range(K)]
        self._fw = None      # eval-forward buffers
        self._train = None   # forward_train / backward buffers, allocated on first use
        self.saved = None

    # -- aL of the destination rows ------------------------------------------------------
    def _post_aL(self, aL):
        """Copy the own aL into the padded block and post every chunk's all-gather."""
        p, H, c, K = self.part, self.H, self.part.block, self.part.chunks
        n = p.n
        self.aLpad[:n].copy_(aL.reshape(n, H))
        self.aLpad[n:].zero_()
        rows = p.world * c
        works = []
        for k in range(K):
            al_k = self.aLall[k * rows:(k + 1) * rows]
            if self.comm is not None:
                works.append(self.comm.all_gather(al_k, self.aLpad[k * c:(k + 1) * c]))
            else:
                al_k.copy_(self.aLpad[k * c:(k + 1) * c])
                works.append(None)
        return works

    def _chunk_aL(self, k, works):
        """aL of chunk k's send rows (after its all-gather landed)."""
        if works[k] is not None:
            works[k].wait()
        rows = self.part.world * self.part.block
        al = self.aLall[k * rows:(k + 1) * rows]
        if not self.sparse:
            return al
        import torch
        out = self.send_rows(self.aLsend, k)
        return torch.index_select(self.aLall, 0, self._al_idx[k], out=out)

    def _owner_scale(self, q, T):
        """q [n, H] times the [n, F] rows T per head (the owner's normalisation)."""
        n, H = q.shape
        return (T.reshape(n, H, self.F // H) * q.view(n, H, 1)).reshape(n, self.F)

    # -- eval forward ----------------------------------------------------------------------
    def __call__(self, aL, aR, X):
        """aL [n, H] (own rows), aR [n, H] and X [n, F] (own columns) -> Y [n, F] (own rows)."""
        p, H, F, n = self.part, self.H, self.F, self.part.n
        if self._fw is None:
            U, Ur = self.alloc(F)
            S, Sr = self.alloc(H)
            self._fw = (U, Ur, S, Sr, self.be.empty(n, F), self.be.empty(n, H))
        U, Ur, S, Sr, Uo, So = self._fw
        al_works = self._post_aL(aL)
        works = []
        for k, gk in enumerate(self.graphs):
            self.be.gat_partial(gk, self._chunk_aL(k, al_works), aR, X, H, self.slope, self.send_rows(U, k),
                                self.send_rows(S, k))
            works += [self.post(U, Ur, k), self.post(S, Sr, k)]
        self.wait(works)
        Uo = self.own_rows(Ur, Uo, view_ok=True)
        So = self.own_rows(Sr, So, view_ok=True)
        return self._owner_scale(1.0 / (So + 1e-12), Uo)

    # -- training pair -----------------------------------------------------------------------
    def _train_buffers(self):
        if self._train is None:
            be, p, H, F = self.be, self.part, self.H, self.F
            own = layout.HostGraph(p.n, p.n, np.zeros(p.n + 1, np.int32), np.zeros(0, np.int32))
            b = {"own": be.graph(own, split=False)}
            b["UU"], b["UUr"] = self.alloc(2 * F)
            b["S"], b["Sr"] = self.alloc(H)
            b["M"], b["Mr"] = self.alloc(H)
            b["P"], b["Pr"] = self.alloc(F)
            b["Ssc"] = be.empty(self.n_send, H)
            b["UUo"], b["So"], b["Mo"], b["Po"] = be.empty(p.n, 2 * F), be.empty(p.n, H), be.empty(p.n, H), \
                be.empty(p.n, F)
            self._train = b
        return self._train

    def forward_train(self, aL, aR, X, wR=None, bR=None):
        """aL [n, H] (own rows), aR [n, H], X [n, F] (own columns) -> Y [n, F]; keeps the
        row statistics (q, Y, Ym, sma of the own rows) for `backward`.  aR None: the source
        logits are the per-head Linear (wR [F], bR [H]) of X, recomputed inside the kernel
        from the gathered rows (the DSL's attnR = ffn(res, out=1)); the same kernels also
        write the own vertices' logits (each from its self-loop edge, gala_gat_fwd_partial_
        stats_ex_f32), which the backward's alpha reuses bit for bit."""
        H, F, n, b = self.H, self.F, self.part.n, self._train_buffers()
        al_works = self._post_aL(aL)
        works = []
        aR_own = self.be.empty(n, H) if aR is None else None
        for k, gk in enumerate(self.graphs):
            UUk = self.send_rows(b["UU"], k)
            self.be.gat_partial_stats(gk, self._chunk_aL(k, al_works), aR, X, H, self.slope, UUk[:, :F],
                                      self.send_rows(b["S"], k), UUk[:, F:], self.send_rows(b["M"], k),
                                      wR=wR, bR=bR, self_col=self._self_col[k] if aR is None else None,
                                      aR_out=aR_own)
            works += [self.post(b["UU"], b["UUr"], k), self.post(b["S"], b["Sr"], k), self.post(b["M"], b["Mr"], k)]
        if aR is None:   # the backward's source logits of the own columns: the forward's own
            aR = aR_own
        self.wait(works)
        UUo, So, Mo = (self.own_rows(b[r], b[o], view_ok=True) for r, o in (("UUr", "UUo"), ("Sr", "So"), ("Mr", "Mo")))
        q = 1.0 / (So + 1e-12)
        Y = self._owner_scale(q, UUo[:, :F])
        Ym = self._owner_scale(q, UUo[:, F:])
        sma = Mo * q
        # the destination logits the backward's alpha needs are snapshotted with the
        # statistics (an eval forward in between re-gathers self.aLall)
        al_snap = self.aLall.clone() if not self.sparse else self.aLsend.clone()
        self.saved = (aL.reshape(n, H), aR, q, Y, Ym, sma, al_snap, X, wR)
        return Y

    def _saved_chunk_aL(self, k, al_snap):
        if self.sparse:
            return self.send_rows(al_snap, k)
        rows = self.part.world * self.part.block
        return al_snap[k * rows:(k + 1) * rows]

    def backward(self, dY, linear=True):
        """dY [n, F] of the own rows -> (dX [n, F], d_aL [n, H]) of the REF layer; with the
        source logits recomputed (forward_train's wR given) and `linear` -> (dX, d_aL, dwR,
        dbR), dX then including the path through aR = X wR + bR, dwR / dbR this rank's rows'
        share (linear=False: the aggregation's own backward only, as gala_gat_bwd_stats_f32)."""
        if self.saved is None:
            raise RuntimeError("VertexCutGat.backward: no forward_train to take the row statistics from")
        H, n, b = self.H, self.part.n, self._train_buffers()
        aL, aR, q, Y, Ym, sma, al_snap, X, wR = self.saved
        works = []
        for k, gk in enumerate(self.graphs):
            self.be.gat_partial(gk, self._saved_chunk_aL(k, al_snap), aR, dY, H, self.slope,
                                self.send_rows(b["P"], k), self.send_rows(b["Ssc"], k))
            works.append(self.post(b["P"], b["Pr"], k))
        # the row-local d_aL needs no edge and overlaps the exchange
        _, d_aL = self.be.gat_bwd_stats(b["own"], aL, aR, dY, q, Y, Ym, sma, H, self.slope)
        d_aL = d_aL.view(n, H)
        grads = None
        linear = linear and wR is not None
        if linear:   # REF: d_aR = d_aL; through aR = X wR + bR (per head)
            grads = self.be.head_linear_grads(X, d_aL, H)
        self.wait(works)
        dX = self._owner_scale(q, self.own_rows(b["Pr"], b["Po"], view_ok=True))
        if not linear:
            return dX, d_aL
        self.be.head_attn_bwd(d_aL, wR, H, dX)
        return (dX, d_aL) + tuple(grads)
