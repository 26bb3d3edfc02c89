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

Numerics: a row's sum is split into per-rank partial sums (each in CSR order) added by
RCCL, so results agree with the one-GPU aggregation to fp32 rounding, not bit for bit
(the row-partition `exact` mode in gala/dist.py is the bit-exact one).

Degrees need no collective: the row structure of the owned rows (their rowptr slice) is
partition metadata, and gala_degree_f32 only reads row offsets.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import layout
from .dist import row_bounds


@dataclass
class VertexCutPartition:
    rank: int
    world: int
    bounds: np.ndarray          # int64 [world+1] vertex ranges (rows owned = columns held)
    chunks: int                 # K
    block: int                  # c: rows per (owner, chunk)
    chunk_graphs: list = field(default_factory=list)  # K x CSR [world*c rows, n local cols]
    deg_graph: layout.HostGraph | None = None          # own rows' offsets (degree pass only)
    split_threshold: int = 0
    nnz: int = 0                # edges held by this rank

    @property
    def n(self) -> int:
        return int(self.bounds[self.rank + 1] - self.bounds[self.rank])

    @property
    def r0(self) -> int:
        return int(self.bounds[self.rank])

    def partial_rows(self) -> int:
        return self.chunks * self.world * self.block

    def comm_bytes(self, F: int) -> int:
        """Bytes this rank sends (= receives) per aggregation in the reduce-scatter."""
        return 4 * F * self.chunks * self.block * (self.world - 1)


def vertex_cut_partition(g: layout.HostGraph, rank: int, world: int, chunks: int = 1,
                         bounds: np.ndarray | None = None) -> VertexCutPartition:
    """Rank `rank`'s column share of the square one-segment graph `g`.  The vertex ranges
    balance stored edges + rows like row_bounds (for a symmetric graph the column counts
    equal the row counts)."""
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
    graphs = []
    for k in range(K):
        rows_k = rk == k
        counts = np.zeros(P * c, np.int64)
        counts[pos[rows_k]] = cnt[rows_k]
        rowptr = np.zeros(P * c + 1, np.int64)
        np.cumsum(counts, out=rowptr[1:])
        keep = sel if K == 1 else (sel & (edge_k == k))
        cols = (g.col[keep] - c0).astype(np.int32)
        graphs.append(layout.HostGraph(P * c, c1 - c0, rowptr.astype(np.int32), cols))
    drp = (rp[c0:c1 + 1] - rp[c0]).astype(np.int32)
    dg = layout.HostGraph(c1 - c0, N, drp, np.zeros(0, np.int32))
    return VertexCutPartition(rank, world, b, K, c, graphs, dg, layout.split_threshold(g.n_rows, g.nnz),
                              int(cs[-1]))


class VertexCutAggregator:
    """norm * A (norm * H) with column ownership (see the module docstring):
        Xs        = norm[V_p] * H                            (ROW_BROADCAST)
        Y_p^k     = A_k[:, V_p] Xs          k = 0..K-1      (SpMM, chunk k's rows)
        S[k-th c] = reduce_scatter(Y^k)     overlapped with the next chunk's SpMM
        out       = norm[V_p] * S[:n]                        (ROW_BROADCAST)
    `backend`: gala.backend.HipBackend / CpuBackend; `comm`: gala.comm.Comm."""

    def __init__(self, part: VertexCutPartition, F: int, backend, comm=None):
        self.part, self.F, self.be, self.comm = part, F, backend, comm
        thr = part.split_threshold
        self.graphs = [backend.graph(h, split=thr) for h in part.chunk_graphs]
        self.deg_graph = backend.graph(part.deg_graph, split=False)
        self.norm = backend.degree(self.deg_graph)
        self._rows = part.world * part.block
        self._bufs = {}
        self.Xs, self.partial, self.S = self._buffers(F)

    def _buffers(self, F):
        """(Xs [n, F], partial rows [K*P*c, F], owner rows [K*c, F]) of width F (a program's
        layers differ in width)."""
        if F not in self._bufs:
            p, be = self.part, self.be
            self._bufs[F] = (be.empty(p.n, F), be.empty(p.chunks * self._rows, F), be.empty(p.chunks * p.block, F))
        return self._bufs[F]

    def refresh_norm(self):
        self.norm = self.be.degree(self.deg_graph)

    def __call__(self, H, out):
        """out = norm * A (norm * H) with the graph's own norm (the GCN aggregation)."""
        return self.apply(H, out, self.norm, self.norm)

    def apply(self, H, out, pre=None, post=None):
        """out = post * A (pre * H) over the own rows (pre / post: [n] vectors or None): the
        generated programs' GCN_AGGREGATE (codegen/gala.cu:442-456) with column ownership."""
        be, p, c, rows = self.be, self.part, self.part.block, self._rows
        Xs, partial, S = self._buffers(H.shape[1])
        if pre is None:
            Xs.copy_(H)
        else:
            be.row_broadcast(pre, H, Xs)
        works = []
        for k, gk in enumerate(self.graphs):
            Yk = partial[k * rows:(k + 1) * rows]
            be.spmm(gk, Xs, Yk, None, False)
            if p.world > 1:
                works.append(self.comm.reduce_scatter(S[k * c:(k + 1) * c], Yk))
            else:
                S[k * c:(k + 1) * c].copy_(Yk)
        if works:
            self.comm.wait(works)
        if post is None:
            return out.copy_(S[:p.n])
        return be.row_broadcast(post, S[:p.n], out)

    def halo_bytes(self) -> int:
        return self.part.comm_bytes(self.F) if self.part.world > 1 else 0


class VertexCutGat:
    """The REF-mode GAT layer forward (edge softmax + attention-weighted aggregation) with
    column ownership.  The softmax of a row spans every column range, so each rank computes
    for its edges the UNNORMALISED partial rows and softmax sums (GALA_GAT_PARTIAL):
        U_p[r] = sum_{e in row r, col in V_p} p_e X[col],   S_p[r, h] = sum p_e,
        p_e = min(exp(LeakyReLU(aL[r] + aR[col])), 1e12)           (common.h:760-773)
    and two reduce-scatters (the partial rows, and the [rows, H] softmax row statistics)
    hand each owner  Y[r] = (sum_p U_p[r]) / (1e-12 + sum_p S_p[r])  -- REF has no max
    subtraction, so partial sums simply add.  aL of every row arrives by an all-gather of
    the owners' [n, H] blocks per chunk (small); aR and X of the own columns are local.

    Training (`forward_train` + `backward`, the REF layer of the generated programs with the
    row statistics of gala_gat_{fwd,bwd}_stats_f32):
      forward   gala_gat_fwd_partial_stats_f32 adds  Um_p[r] = sum m_e p_e X[col] and
                M_p[r, h] = sum m_e p_e (m_e the LeakyReLU factor) to U_p and S_p; ONE
                reduce-scatter of the packed [U | Um] rows (plus the two [rows, H] sums)
                gives the owner q = 1/(S + 1e-12), Y = q U, Ym = q Um, sma = q M.
      backward  the REF dX[r] = sum_e alpha_e dY[col_e] (A, not A^T: common.h:835-894) only
                reads dY of the columns a rank holds -- its own rows -- so each rank runs the
                same partial forward kernel with dY in place of X (P_p[r] = sum p_e dY[col])
                and one reduce-scatter hands the owner dX = q P.  d_aL of a row needs no edge:
                <dY, Ym> - (<dY, Y> + 1e-12) sma (+1e-12) per head, from the owner's rows
                (gala_gat_bwd_stats_f32 on the owner's rows without edges).
    No dY or X row crosses the links; per layer the collectives move (2F + 2H) floats per
    row forward and F backward.  Results agree with one GPU to fp32 rounding (each row's
    sums are regrouped by column range, and dX is q * sum p dY instead of sum fl(p q) dY)."""

    def __init__(self, part: VertexCutPartition, F: int, heads: int, backend, comm=None, slope: float = 0.2):
        self.part, self.F, self.H, self.be, self.comm, self.slope = part, F, heads, backend, comm, slope
        thr = part.split_threshold
        self.graphs = [backend.graph(h, split=thr) for h in part.chunk_graphs]
        P, c, K = part.world, part.block, part.chunks
        self._rows = P * c
        self.U = backend.empty(K * P * c, F)
        self.S = backend.empty(K * P * c * heads)
        self.Uown = backend.empty(K * c, F)
        self.Sown = backend.empty(K * c * heads)
        self.aLpad = backend.empty(K * c, heads)
        self.aLall = backend.empty(K * P * c, heads)
        self._train = None   # buffers of forward_train / backward, allocated on first use
        self.saved = None

    def __call__(self, aL, aR, X):
        """aL [n, H] (own rows), aR [n, H] and X [n, F] (own columns) -> Y [n, F] (own rows)."""
        p, H, c, rows = self.part, self.H, self.part.block, self._rows
        n = p.n
        self.aLpad[:n].copy_(aL.reshape(n, H))
        self.aLpad[n:].zero_()
        works = []
        for k, gk in enumerate(self.graphs):
            al_k = self.aLall[k * rows:(k + 1) * rows]
            if p.world > 1:
                self.comm.wait([self.comm.all_gather(al_k, self.aLpad[k * c:(k + 1) * c])])
            else:
                al_k.copy_(self.aLpad[k * c:(k + 1) * c])
            Uk = self.U[k * rows:(k + 1) * rows]
            Sk = self.S[k * rows * H:(k + 1) * rows * H]
            self.be.gat_partial(gk, al_k, aR, X, H, self.slope, Uk, Sk)
            if p.world > 1:
                works.append(self.comm.reduce_scatter(self.Uown[k * c:(k + 1) * c], Uk))
                works.append(self.comm.reduce_scatter(self.Sown[k * c * H:(k + 1) * c * H], Sk))
            else:
                self.Uown[k * c:(k + 1) * c].copy_(Uk)
                self.Sown[k * c * H:(k + 1) * c * H].copy_(Sk)
        if works:
            self.comm.wait(works)
        q = 1.0 / (self.Sown[:n * H].view(n, H) + 1e-12)
        D = self.F // H
        return (self.Uown[:n].view(n, H, D) * q.view(n, H, 1)).reshape(n, self.F)

    def _gather_aL(self, aL):
        """aLall chunk by chunk (the [rows, H] logits of every destination row)."""
        p, H, c, rows = self.part, self.H, self.part.block, self._rows
        n = p.n
        self.aLpad[:n].copy_(aL.reshape(n, H))
        self.aLpad[n:].zero_()
        for k in range(p.chunks):
            al_k = self.aLall[k * rows:(k + 1) * rows]
            if p.world > 1:
                self.comm.wait([self.comm.all_gather(al_k, self.aLpad[k * c:(k + 1) * c])])
            else:
                al_k.copy_(self.aLpad[k * c:(k + 1) * c])

    def _train_buffers(self):
        if self._train is None:
            be, p, H, F = self.be, self.part, self.H, self.F
            K, P, c = p.chunks, p.world, p.block
            own = layout.HostGraph(p.n, p.n, np.zeros(p.n + 1, np.int32), np.zeros(0, np.int32))
            self._train = {
                "UU": be.empty(K * P * c, 2 * F), "UUown": be.empty(K * c, 2 * F),
                "M": be.empty(K * P * c * H), "Mown": be.empty(K * c * H),
                "P": be.empty(K * P * c, F), "Pown": be.empty(K * c, F), "Ssc": be.empty(K * P * c * H),
                "own": be.graph(own, split=False),
            }
        return self._train

    def _owner_scale(self, q, T):
        """q [n, H] times the [n, F] rows T per head (the owner's normalisation)."""
        n, H = q.shape
        return (T.reshape(n, H, self.F // H) * q.view(n, H, 1)).reshape(n, self.F)

    def forward_train(self, aL, aR, X, wR=None, bR=None):
        """aL [n, H] (own rows), aR [n, H], X [n, F] (own columns) -> Y [n, F]; keeps the
        row statistics (q, Y, Ym, sma of the own rows) for `backward`.  aR None: the source
        logits are the per-head Linear (wR [F], bR [H]) of X, recomputed inside the kernel
        from the gathered rows (the DSL's attnR = ffn(res, out=1)); the backward then takes
        them from one gala_head_attn_f32 pass over the own rows."""
        p, H, F, c, rows = self.part, self.H, self.F, self.part.block, self._rows
        n, b = p.n, self._train_buffers()
        self._gather_aL(aL)
        works = []
        for k, gk in enumerate(self.graphs):
            UUk = b["UU"][k * rows:(k + 1) * rows]
            Sk = self.S[k * rows * H:(k + 1) * rows * H]
            Mk = b["M"][k * rows * H:(k + 1) * rows * H]
            self.be.gat_partial_stats(gk, self.aLall[k * rows:(k + 1) * rows], aR, X, H, self.slope,
                                      UUk[:, :F], Sk, UUk[:, F:], Mk, wR=wR, bR=bR)
            dst = (b["UUown"][k * c:(k + 1) * c], self.Sown[k * c * H:(k + 1) * c * H],
                   b["Mown"][k * c * H:(k + 1) * c * H])
            for d, s in zip(dst, (UUk, Sk, Mk)):
                if p.world > 1:
                    works.append(self.comm.reduce_scatter(d, s))
                else:
                    d.copy_(s)
        if aR is None:   # the backward's source logits of the own columns
            aR = self.be.head_attn(X, wR, bR, H)
        if works:
            self.comm.wait(works)
        q = 1.0 / (self.Sown[:n * H].view(n, H) + 1e-12)
        Y = self._owner_scale(q, b["UUown"][:n, :F])
        Ym = self._owner_scale(q, b["UUown"][:n, F:])
        sma = b["Mown"][:n * H].view(n, H) * q
        self.saved = (aL.reshape(n, H), aR, q, Y, Ym, sma)
        return Y

    def backward(self, dY):
        """dY [n, F] of the own rows -> (dX [n, F], d_aL [n, H]) of the REF layer."""
        if self.saved is None:
            raise RuntimeError("VertexCutGat.backward: no forward_train to take the row statistics from")
        p, H, F, c, rows = self.part, self.H, self.F, self.part.block, self._rows
        n, b = p.n, self._train_buffers()
        aL, aR, q, Y, Ym, sma = self.saved
        works = []
        for k, gk in enumerate(self.graphs):
            Pk = b["P"][k * rows:(k + 1) * rows]
            self.be.gat_partial(gk, self.aLall[k * rows:(k + 1) * rows], aR, dY, H, self.slope, Pk,
                                b["Ssc"][k * rows * H:(k + 1) * rows * H])
            if p.world > 1:
                works.append(self.comm.reduce_scatter(b["Pown"][k * c:(k + 1) * c], Pk))
            else:
                b["Pown"][k * c:(k + 1) * c].copy_(Pk)
        # the row-local d_aL needs no edge and overlaps the reduce-scatter
        _, d_aL = self.be.gat_bwd_stats(b["own"], aL, aR, dY, q, Y, Ym, sma, H, self.slope)
        if works:
            self.comm.wait(works)
        return self._owner_scale(q, b["Pown"][:n]), d_aL.view(n, H)
