"""The local operator tables the multi-GPU aggregators run on.

`HipBackend` launches the HIP kernels of libgala_hip.so on torch's current stream (device
tensors, gala.ops).  `CpuBackend` runs the same operators on the host cores through
libgala_cpu.so (include/gala_cpu.h: same signatures, same per-row order and rounding, so
its results are bit-identical to the HIP kernels').  The CPU table exists for the CPU test
suite and for plumbing runs of bench.py (`--device cpu`); it is chosen explicitly by the
caller and is never a fallback for a missing HIP library.

Both expose the four operations one GCN aggregation `norm * A (norm * H)` needs
(codegen/gala.cu:433-456): graph upload, SpMM, ROW_BROADCAST and the degree pass.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _abi
from .layout import HostGraph


class HipBackend:
    name = "hip"

    def __init__(self, device="cuda", hub="exact"):
        from . import ops
        self.ops = ops
        self.device = torch.device(device)
        # hub rows of a split plan: "exact" (the reference's order, bit-identical) or
        # "chunked" (GALA_SPMM_HUB_CHUNKED, the fast mode)
        self.hub = hub

    def graph(self, hg: HostGraph, split="auto"):
        return self.ops.DeviceGraph.from_host(hg, self.device, split=split)

    def spmm(self, g, X, out, dst_scale=None, accum=False, samp=None):
        """samp (nsamp, ra, rb): the kernel-sampled aggregation (GALA_SPMM_SAMPLE)."""
        if samp is None:
            return self.ops.spmm(g, X, out=out, dst_scale=dst_scale, accum=accum, hub=self.hub)
        return self.ops.spmm(g, X, out=out, dst_scale=dst_scale, accum=accum, nsamp=samp[0], ra=samp[1], rb=samp[2])

    def row_broadcast(self, scale, X, out):
        return self.ops.row_broadcast(scale, X, out=out)

    def spmm_deg(self, g, X, out, out2=None):
        """out = deg^-0.5 * A X with the norm formed from the rowptr inside the SpMM, and
        optionally out2 = deg^-0.5 * out (gala_spmm_ex_f32's epilogue)."""
        return self.ops.spmm(g, X, out=out, dst_deg=True, out2=out2, hub=self.hub)

    def row_broadcast_deg(self, g, X, out):
        """out = deg^-0.5 * X, the norm from g's rowptr (gala_row_broadcast_deg_f32)."""
        return self.ops.row_broadcast_deg(g, X, out=out)

    def degree(self, g, power=-0.5):
        return self.ops.degree(g, power=power)

    def gat_partial(self, g, aL, aR, X, heads, slope, Y, sums):
        """REF GAT forward over one column range, unnormalised (GALA_GAT_PARTIAL)."""
        return self.ops.gat_fwd_partial(g, aL, X, aR=aR, heads=heads, slope=slope, Y=Y, sums=sums)

    def gat_partial_stats(self, g, aL, aR, X, heads, slope, U, sums, Um, msums, wR=None, bR=None,
                          self_col=None, aR_out=None):
        """REF row-statistics forward over one column range, unnormalised (vertex cut); aR
        None: recomputed per head from X (wR, bR), and with self_col / aR_out the own
        vertices' recomputed logits are written out."""
        return self.ops.gat_fwd_partial_stats(g, aL, X, aR=aR, wR=wR, bR=bR, heads=heads, slope=slope, U=U,
                                              sums=sums, Um=Um, msums=msums, self_col=self_col, aR_out=aR_out)

    def gat_continue(self, g, aL, aR, X, heads, slope, U0, S0, Um0=None, M0=None, wR=None, bR=None, partial=False):
        """REF forward (or, with Um0 / M0, the row statistics) continued from the partials of
        an earlier column range, in place (gala_gat_fwd_continue_f32; partial: unnormalised)."""
        return self.ops.gat_fwd_continue(g, aL, X, U0, S0, aR=aR, wR=wR, bR=bR, heads=heads, slope=slope, Um0=Um0,
                                         M0=M0, partial=partial)

    def gat_bwd_stats(self, g, aL, aR, dY, q, Y, Ym, sma, heads, slope):
        """(dX, d_aL) of the REF layer from its row statistics (gala_gat_bwd_stats_f32)."""
        return self.ops.gat_bwd_stats(g, aL, aR, dY, q, Y, Ym, sma, heads=heads, slope=slope)

    def head_attn(self, X, w, b, heads):
        """[n, heads] per-head attention logits <X[:, head h], w_h> + b_h (gala_head_attn_f32)."""
        return self.ops.head_attn(X, w, b, heads=heads)

    def gat_stats_table(self, g, aL, aR, X, heads, slope, self_col, aR_out, wR=None, bR=None):
        """REF statistics forward over a gathered table (gala_gat_fwd_stats_ex_f32)."""
        return self.ops.gat_fwd_stats(g, aL, X, aR=aR, wR=wR, bR=bR, heads=heads, slope=slope, self_col=self_col,
                                      aR_out=aR_out)

    def gat_bwd_stats_table(self, g, aL, aR, dY, dY_rows, q, Y, Ym, sma, heads, slope, wR=None):
        """(dX, d_aL) over a gathered table (gala_gat_bwd_stats_ex_f32); wR: dX also takes the
        source logit's per-head Linear (gala_gat_bwd_stats_linear_f32)."""
        return self.ops.gat_bwd_stats(g, aL, aR, dY, q, Y, Ym, sma, heads=heads, slope=slope, dY_rows=dY_rows, wR=wR)

    def row_scale_relu(self, act, pre, X, out):
        """out = pre * relu(act * X) (gala_row_scale_relu_f32: the ReLU prologue)."""
        return self.ops.row_scale_relu(X, act, pre, out=out)

    def relu_scale_backward(self, act, X, G, out):
        """out = act * (relu(act * X) <= 0 ? 0 : G) (gala_relu_scale_backward_f32)."""
        return self.ops.relu_scale_backward(X, G, act, out=out)

    def head_attn_bwd(self, g, w, heads, dX):
        """dX[:, head h] += g[:, h] * w[head h] (gala_head_attn_bwd_f32, accumulating)."""
        return self.ops.head_attn_bwd(g.contiguous(), w, heads=heads, dX=dX, n_rows=dX.shape[0])

    def head_linear_grads(self, X, g, heads):
        """(dW [F], db [H]) of the per-head attention Linear, d logit g [n, H]: the block
        diagonal of dense_grad's [H, F] (head h's weights are columns h*D:(h+1)*D)."""
        full, db = self.ops.dense_grad(X, g.contiguous())
        return _block_diag(full, heads), db

    def empty(self, *shape):
        return torch.empty(shape, device=self.device, dtype=torch.float32)

    def synchronize(self):
        torch.cuda.synchronize(self.device)


def _block_diag(full, heads):
    F = full.shape[1]
    D = F // heads
    return full.view(heads, heads, D).diagonal(0, 0, 1).t().reshape(F).contiguous()


class CpuGraph:
    """A HostGraph with its gala_csr_t view (host pointers) for libgala_cpu.so."""

    def __init__(self, hg: HostGraph):
        self.hg = hg
        self.n_rows, self.n_cols = hg.n_rows, hg.n_cols
        self.rowptr = np.ascontiguousarray(hg.rowptr, np.int32)
        self.col = np.ascontiguousarray(hg.col, np.int32)
        self.bounds = None if hg.bounds is None else np.ascontiguousarray(hg.bounds, np.int32)
        c = _abi.gala_csr_t()
        c.n_rows, c.n_cols, c.nnz = hg.n_rows, hg.n_cols, int(self.col.shape[0])
        c.rowptr = self.rowptr.ctypes.data if hg.n_rows > 0 else None
        c.col = self.col.ctypes.data if self.col.shape[0] > 0 else None
        c.val, c.val_heads, c.split = None, 1, None
        c.n_seg = hg.n_seg
        c.seg_bounds = None if self.bounds is None else self.bounds.ctypes.data
        self.c = c

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])

    def csr(self):
        return ctypes.byref(self.c)


def _hp(t: torch.Tensor):
    if t is None:
        return None
    if t.is_cuda:
        raise ValueError("CpuBackend takes host tensors")
    return t.data_ptr()


class CpuBackend:
    name = "cpu"
    device = torch.device("cpu")
    hub = "exact"   # the host rows are always one sequential pass

    def graph(self, hg: HostGraph, split="auto"):
        return CpuGraph(hg)

    def spmm(self, g: CpuGraph, X, out, dst_scale=None, accum=False, samp=None):
        flags = (_abi.GALA_SPMM_ACCUM if accum else 0) | (_abi.GALA_SPMM_SAMPLE if samp is not None else 0)
        ns, ra, rb = samp if samp is not None else (0, 5, 7)
        _abi.call_cpu("gala_spmm_f32", g.csr(), _hp(X), X.stride(0), _hp(out), out.stride(0), X.shape[1],
                      None, _hp(dst_scale), flags, ns, ra, rb, None)
        return out

    def row_broadcast(self, scale, X, out):
        _abi.call_cpu("gala_row_broadcast_f32", X.shape[0], X.shape[1], _hp(scale), _hp(X), X.stride(0),
                      _hp(out), out.stride(0), None)
        return out

    def spmm_deg(self, g: CpuGraph, X, out, out2=None):
        epi = _abi.gala_spmm_epilogue_t()
        epi.dst_deg_rsqrt = 1
        epi.Y2, epi.ldy2, epi.y2_scale = _hp(out2), (out2.stride(0) if out2 is not None else 0), None
        _abi.call_cpu("gala_spmm_ex_f32", g.csr(), _hp(X), X.stride(0), _hp(out), out.stride(0), X.shape[1], None,
                      None, 0, 0, 5, 7, ctypes.byref(epi), None)
        return out

    def row_broadcast_deg(self, g: CpuGraph, X, out):
        _abi.call_cpu("gala_row_broadcast_deg_f32", g.csr(), X.shape[1], _hp(X), X.stride(0), _hp(out),
                      out.stride(0), None)
        return out

    def degree(self, g: CpuGraph, power=-0.5):
        out = torch.empty(g.n_rows, dtype=torch.float32)
        _abi.call_cpu("gala_degree_f32", g.csr(), _hp(out), power, 0, 0, None)
        return out

    def gat_partial(self, g: CpuGraph, aL, aR, X, heads, slope, Y, sums):
        _abi.call_cpu("gala_gat_fwd_ex_f32", g.csr(), _hp(aL), _hp(aR), None, None, _hp(X), X.stride(0), X.shape[1],
                      heads, slope, _abi.GALA_SOFTMAX_REF | _abi.GALA_GAT_PARTIAL, _hp(Y), Y.stride(0), None,
                      _hp(sums), None)
        return Y, sums

    def gat_partial_stats(self, g: CpuGraph, aL, aR, X, heads, slope, U, sums, Um, msums, wR=None, bR=None,
                          self_col=None, aR_out=None):
        _abi.call_cpu("gala_gat_fwd_partial_stats_ex_f32", g.csr(), _hp(aL), _hp(aR), _hp(wR), _hp(bR), _hp(X),
                      X.stride(0), X.shape[1], heads, slope, _hp(U), U.stride(0), _hp(sums), _hp(Um), Um.stride(0),
                      _hp(msums), _hp(self_col), _hp(aR_out), None)
        return U, sums, Um, msums

    def gat_continue(self, g: CpuGraph, aL, aR, X, heads, slope, U0, S0, Um0=None, M0=None, wR=None, bR=None,
                     partial=False):
        _abi.call_cpu("gala_gat_fwd_continue_f32", g.csr(), _hp(aL), _hp(aR), _hp(wR), _hp(bR), _hp(X), X.stride(0),
                      X.shape[1], heads, slope, _abi.GALA_GAT_PARTIAL if partial else 0, _hp(U0), U0.stride(0), _hp(S0), _hp(Um0),
                      Um0.stride(0) if Um0 is not None else 0, _hp(M0), _hp(U0), U0.stride(0), _hp(S0), _hp(Um0),
                      Um0.stride(0) if Um0 is not None else 0, _hp(M0), None)
        return (U0, S0) if Um0 is None else (U0, S0, Um0, M0)

    def gat_bwd_stats(self, g: CpuGraph, aL, aR, dY, q, Y, Ym, sma, heads, slope):
        F = dY.shape[1]
        dX = torch.empty((g.n_rows, F), dtype=torch.float32)
        d_aL = torch.empty(g.n_rows * heads, dtype=torch.float32)
        _abi.call_cpu("gala_gat_bwd_stats_f32", g.csr(), _hp(aL), _hp(aR), None, _hp(dY), dY.stride(0), F, heads,
                      slope, _hp(q), _hp(Y), Y.stride(0), _hp(Ym), Ym.stride(0), _hp(sma), _hp(dX), dX.stride(0),
                      _hp(d_aL), None)
        return dX, d_aL

    def gat_stats_table(self, g: CpuGraph, aL, aR, X, heads, slope, self_col, aR_out, wR=None, bR=None):
        n, F = g.n_rows, X.shape[1]
        Y, Ym = torch.empty((n, F)), torch.empty((n, F))
        q, sma = torch.empty(n * heads), torch.empty(n * heads)
        _abi.call_cpu("gala_gat_fwd_stats_ex_f32", g.csr(), _hp(aL), _hp(aR), _hp(wR), _hp(bR), _hp(X), X.stride(0),
                      F, heads, slope, _hp(Y), F, _hp(q), _hp(Ym), F, _hp(sma), _hp(self_col), _hp(aR_out), None, None)
        return Y, q, Ym, sma

    def gat_bwd_stats_table(self, g: CpuGraph, aL, aR, dY, dY_rows, q, Y, Ym, sma, heads, slope, wR=None):
        F = dY.shape[1]
        dX = torch.empty((g.n_rows, F), dtype=torch.float32)
        d_aL = torch.empty(g.n_rows * heads, dtype=torch.float32)
        if wR is not None:
            _abi.call_cpu("gala_gat_bwd_stats_linear_f32", g.csr(), _hp(aL), _hp(aR), None, _hp(dY), dY.stride(0),
                          _hp(dY_rows), F, heads, slope, _hp(q), _hp(Y), Y.stride(0), _hp(Ym), Ym.stride(0),
                          _hp(sma), _hp(wR), _hp(dX), dX.stride(0), _hp(d_aL), None)
            return dX, d_aL
        _abi.call_cpu("gala_gat_bwd_stats_ex_f32", g.csr(), _hp(aL), _hp(aR), None, _hp(dY), dY.stride(0),
                      _hp(dY_rows), F, heads, slope, _hp(q), _hp(Y), Y.stride(0), _hp(Ym), Ym.stride(0), _hp(sma),
                      _hp(dX), dX.stride(0), _hp(d_aL), None)
        return dX, d_aL

    def head_attn(self, X, w, b, heads):
        out = torch.empty((X.shape[0], heads), dtype=torch.float32)
        _abi.call_cpu("gala_head_attn_f32", X.shape[0], X.shape[1], heads, _hp(X), X.stride(0), _hp(w), _hp(b),
                      _hp(out), None)
        return out

    def row_scale_relu(self, act, pre, X, out):
        _abi.call_cpu("gala_row_scale_relu_f32", X.shape[0], X.shape[1], _hp(act), _hp(pre), _hp(X), X.stride(0),
                      _hp(out), out.stride(0), None)
        return out

    def relu_scale_backward(self, act, X, G, out):
        _abi.call_cpu("gala_relu_scale_backward_f32", X.shape[0], X.shape[1], _hp(act), _hp(X), X.stride(0), _hp(G),
                      G.stride(0), _hp(out), out.stride(0), None)
        return out

    def head_attn_bwd(self, g, w, heads, dX):
        g = g.contiguous()
        _abi.call_cpu("gala_head_attn_bwd_f32", dX.shape[0], w.numel(), heads, _hp(g), _hp(w), _hp(dX), dX.stride(0),
                      1, None)
        return dX

    def head_linear_grads(self, X, g, heads):
        g = g.contiguous()
        N, K = X.shape
        full = torch.empty((heads, K), dtype=torch.float32)
        db = torch.empty(heads, dtype=torch.float32)
        wsb = int(_abi.cpu_lib().gala_cpu_dense_grad_workspace(N, K, heads))
        ws = torch.empty(max(wsb // 4, 1), dtype=torch.float32)
        _abi.call_cpu("gala_dense_grad_f32", N, K, heads, _hp(X), X.stride(0), _hp(g), heads, _hp(full), _hp(db), 0,
                      _hp(ws), wsb, None)
        return _block_diag(full, heads), db

    def empty(self, *shape):
        return torch.empty(shape, dtype=torch.float32)

    def synchronize(self):
        pass


def make_backend(device) -> "HipBackend | CpuBackend":
    d = torch.device(device)
    return CpuBackend() if d.type == "cpu" else HipBackend(d)
