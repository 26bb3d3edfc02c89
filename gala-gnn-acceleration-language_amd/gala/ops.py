"""torch-facing functional ops over the C ABI (device tensors, current HIP stream).

Each op allocates its output with the torch caching allocator and launches the HIP
kernel on torch's current stream.  There is no CPU fallback: CPU tensors raise.
The C++/libtorch mirror of the reference's emitted operator API (the `*_call`
wrappers and autograd Functions of codegen/gala.cu) lives in host/gala_torch.cpp.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _abi
from .layout import HostGraph, split_threshold


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _dp(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("gala ops take device tensors (no CPU fallback)")
    return t.data_ptr()


class DeviceGraph:
    """Device-resident graph (the generated code's global_*_graph slots, gala.cu:32-43)."""

    def __init__(self, n_rows, n_cols, rowptr, col, val=None, n_seg=1, bounds=None, val_heads=1,
                 val_row_scale=None):
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)
        self.rowptr, self.col, self.val = rowptr, col, val
        self.val_row_scale = val_row_scale
        self.n_seg = int(n_seg)
        self.val_heads = int(val_heads)
        self.bounds = None if bounds is None else np.ascontiguousarray(bounds, np.int32)
        self._csr = None
        # hub-row split plan, shared with with_values() views:
        # {"plan": gala_split_plan_t, "arrays": device index arrays, "ws": workspace tensor}
        self._split = None

    @classmethod
    def from_host(cls, g: HostGraph, device="cuda", split="auto"):
        rp = torch.from_numpy(np.ascontiguousarray(g.rowptr)).to(device)
        col = torch.from_numpy(np.ascontiguousarray(g.col)).to(device)
        val = None if g.val is None else torch.from_numpy(np.ascontiguousarray(g.val, np.float32)).to(device)
        dg = cls(g.n_rows, g.n_cols, rp, col, val, g.n_seg, g.bounds, g.val_heads)
        if split and g.n_seg == 1 and g.n_rows > 0:
            deg = np.diff(g.rowptr)
            mean = g.nnz / max(g.n_rows, 1)
            thr = split_threshold(g.n_rows, g.nnz)
            if split != "auto":
                thr = int(split)
            hubs = deg.max(initial=0) > thr
            skewed = deg.max(initial=0) > 4 * max(mean, 1.0)
            if hubs or skewed:
                dg.set_split_plan(g.rowptr, thr if hubs else 0, chunk=512, row_order=skewed)
        return dg

    def set_split_plan(self, host_rowptr, threshold: int, chunk: int = 512, row_order: bool = False):
        """Hub-row splitting and / or a degree-ordered row schedule (gala_split_plan_t), built
        from the host rowptr.  threshold 0: no hub rows, only the row order."""
        rp = np.ascontiguousarray(host_rowptr, np.int32)
        nr = ctypes.c_int64(0)
        nc = ctypes.c_int64(0)
        rows, rc0, crow = np.zeros(1, np.int32), np.zeros(1, np.int32), np.zeros(1, np.int32)
        if threshold > 0:
            _abi.call("gala_host_split_plan", self.n_rows, rp.ctypes.data, threshold, chunk, None, None,
                      None, ctypes.byref(nr), ctypes.byref(nc))
            rows = np.empty(max(nr.value, 1), np.int32)
            rc0 = np.empty(nr.value + 1, np.int32)
            crow = np.empty(max(nc.value, 1), np.int32)
            _abi.call("gala_host_split_plan", self.n_rows, rp.ctypes.data, threshold, chunk,
                      rows.ctypes.data, rc0.ctypes.data, crow.ctypes.data, ctypes.byref(nr), ctypes.byref(nc))
        order = None
        if row_order:
            order = np.empty(max(self.n_rows, 1), np.int32)
            _abi.call("gala_host_row_order", self.n_rows, rp.ctypes.data, order.ctypes.data)
        dev = self.col.device
        arrays = tuple(torch.from_numpy(a).to(dev) for a in (rows, rc0, crow))
        order_t = None if order is None else torch.from_numpy(order).to(dev)
        plan = _abi.gala_split_plan_t()
        plan.threshold, plan.chunk = max(threshold, 1), chunk
        plan.n_rows_split, plan.n_chunks = nr.value, nc.value
        plan.rows, plan.row_chunk0, plan.chunk_row = (a.data_ptr() for a in arrays)
        plan.workspace, plan.ws_cols = None, 0
        plan.row_order = None if order_t is None else order_t.data_ptr()
        aux = None
        if nr.value > 0 and dev.type == "cuda":
            # the REF-order hub rows run beside the row kernel on a side stream (fork / join
            # events recorded by the library on the caller's stream); a high-priority one, so
            # the longest serial chains (the hub launch's first workgroups) are dispatched
            # before the row kernel fills the CUs (R-MAT: 1.87 -> 1.81 ms,
            # profiles/r06_hub_clock_swizzle.jsonl)
            aux = (torch.cuda.Stream(device=dev, priority=-1), torch.cuda.Event(), torch.cuda.Event())
            for ev in aux[1:]:
                ev.record(aux[0])   # creates the event handles
            plan.aux_stream = aux[0].cuda_stream
            plan.aux_events[0], plan.aux_events[1] = aux[1].cuda_event, aux[2].cuda_event
        self._split = {"plan": plan, "arrays": arrays + (order_t,), "ws": None, "aux": aux}
        self._csr = None

    @property
    def split_rows(self) -> int:
        return 0 if self._split is None else int(self._split["plan"].n_rows_split)

    @property
    def nnz(self) -> int:
        return int(self.col.numel())

    def with_values(self, val, val_heads=1, row_scale=None) -> "DeviceGraph":
        """The same structure with edge values val [nnz, val_heads]; row_scale [n_rows,
        val_heads] stores them factored (A_e,h = val[e,h] * row_scale[row,h], rounded: the
        GAT forward's (p, q) output used as alpha)."""
        g = DeviceGraph(self.n_rows, self.n_cols, self.rowptr, self.col, val, self.n_seg,
                        self.bounds, val_heads, row_scale)
        g._split = self._split
        return g

    def csr(self, F: int = 0):
        if self._split is not None and F > 0:
            F = (F + 3) // 4 * 4  # chunk rows hold whole float4 vectors (padded rows included)
            plan = self._split["plan"]
            if plan.ws_cols < F:  # workspace for the chunk partials, grown on demand
                ws = torch.empty(max(int(plan.n_chunks), 1) * F, device=self.col.device)
                self._split["ws"] = ws
                plan.workspace, plan.ws_cols = ws.data_ptr(), F
            self._csr = None
        if self._csr is None:
            c = _abi.gala_csr_t()
            c.n_rows, c.n_cols, c.nnz = self.n_rows, self.n_cols, self.nnz
            c.rowptr = _dp(self.rowptr)
            c.col = _dp(self.col)
            c.val = _dp(self.val)
            c.val_heads = self.val_heads
            c.n_seg = self.n_seg
            c.seg_bounds = None if self.bounds is None else self.bounds.ctypes.data
            c.split = None
            c.val_row_scale = _dp(self.val_row_scale)
            if self._split is not None:
                c.split = ctypes.addressof(self._split["plan"])
            self._csr = c
        return ctypes.byref(self._csr)


def pad_rows(X: torch.Tensor, mult: int = 4) -> torch.Tensor:
    """X as a [N, F] view of row-padded storage (row stride F rounded up to `mult`; a zero-
    padded copy unless X already is one).  With padded rows the kernels use whole float4
    vectors when F % 4 != 0 (F = 47: a gathered row spans 2 cache lines instead of 2.4 on
    average); padding columns are read, zeroed before any dot product, never written."""
    F = X.shape[1]
    Fp = (F + mult - 1) // mult * mult
    if X.stride(1) == 1 and X.stride(0) >= Fp and X.stride(0) % mult == 0:
        return X
    buf = torch.zeros((X.shape[0], Fp), device=X.device, dtype=X.dtype)
    buf[:, :F].copy_(X)
    return buf[:, :F]


def _rows_like(X: torch.Tensor, n_rows: int, zero: bool = False) -> torch.Tensor:
    """An [n_rows, F] output with X's row padding (so the padded float4 path applies)."""
    F, ld = X.shape[1], X.stride(0)
    alloc = torch.zeros if zero else torch.empty
    if X.dim() == 2 and X.stride(1) == 1 and ld > F:
        return alloc((n_rows, ld), device=X.device, dtype=torch.float32)[:, :F]
    return alloc((n_rows, F), device=X.device, dtype=torch.float32)


def spmm(g: DeviceGraph, X: torch.Tensor, src_scale=None, dst_scale=None, out=None,
         accum=False, nsamp=None, ra=5, rb=7, exact=False, hub="exact", dst_deg=False, out2=None,
         out2_scale=None, src_relu=False, src_act=None, relu_x=None, relu_act=None) -> torch.Tensor:
    """Y (+)= dst_scale * A (src_scale * X) (gala_spmm_f32).  hub: how the rows of the
    graph's hub-row plan are summed -- "exact" (default, the reference's sequential CSR
    order, bit-identical) or "chunked" (GALA_SPMM_HUB_CHUNKED: 512-edge chunk partials and
    an ordered fix-up, the fast mode within fp32 summation rounding).  Epilogue
    (gala_spmm_ex_f32): dst_deg -- the dst factor is deg(r)^-0.5 from the rowptr; out2 --
    also out2 = out2_scale (or the dst factor) * Y, the next aggregation's pre-scaled input;
    src_relu -- the gathered source is src_scale * relu(src_act * X) (the next layer's ReLU
    prologue, gala_row_scale_relu_f32's roundings); relu_x -- the ReLU backward of the layer's
    input on the result, Y = relu_act * (relu(relu_act * relu_x) <= 0 ? 0 : Y)
    (gala_relu_scale_backward_f32's roundings).  The ReLU fields need an unweighted, unsampled
    graph without hub rows (else GalaError UNSUPPORTED)."""
    F = X.shape[1]
    if out is None:
        out = _rows_like(X, g.n_rows, zero=accum)
    if hub not in ("exact", "chunked"):
        raise ValueError(f"spmm: hub {hub!r} (exact | chunked)")
    chunked = hub == "chunked" and not exact
    flags = ((_abi.GALA_SPMM_ACCUM if accum else 0) | (_abi.GALA_SPMM_SAMPLE if nsamp is not None else 0)
             | (_abi.GALA_SPMM_EXACT if exact else 0) | (_abi.GALA_SPMM_HUB_CHUNKED if chunked else 0))
    if dst_deg or out2 is not None or src_relu or relu_x is not None:
        epi = _abi.gala_spmm_epilogue_t()
        epi.dst_deg_rsqrt = int(bool(dst_deg))
        epi.Y2, epi.ldy2 = _dp(out2), (out2.stride(0) if out2 is not None else 0)
        epi.y2_scale = _dp(out2_scale)
        epi.src_relu, epi.src_act = int(bool(src_relu)), _dp(src_act)
        epi.relu_x, epi.ldrx = _dp(relu_x), (relu_x.stride(0) if relu_x is not None else 0)
        epi.relu_act = _dp(relu_act)
        _abi.call("gala_spmm_ex_f32", g.csr(F), _dp(X), X.stride(0), _dp(out), out.stride(0), F,
                  _dp(src_scale), _dp(dst_scale), flags, nsamp or 0, ra, rb, ctypes.byref(epi), _stream())
        return out
    _abi.call("gala_spmm_f32", g.csr(F), _dp(X), X.stride(0), _dp(out), out.stride(0), F,
              _dp(src_scale), _dp(dst_scale), flags, nsamp or 0, ra, rb, _stream())
    return out


def row_broadcast_deg(g: DeviceGraph, X, out=None) -> torch.Tensor:
    """out[r, :] = deg(r)^-0.5 * X[r, :], deg from g's rowptr (gala_row_broadcast_deg_f32: the
    degree pass, pow(-0.5) and ROW_BROADCAST in one pass)."""
    if out is None:
        out = _rows_like(X, g.n_rows)
    _abi.call("gala_row_broadcast_deg_f32", g.csr(), X.shape[1], _dp(X), X.stride(0), _dp(out), out.stride(0),
              _stream())
    return out


def degree(g: DeviceGraph, power=1.0, nsamp=None) -> torch.Tensor:
    out = torch.empty(g.n_rows, device=g.col.device, dtype=torch.float32)
    flags = _abi.GALA_SPMM_SAMPLE if nsamp is not None else 0
    _abi.call("gala_degree_f32", g.csr(), _dp(out), power, flags, nsamp or 0, _stream())
    return out


def row_broadcast(scale, X, out=None) -> torch.Tensor:
    """out[r, :] = scale[r] * X[r, :] (ROW_BROADCAST_OP, `norm * res`)."""
    if out is None:
        out = torch.empty_like(X)
    _abi.call("gala_row_broadcast_f32", X.shape[0], X.shape[1], _dp(scale), _dp(X), X.stride(0),
              _dp(out), out.stride(0), _stream())
    return out


def row_scale_relu(X, act=None, pre=None, out=None) -> torch.Tensor:
    """out[r, :] = pre[r] * relu(act[r] * X[r, :]) (gala_row_scale_relu_f32; factors optional)."""
    if out is None:
        out = _rows_like(X, X.shape[0])
    _abi.call("gala_row_scale_relu_f32", X.shape[0], X.shape[1], _dp(act), _dp(pre), _dp(X), X.stride(0),
              _dp(out), out.stride(0), _stream())
    return out


def relu_scale_backward(X, G, act=None, out=None) -> torch.Tensor:
    """dX = act * (relu(act * X) <= 0 ? 0 : G) (gala_relu_scale_backward_f32)."""
    if out is None:
        out = _rows_like(X, X.shape[0])
    _abi.call("gala_relu_scale_backward_f32", X.shape[0], X.shape[1], _dp(act), _dp(X), X.stride(0), _dp(G),
              G.stride(0), _dp(out), out.stride(0), _stream())
    return out


def sddvv(g: DeviceGraph, a, b, op=_abi.GALA_SDDVV_ADD, heads=1, slope=0.2) -> torch.Tensor:
    out = torch.empty(g.nnz * heads, device=a.device, dtype=torch.float32)
    _abi.call("gala_sddvv_f32", g.csr(), _dp(a), _dp(b), heads, op, slope, _dp(out), _stream())
    return out


def row_sum(g: DeviceGraph, v, heads=1, eps=1e-12, out=None, accum=False, hub="exact") -> torch.Tensor:
    """out[r, h] (+)= eps + sum_{e in row r} v[e, h] (K7, gala_row_sum_f32) in the reference's
    order, bit-identical; hub="chunked": the plan's hub rows as chunk partials (fast mode)."""
    if out is None:
        out = torch.zeros(g.n_rows * heads, device=v.device, dtype=torch.float32)
    flags = (_abi.GALA_SPMM_ACCUM if accum else 0) | (_abi.GALA_SPMM_HUB_CHUNKED if hub == "chunked" else 0)
    _abi.call("gala_row_sum_f32", g.csr(2 * heads if hub == "chunked" else 0), _dp(v), heads, eps, _dp(out),
              flags, _stream())
    return out


def row_scale_(g: DeviceGraph, q, v, heads=1) -> torch.Tensor:
    _abi.call("gala_row_scale_f32", g.csr(), _dp(q), heads, _dp(v), _stream())
    return v


def sddmm(g: DeviceGraph, A, B, heads=1) -> torch.Tensor:
    out = torch.empty(g.nnz * heads, device=A.device, dtype=torch.float32)
    _abi.call("gala_sddmm_dot_f32", g.csr(), _dp(A), A.stride(0), _dp(B), B.stride(0),
              A.shape[1], heads, _dp(out), _stream())
    return out


def edge_softmax(g: DeviceGraph, logits, heads=1, mode=_abi.GALA_SOFTMAX_REF) -> torch.Tensor:
    out = torch.empty_like(logits)
    _abi.call("gala_edge_softmax_fwd_f32", g.csr(2 * heads), _dp(logits), heads, mode, _dp(out), _stream())
    return out


def edge_softmax_bwd(g: DeviceGraph, alpha, d_alpha, heads=1, mode=_abi.GALA_SOFTMAX_REF):
    out = torch.empty_like(alpha)
    _abi.call("gala_edge_softmax_bwd_f32", g.csr(2 * heads), _dp(alpha), _dp(d_alpha), heads, mode,
              _dp(out), _stream())
    return out


def gat_fwd(g: DeviceGraph, aL, aR, X, heads=1, slope=0.2, mode=_abi.GALA_SOFTMAX_REF,
            want_alpha=False):
    F = X.shape[1]
    Y = _rows_like(X, g.n_rows)
    alpha = torch.empty(g.nnz * heads, device=X.device, dtype=torch.float32) if want_alpha else None
    _abi.call("gala_gat_fwd_f32", g.csr(F + 2 * heads), _dp(aL), _dp(aR), _dp(X), X.stride(0), F, heads, slope,
              mode, _dp(Y), Y.stride(0), _dp(alpha), _stream())
    return (Y, alpha) if want_alpha else Y


def gat_fwd_attn(g: DeviceGraph, aL, wR, bR, X, slope=0.2, mode=_abi.GALA_SOFTMAX_REF, want_alpha=False):
    """gala_gat_fwd_attn_f32: aR recomputed as X @ wR + bR inside the kernel (one head)."""
    F = X.shape[1]
    Y = _rows_like(X, g.n_rows)
    alpha = torch.empty(g.nnz, device=X.device, dtype=torch.float32) if want_alpha else None
    _abi.call("gala_gat_fwd_attn_f32", g.csr(F + 2), _dp(aL), _dp(wR), _dp(bR), _dp(X), X.stride(0), F, slope,
              mode, _dp(Y), Y.stride(0), _dp(alpha), _stream())
    return (Y, alpha) if want_alpha else Y


def gat_bwd_attn(g: DeviceGraph, aL, wR, bR, X, dY, alpha, slope=0.2):
    """gala_gat_bwd_attn_f32 (REF mode): d_aL (= d_aR)."""
    d_aL = torch.empty(g.n_rows, device=X.device, dtype=torch.float32)
    _abi.call("gala_gat_bwd_attn_f32", g.csr(3), _dp(aL), _dp(wR), _dp(bR), _dp(X), X.stride(0), _dp(dY),
              dY.stride(0), X.shape[1], slope, _dp(alpha), _dp(d_aL), _stream())
    return d_aL


def gat_bwd(g: DeviceGraph, aL, aR, X, dY, alpha, heads=1, slope=0.2, mode=_abi.GALA_SOFTMAX_REF,
            want_dz=False):
    """Fused GAT edge backward (gala_gat_bwd_f32): returns (d_aL, dz or None)."""
    F = X.shape[1]
    d_aL = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32)
    dz = (torch.empty(g.nnz * heads, device=X.device, dtype=torch.float32)
          if (want_dz or mode == _abi.GALA_SOFTMAX_FIXED) else None)
    _abi.call("gala_gat_bwd_f32", g.csr(3 * heads), _dp(aL), _dp(aR), _dp(X), X.stride(0), _dp(dY),
              dY.stride(0), F, heads, slope, mode, _dp(alpha), _dp(dz), _dp(d_aL), _stream())
    return d_aL, dz

def gat_fwd_ex(g: DeviceGraph, aL, X, aR=None, wR=None, bR=None, heads=1, slope=0.2,
               mode=_abi.GALA_SOFTMAX_REF, want_alpha=False, factored=False):
    """gala_gat_fwd_ex_f32: aR given, or recomputed per head from X (wR [F], bR [heads]).
    factored=True (REF): returns (Y, p, q) with alpha = p * q; factored="q": (Y, q) only,
    for gat_bwd_fused; else (Y, alpha) / Y."""
    F = X.shape[1]
    Y = _rows_like(X, g.n_rows)
    alpha = (torch.empty(g.nnz * heads, device=X.device, dtype=torch.float32)
             if (want_alpha or factored == True) else None)  # noqa: E712
    q = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32) if factored else None
    _abi.call("gala_gat_fwd_ex_f32", g.csr(F + 2 * heads), _dp(aL), _dp(aR), _dp(wR), _dp(bR), _dp(X),
              X.stride(0), F, heads, slope, mode, _dp(Y), Y.stride(0), _dp(alpha), _dp(q), _stream())
    if factored == "q":
        return Y, q
    if factored:
        return Y, alpha, q
    return (Y, alpha) if want_alpha else Y


def gat_bwd_ex(g: DeviceGraph, aL, X, dY, alpha, q=None, aR=None, wR=None, bR=None, heads=1, slope=0.2,
               mode=_abi.GALA_SOFTMAX_REF, want_dz=False):
    """gala_gat_bwd_ex_f32: (d_aL, dz or None); q given: alpha holds p (alpha = p * q)."""
    F = X.shape[1]
    d_aL = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32)
    dz = (torch.empty(g.nnz * heads, device=X.device, dtype=torch.float32)
          if (want_dz or mode == _abi.GALA_SOFTMAX_FIXED) else None)
    _abi.call("gala_gat_bwd_ex_f32", g.csr(3 * heads), _dp(aL), _dp(aR), _dp(wR), _dp(bR), _dp(X), X.stride(0),
              _dp(dY), dY.stride(0), F, heads, slope, mode, _dp(alpha), _dp(q), _dp(dz), _dp(d_aL), _stream())
    return d_aL, dz


def gat_fwd_partial(g: DeviceGraph, aL, X, aR=None, wR=None, bR=None, heads=1, slope=0.2, Y=None, sums=None):
    """REF forward over one column range (GALA_GAT_PARTIAL): returns (Y, sums) with Y[r] =
    sum_e p_e X[col_e] unnormalised and sums[r, h] = sum_e p_e, for the vertex cut."""
    F = X.shape[1]
    if Y is None:
        Y = _rows_like(X, g.n_rows)
    if sums is None:
        sums = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32)
    _abi.call("gala_gat_fwd_ex_f32", g.csr(F + 2 * heads), _dp(aL), _dp(aR), _dp(wR), _dp(bR), _dp(X),
              X.stride(0), F, heads, slope, _abi.GALA_SOFTMAX_REF | _abi.GALA_GAT_PARTIAL, _dp(Y), Y.stride(0),
              None, _dp(sums), _stream())
    return Y, sums


def gat_bwd_fused(g: DeviceGraph, aL, X, dY, q, aR=None, wR=None, bR=None, heads=1, slope=0.2):
    """gala_gat_bwd_fused_f32 (REF): attention recomputed from (aL, aR | wR, bR, q); returns
    (dX, d_aL) with dX = A_alpha dY on the forward pattern."""
    F = X.shape[1]
    dX = _rows_like(dY, g.n_rows)
    d_aL = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32)
    _abi.call("gala_gat_bwd_fused_f32", g.csr((F + 3) // 4 * 4 + 3 * heads), _dp(aL), _dp(aR), _dp(wR), _dp(bR),
              _dp(X), X.stride(0), _dp(dY), dY.stride(0), F, heads, slope, _dp(q), _dp(dX), dX.stride(0),
              _dp(d_aL), _stream())
    return dX, d_aL


def gat_fwd_stats(g: DeviceGraph, aL, X, aR=None, wR=None, bR=None, heads=1, slope=0.2, want_aR=False,
                  want_p=False, self_col=None, aR_out=None):
    """gala_gat_fwd_stats_f32 (REF, square pattern): returns (Y, q, Ym, sma[, aR_out][, p]) with
    Ym[r] = sum_e m_e alpha_e X[col_e], sma[r, h] = sum_e m_e alpha_e (m_e the LeakyReLU
    factor); aR_out (aR recomputed from wR, bR) the rows' own source logits; p the edges'
    exp terms.  self_col (int32 [rows]): X is a gathered table whose column self_col[r] is
    row r's own vertex (gala_gat_fwd_stats_ex_f32); aR_out is then a caller-given
    column-indexed [n_cols, heads] buffer, written at the own columns."""
    if self_col is not None:
        F = X.shape[1]
        Y, Ym = _rows_like(X, g.n_rows), _rows_like(X, g.n_rows)
        q = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32)
        sma = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32)
        _abi.call("gala_gat_fwd_stats_ex_f32", g.csr(2 * ((F + 3) // 4 * 4) + 3 * heads), _dp(aL), _dp(aR), _dp(wR),
                  _dp(bR), _dp(X), X.stride(0), F, heads, slope, _dp(Y), Y.stride(0), _dp(q), _dp(Ym), Ym.stride(0),
                  _dp(sma), _dp(self_col), _dp(aR_out), None, _stream())
        return Y, q, Ym, sma
    F = X.shape[1]
    Y = _rows_like(X, g.n_rows)
    Ym = _rows_like(X, g.n_rows)
    q = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32)
    sma = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32)
    aR_out = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32) if want_aR else None
    p = torch.empty(g.nnz * heads, device=X.device, dtype=torch.float32) if want_p else None
    _abi.call("gala_gat_fwd_stats_f32", g.csr(2 * ((F + 3) // 4 * 4) + 3 * heads), _dp(aL), _dp(aR), _dp(wR),
              _dp(bR), _dp(X), X.stride(0), F, heads, slope, _dp(Y), Y.stride(0), _dp(q), _dp(Ym), Ym.stride(0),
              _dp(sma), _dp(aR_out), _dp(p), _stream())
    out = (Y, q, Ym, sma)
    if want_aR:
        out += (aR_out,)
    if want_p:
        out += (p,)
    return out


def gat_fwd_partial_stats(g: DeviceGraph, aL, X, aR=None, wR=None, bR=None, heads=1, slope=0.2, U=None, sums=None,
                          Um=None, msums=None, self_col=None, aR_out=None):
    """gala_gat_fwd_partial_stats_f32 (vertex cut): the row-statistics forward over one
    column range, unnormalised -- (U, sums, Um, msums) = (sum p X, sum p, sum m p X, sum m p)
    per row (and head); U / Um may be strided views (e.g. the two halves of one buffer).
    self_col (int32 [rows], -1 = none) + aR_out ([n_cols, heads]): the own vertices'
    recomputed source logits (gala_gat_fwd_partial_stats_ex_f32)."""
    F = X.shape[1]
    U = _rows_like(X, g.n_rows) if U is None else U
    Um = _rows_like(X, g.n_rows) if Um is None else Um
    sums = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32) if sums is None else sums
    msums = torch.empty(g.n_rows * heads, device=X.device, dtype=torch.float32) if msums is None else msums
    args = (g.csr(2 * ((F + 3) // 4 * 4) + 3 * heads), _dp(aL), _dp(aR), _dp(wR), _dp(bR), _dp(X), X.stride(0), F,
            heads, slope, _dp(U), U.stride(0), _dp(sums), _dp(Um), Um.stride(0), _dp(msums))
    if self_col is None and aR_out is None:
        _abi.call("gala_gat_fwd_partial_stats_f32", *args, _stream())
    else:
        _abi.call("gala_gat_fwd_partial_stats_ex_f32", *args, _dp(self_col), _dp(aR_out), _stream())
    return U, sums, Um, msums


def gat_fwd_continue(g: DeviceGraph, aL, X, U0, S0, aR=None, wR=None, bR=None, heads=1, slope=0.2, Um0=None,
                     M0=None, Y=None, q=None, Ym=None, sma=None, partial=False):
    """gala_gat_fwd_continue_f32: the REF forward (Um0 None) or the row-statistics forward of
    rows whose first column range already gave the partials (U0, S0[, Um0, M0]); the outputs
    default to those buffers (in place).  partial: left unnormalised for a further range.
    Returns (Y, q) or (Y, q, Ym, sma)."""
    F = X.shape[1]
    Y = U0 if Y is None else Y
    q = S0 if q is None else q
    if Um0 is not None:
        Ym = Um0 if Ym is None else Ym
        sma = M0 if sma is None else sma
    w = (F + 3) // 4 * 4
    _abi.call("gala_gat_fwd_continue_f32", g.csr(2 * w + 3 * heads if Um0 is not None else w + 2 * heads),
              _dp(aL), _dp(aR), _dp(wR), _dp(bR), _dp(X), X.stride(0), F, heads, slope,
              _abi.GALA_GAT_PARTIAL if partial else 0, _dp(U0), U0.stride(0),
              _dp(S0), _dp(Um0), Um0.stride(0) if Um0 is not None else 0, _dp(M0), _dp(Y), Y.stride(0), _dp(q),
              _dp(Ym), Ym.stride(0) if Ym is not None else 0, _dp(sma), _stream())
    return (Y, q) if Um0 is None else (Y, q, Ym, sma)


def gat_bwd_stats(g: DeviceGraph, aL, aR, dY, q, Y, Ym, sma, heads=1, slope=0.2, p=None, dY_rows=None, wR=None):
    """gala_gat_bwd_stats_f32 (REF): (dX, d_aL) from the forward's row statistics; gathers
    dY[col] only (alpha from aR, or from the forward's p when given).  dY_rows: dY is a
    gathered table and dY_rows the rows' own dY (gala_gat_bwd_stats_ex_f32).  wR: dX also
    takes the source logit's per-head Linear, d_aL * wR (gala_gat_bwd_stats_linear_f32)."""
    F = dY.shape[1]
    dX = _rows_like(dY, g.n_rows)
    d_aL = torch.empty(g.n_rows * heads, device=dY.device, dtype=torch.float32)
    if wR is not None:
        _abi.call("gala_gat_bwd_stats_linear_f32", g.csr((F + 3) // 4 * 4), _dp(aL), _dp(aR), _dp(p), _dp(dY),
                  dY.stride(0), _dp(dY_rows), F, heads, slope, _dp(q), _dp(Y), Y.stride(0), _dp(Ym), Ym.stride(0),
                  _dp(sma), _dp(wR), _dp(dX), dX.stride(0), _dp(d_aL), _stream())
        return dX, d_aL
    if dY_rows is not None:
        _abi.call("gala_gat_bwd_stats_ex_f32", g.csr((F + 3) // 4 * 4), _dp(aL), _dp(aR), _dp(p), _dp(dY),
                  dY.stride(0), _dp(dY_rows), F, heads, slope, _dp(q), _dp(Y), Y.stride(0), _dp(Ym), Ym.stride(0),
                  _dp(sma), _dp(dX), dX.stride(0), _dp(d_aL), _stream())
        return dX, d_aL
    _abi.call("gala_gat_bwd_stats_f32", g.csr((F + 3) // 4 * 4), _dp(aL), _dp(aR), _dp(p), _dp(dY), dY.stride(0), F,
              heads, slope, _dp(q), _dp(Y), Y.stride(0), _dp(Ym), Ym.stride(0), _dp(sma), _dp(dX), dX.stride(0),
              _dp(d_aL), _stream())
    return dX, d_aL


def head_attn(X, w, b=None, heads=1):
    """gala_head_attn_f32: out[r, h] = <X[r, head h], w[head h]> + b[h] ([N, heads])."""
    N, F = X.shape
    out = torch.empty((N, heads), device=X.device, dtype=torch.float32)
    _abi.call("gala_head_attn_f32", N, F, heads, _dp(X), X.stride(0), _dp(w), _dp(b), _dp(out), _stream())
    return out


def head_attn_bwd(g, w, heads=1, dX=None, n_rows=None):
    """gala_head_attn_bwd_f32: dX[r, head h] (+)= g[r, h] * w[head h] (accumulates into dX
    when given)."""
    F = w.numel()
    N = g.numel() // heads if n_rows is None else n_rows
    acc = dX is not None
    if dX is None:
        dX = torch.empty((N, F), device=g.device, dtype=torch.float32)
    _abi.call("gala_head_attn_bwd_f32", N, F, heads, _dp(g), _dp(w), _dp(dX), dX.stride(0), int(acc), _stream())
    return dX


def edge_permute(perm, src, heads=1):
    n = perm.numel()
    dst = torch.empty(n * heads, device=src.device, dtype=torch.float32)
    _abi.call("gala_edge_permute_f32", _dp(perm), _dp(src), n, heads, _dp(dst), _stream())
    return dst


def ffn_fwd(X, W, b=None, out=None):
    """Y = X W^T + b on the matrix cores (gala_ffn_fwd_f32; W^T must fit 24K floats)."""
    X = X if X.stride(1) == 1 else X.contiguous()
    W = W.contiguous()
    N, K = X.shape
    M = W.shape[0]
    if out is None:
        out = torch.empty((N, M), device=X.device, dtype=torch.float32)
    _abi.call("gala_ffn_fwd_f32", N, K, M, _dp(X), max(X.stride(0), K), _dp(W), _dp(b), _dp(out),
              out.stride(0), _stream())
    return out


def dense_grad(X, dY, bias=True, dW=None, db=None, accumulate=False):
    """FFN weight / bias gradients dW = dY^T X [M, K], db = dY.sum(0) (gala_dense_grad_f32)."""
    # row strides pass through (row-padded views included); columns must be unit-stride
    X = X if X.stride(1) == 1 else X.contiguous()
    dY = dY if dY.stride(1) == 1 else dY.contiguous()
    N, K = X.shape
    M = dY.shape[1]
    if dW is None:
        dW = torch.empty(M, K, device=X.device, dtype=torch.float32)
    if bias and db is None:
        db = torch.empty(M, device=X.device, dtype=torch.float32)
    wsb = _abi.lib().gala_dense_grad_workspace(N, K, M)
    ws = torch.empty(max(wsb // 4, 1), device=X.device, dtype=torch.float32)
    ldx, ldy = max(X.stride(0), K), max(dY.stride(0), M)  # (empty tensors report any stride)
    _abi.call("gala_dense_grad_f32", N, K, M, _dp(X), ldx, _dp(dY), ldy, _dp(dW),
              _dp(db) if bias else None, int(accumulate), _dp(ws), wsb, _stream())
    return (dW, db) if bias else dW


# ---- the multi-head GAT layer in input space (gala_gat_in_*) ------------------------------
def gat_in_compose(W, b, wL, bL, wR, bR, heads):
    """The attention vectors folded through the Linear: u [2H, fin] (uL_h = W_h^T wL_h, then
    uR) and c [2H] (cL_h = b_h . wL_h + bL_h, then cR) -- the mirror's GatInputLayer spelling."""
    F, fin = W.shape
    H, D = heads, F // heads
    w3 = W.reshape(H, D, fin)
    bb = b.reshape(H, D) if b is not None else torch.zeros(H, D, device=W.device)
    uL, uR = (w3 * wL.reshape(H, D, 1)).sum(1), (w3 * wR.reshape(H, D, 1)).sum(1)
    cL, cR = (bb * wL.reshape(H, D)).sum(1) + bL.reshape(H), (bb * wR.reshape(H, D)).sum(1) + bR.reshape(H)
    return torch.cat([uL, uR]).contiguous(), torch.cat([cL, cR]).contiguous()


def gat_in_prep(X, u, c, heads, xext=None):
    """gala_gat_in_prep_f32: the extended rows [N, 128] (features, ones, aR, aL)."""
    N, fin = X.shape
    xext = torch.empty(N, 128, device=X.device, dtype=torch.float32) if xext is None else xext
    _abi.call("gala_gat_in_prep_f32", N, fin, _dp(X), X.stride(0), heads, _dp(u), _dp(c), _dp(xext), _stream())
    return xext


def gat_in_fwd(g: DeviceGraph, xext, W, b, heads, fin, slope=0.2, order=None, relu=False, T=None):
    """gala_gat_in_fwd_f32: (Y, Ym, q, sma); writes q into xext.  order: int32 row order.
    T ([N, 896], symmetric g only): gala_gat_in_fwd_t_f32, which also forms the backward's
    per-column aggregates there."""
    F = W.shape[0]
    D = F // heads
    Y = torch.empty(g.n_rows, F, device=W.device, dtype=torch.float32)
    Ym = torch.empty_like(Y)
    q = torch.empty(g.n_rows, heads, device=W.device, dtype=torch.float32)
    sma = torch.empty_like(q)
    flags = _abi.GALA_GAT_IN_RELU if relu else 0
    if T is None:
        _abi.call("gala_gat_in_fwd_f32", g.csr(0), _dp(order), fin, heads, D, slope, _dp(xext), _dp(W), W.stride(0),
                  _dp(b), _dp(Y), _dp(Ym), F, _dp(q), _dp(sma), flags, _stream())
    else:
        _abi.call("gala_gat_in_fwd_t_f32", g.csr(0), _dp(order), fin, heads, D, slope, _dp(xext), _dp(W),
                  W.stride(0), _dp(b), _dp(Y), _dp(Ym), F, _dp(q), _dp(sma), flags, _dp(T), _stream())
    return Y, Ym, q, sma


def gat_in_bwd(gT: DeviceGraph, xext, dY, Y, Ym, sma, heads, fin, slope=0.2, order=None, relu=False, T=None):
    """gala_gat_in_bwd_f32 over the transposed pattern gT: (d_aL [N, H], M [H, D, fin + 1]);
    with T (the T-mode forward's), gala_gat_in_bwd_t_f32 (no walk over the pattern)."""
    F = dY.shape[1]
    D = F // heads
    n = dY.shape[0]
    daL = torch.empty(n, heads, device=dY.device, dtype=torch.float32)
    M = torch.empty(heads, D, fin + 1, device=dY.device, dtype=torch.float32)
    wsb = _abi.lib().gala_gat_in_bwd_workspace(heads)
    ws = torch.empty(max(wsb // 4, 1), device=dY.device, dtype=torch.float32)
    flags = _abi.GALA_GAT_IN_RELU if relu else 0
    if T is None:
        _abi.call("gala_gat_in_bwd_f32", gT.csr(0), _dp(order), fin, heads, D, slope, _dp(xext), _dp(dY), _dp(Y),
                  _dp(Ym), F, _dp(sma), _dp(daL), _dp(M), _dp(ws), wsb, flags, _stream())
    else:
        _abi.call("gala_gat_in_bwd_t_f32", n, _dp(order), fin, heads, D, _dp(T), _dp(dY), _dp(Y), _dp(Ym), F,
                  _dp(sma), _dp(daL), _dp(M), _dp(ws), wsb, flags, _stream())
    return daL, M


def degree_order(rowptr):
    """Rows by descending degree (gala_host_row_order), int32 on the host."""
    rp = np.ascontiguousarray(rowptr, np.int32)
    order = np.empty(len(rp) - 1, np.int32)
    _abi.call("gala_host_row_order", len(order), rp.ctypes.data, order.ctypes.data)
    return order


def gat_input_layer(g: DeviceGraph, X, W, b, wL, bL, wR, bR, heads, slope=0.2, dY=None, gT=None, order=None,
                    order_t=None, relu=False, tmode=False):
    """Config 3's layer 1 in input space through the C ABI, the composition of the mirror's
    GatInputLayer: forward (Y, q, sma, xext) and, with dY, the gradients
    {W, b, wL, bL, wR, bR} (REF: d aR = d aL) and d_aL.  gT: the transposed pattern (default g,
    the symmetric graph of an undirected program)."""
    F, fin = W.shape
    H, D = heads, F // heads
    u, c = gat_in_compose(W, b, wL, bL, wR, bR, heads)
    xext = gat_in_prep(X, u, c, heads)
    # T mode (tmode, the symmetric g of an undirected program: gT None): the forward also forms
    # the backward's per-column aggregates
    T = torch.empty(g.n_rows, 896, device=X.device, dtype=torch.float32) if tmode and gT is None else None
    Y, Ym, q, sma = gat_in_fwd(g, xext, W, b, heads, fin, slope, order=order, relu=relu, T=T)
    out = {"Y": Y, "Ym": Ym, "q": q, "sma": sma, "xext": xext, "T": T}
    if dY is None:
        return out
    daL, M = gat_in_bwd(g if gT is None else gT, xext, dY, Y, Ym, sma, heads, fin, slope,
                        order=order if gT is None else order_t, relu=relu, T=T)
    Gw, Gb = dense_grad(X, daL)
    sLR = wL.reshape(H, D) + wR.reshape(H, D)
    bb = b.reshape(H, D) if b is not None else torch.zeros(H, D, device=W.device)
    dw = (W.reshape(H, D, fin) * Gw.unsqueeze(1)).sum(2) + bb * Gb.unsqueeze(1)
    out.update(daL=daL, M=M, G=Gw, dW=(M[:, :, :fin] + sLR.unsqueeze(2) * Gw.unsqueeze(1)).reshape(F, fin),
               db=(M[:, :, fin] + sLR * Gb.unsqueeze(1)).reshape(F), dwL=dw.reshape(-1), dwR=dw.reshape(-1),
               dbL=Gb, dbR=Gb)
    return out
