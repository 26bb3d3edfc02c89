"""TEST INFRASTRUCTURE ONLY — numpy/ctypes front of the C oracle (oracle/gala_oracle.c)
and of the reference harness (oracle/_ref/libgala_ref.so, built from /root/reference).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
the checker / CPU baseline.  Nothing in the product package imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(HERE, "_build", "liboracle.so")
_REF = os.path.join(HERE, "_ref", "libgala_ref.so")

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def build() -> None:
    """Compile the oracle (and the reference harness when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "_build/liboracle.so"], check=True)
    subprocess.run([os.path.join(HERE, "build_ref.sh")], check=True)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.run(["make", "-s", "-C", HERE, "_build/liboracle.so"], check=True)
        _lib = ctypes.CDLL(_LIB)
    return _lib


def ref_available() -> bool:
    return os.path.exists(_REF)


def ref():
    """The reference's own CPU code (compiled from /root/reference)."""
    global _ref
    if _ref is None:
        _ref = ctypes.CDLL(_REF)
    return _ref


@dataclass
class Graph:
    """CSR (n_seg == 1) or column-tiled (n_seg > 1) graph on the host."""

    n_rows: int
    n_cols: int
    rowptr: np.ndarray  # int32 [(n_rows+1)*n_seg]
    col: np.ndarray  # int32 [nnz]
    val: np.ndarray | None = None  # float32 [nnz*val_heads]
    n_seg: int = 1
    bounds: np.ndarray | None = None  # int32 [2*n_seg]
    val_heads: int = 1

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])

    @property
    def seg_base(self):
        return None if self.n_seg == 1 else np.ascontiguousarray(self.bounds[0::2], dtype=np.int32)


def _g(g: Graph):
    return (_i64(g.n_rows), _i32(g.n_seg), _ptr(g.rowptr), _ptr(g.seg_base))


def spmm(g: Graph, X, F=None, src_scale=None, dst_scale=None, Y=None, accum=False,
         sample=False, nsamp=0, ra=5, rb=7):
    X = np.ascontiguousarray(X, dtype=np.float32)
    F = X.shape[1] if F is None else F
    if Y is None:
        Y = np.zeros((g.n_rows, F), dtype=np.float32)
    L = lib()
    L.orc_spmm(*_g(g), _ptr(g.col), _ptr(g.val), _i32(g.val_heads), _ptr(X), _i64(X.shape[1]),
               _i32(F), _ptr(src_scale), _ptr(dst_scale), ctypes.c_int(int(accum)),
               ctypes.c_int(int(sample)), _i32(nsamp), _i32(ra), _i32(rb), _ptr(Y),
               _i64(Y.shape[1]))
    return Y


def gspmm(g: Graph, X):
    X = np.ascontiguousarray(X, dtype=np.float32)
    Y = np.zeros((g.n_rows, X.shape[1]), dtype=np.float32)
    lib().orc_gspmm(_i64(g.n_rows), _ptr(g.rowptr), _ptr(g.col), _ptr(g.val), _ptr(X),
                    _i32(X.shape[1]), _ptr(Y))
    return Y


def degree(g: Graph, power=1.0, sample=False, nsamp=0):
    out = np.zeros(g.n_rows, dtype=np.float32)
    lib().orc_degree(*_g(g), _ptr(g.val), ctypes.c_float(power), ctypes.c_int(int(sample)),
                     _i32(nsamp), _ptr(out))
    return out


def sddvv(g: Graph, a, b, heads=1, op=0, slope=0.2):
    out = np.zeros(g.nnz * heads, dtype=np.float32)
    lib().orc_sddvv(*_g(g), _ptr(g.col), _ptr(np.ascontiguousarray(a, np.float32)),
                    _ptr(np.ascontiguousarray(b, np.float32)), _i32(heads), _i32(op),
                    ctypes.c_float(slope), _ptr(out))
    return out


def row_sum(g: Graph, v, heads=1, eps=1e-12, out=None, accum=False):
    if out is None:
        out = np.zeros(g.n_rows * heads, dtype=np.float32)
    lib().orc_row_sum(*_g(g), _ptr(np.ascontiguousarray(v, np.float32)), _i32(heads),
                      ctypes.c_float(eps), ctypes.c_int(int(accum)), _ptr(out))
    return out


def row_scale(g: Graph, q, v, heads=1):
    v = np.array(v, dtype=np.float32, copy=True)
    lib().orc_row_scale(*_g(g), _ptr(np.ascontiguousarray(q, np.float32)), _i32(heads), _ptr(v))
    return v


def sddmm(g: Graph, A, B, heads=1):
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    out = np.zeros(g.nnz * heads, dtype=np.float32)
    lib().orc_sddmm(*_g(g), _ptr(g.col), _ptr(A), _i64(A.shape[1]), _ptr(B), _i64(B.shape[1]),
                    _i32(A.shape[1]), _i32(heads), _ptr(out))
    return out


def softmax_fwd(g: Graph, logit, heads=1, mode=0):
    out = np.zeros(g.nnz * heads, dtype=np.float32)
    lib().orc_softmax_fwd(*_g(g), _ptr(np.ascontiguousarray(logit, np.float32)), _i32(heads),
                          ctypes.c_int(mode), _ptr(out))
    return out


def softmax_bwd(g: Graph, alpha, dalpha, heads=1, mode=0):
    out = np.zeros(g.nnz * heads, dtype=np.float32)
    lib().orc_softmax_bwd(*_g(g), _ptr(np.ascontiguousarray(alpha, np.float32)),
                          _ptr(np.ascontiguousarray(dalpha, np.float32)), _i32(heads),
                          ctypes.c_int(mode), _ptr(out))
    return out


def gat_fwd(g: Graph, aL, aR, X, heads=1, slope=0.2, mode=0):
    """Reference GAT layer forward: edge_sddvv -> LeakyReLU -> softmax ->
    weighted aggregation, composed from the restated kernels."""
    s = sddvv(g, aL, aR, heads=heads, op=2, slope=slope)
    alpha = softmax_fwd(g, s, heads=heads, mode=mode)
    gw = Graph(g.n_rows, g.n_cols, g.rowptr, g.col, alpha, g.n_seg, g.bounds, heads)
    return spmm(gw, X), alpha


def gat_bwd(g: Graph, aL, aR, X, dY, alpha, heads=1, slope=0.2, mode=0):
    """Reference GAT edge backward on one pattern, composed from the restated kernels:
    edge_sddmm (cuda.h:808-845) -> softmax backward (common.h:791-799) -> LeakyReLU
    backward (torch where(z > 0, ds, ds*slope) on z = aL[row]+aR[col], common.h:1175-1184)
    -> node_spmv_backward_of_sddmm row sum (cuda.h:505-524; eps 1e-12 in REF mode).
    Returns (dz per (edge, head), d_aL [n_rows*heads])."""
    dalpha = sddmm(g, dY, X, heads=heads)
    ds = softmax_bwd(g, alpha, dalpha, heads=heads, mode=mode)
    z = sddvv(g, aL, aR, heads=heads, op=0)
    dz = np.where(z > 0, ds, (ds * np.float32(slope)).astype(np.float32)).astype(np.float32)
    daL = row_sum(g, dz, heads=heads, eps=1e-12 if mode == 0 else 0.0)
    return dz, daL


def set_threads(n: int) -> None:
    lib().orc_set_threads(ctypes.c_int(int(n)))


def head_attn(X, wR, bR, heads, r0=0, r1=None, aR=None):
    """aR[r, h] = <X[r, head h], wR_h> + bR_h for rows [r0, r1) (attnR = efc(res) per head)."""
    X = np.ascontiguousarray(X, np.float32)
    r1 = X.shape[0] if r1 is None else r1
    if aR is None:
        aR = np.zeros((X.shape[0], heads), np.float32)
    lib().orc_head_attn(_i64(r0), _i64(r1), _ptr(X), _i64(X.shape[1]), _i32(heads),
                        _i32(X.shape[1] // heads), _ptr(np.ascontiguousarray(wR, np.float32)),
                        _ptr(None if bR is None else np.ascontiguousarray(bR, np.float32)), _ptr(aR))
    return aR


class GatRefLayer:
    """CPU baseline of the SDDMM + edge-softmax half (orc_gat_ref_layer): one REF GAT layer,
    forward + backward, pass by pass as the generated program composes it, over the rows
    [0, n_rows) of a CSR graph (a row sample of it when n_rows < the graph's).  Buffers are
    allocated (and prefaulted) once here; run() touches only them."""

    def __init__(self, rowptr, col, n_rows, X, dY, aL, wR, bR, heads, slope=0.2, row_ids=None, aR=None):
        """row_ids: row r of (rowptr, col) is the layer's row row_ids[r] of a larger graph
        (aL and the row side of dY are read there; columns stay global; outputs at r).
        aR: the source logits [rows, heads] to use (with row_ids; otherwise head_attn's)."""
        self.rid = None if row_ids is None else np.ascontiguousarray(row_ids, np.int64)
        self.rowptr = np.ascontiguousarray(rowptr, np.int32)
        self.col = np.ascontiguousarray(col, np.int32)
        self.n_rows, self.H = int(n_rows), int(heads)
        self.X = np.ascontiguousarray(X, np.float32)
        self.dY = np.ascontiguousarray(dY, np.float32)
        self.aL = np.ascontiguousarray(aL, np.float32)
        self.wR = np.ascontiguousarray(wR, np.float32)
        self.bR = None if bR is None else np.ascontiguousarray(bR, np.float32)
        self.F = self.X.shape[1]
        self.slope = slope
        ne = int(self.rowptr[self.n_rows]) * self.H
        self.nnz = int(self.rowptr[self.n_rows])
        # attention logits of every source row; run() recomputes rows [0, n_rows) itself
        # (unless row_ids is given)
        self.aR = (head_attn(self.X, self.wR, self.bR, self.H) if aR is None
                   else np.ascontiguousarray(aR, np.float32).reshape(-1, self.H))
        assert aR is None or self.rid is not None, "aR is used as given only with row_ids"
        self.s, self.pa, self.da, self.res = (np.ones(ne, np.float32) for _ in range(4))
        self.q = np.ones((self.n_rows, self.H), np.float32)
        self.daL = np.ones((self.n_rows, self.H), np.float32)
        self.Y = np.ones((self.n_rows, self.F), np.float32)
        self.dX = np.ones((self.n_rows, self.F), np.float32)

    def run(self):
        args = (_i64(self.n_rows), _ptr(self.rowptr), _ptr(self.col), _i32(self.H),
                _i32(self.F // self.H), _ptr(self.aL), _ptr(self.X), _ptr(self.wR),
                _ptr(self.bR), _ptr(self.dY), ctypes.c_float(self.slope), _ptr(self.aR),
                _ptr(self.s), _ptr(self.pa), _ptr(self.da), _ptr(self.res), _ptr(self.q),
                _ptr(self.Y), _ptr(self.dX), _ptr(self.daL))
        if self.rid is None:
            lib().orc_gat_ref_layer(*args)
        else:
            lib().orc_gat_ref_layer_rows(*args, _ptr(self.rid))
        return self


def usable_cores() -> dict:
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota when
    one is set (a container's share can be far below the machine's CPU count)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return {"affinity_cpus": aff, "cgroup_cpu_limit": quota,
            "threads": min(aff, quota) if quota else aff}


def csr_build(n_rows, src, dst):
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    rowptr = np.zeros(n_rows + 1, np.int32)
    col = np.zeros(src.shape[0], np.int32)
    rc = lib().orc_csr_build(_i64(n_rows), _i64(src.shape[0]), _ptr(src), _ptr(dst), _ptr(rowptr),
                             _ptr(col))
    assert rc == 0
    return rowptr, col


def col_tile(g: Graph, cols_per_partition):
    S = (g.n_cols + cols_per_partition - 1) // cols_per_partition
    rp = np.zeros((g.n_rows + 1) * max(S, 1), np.int32)
    col = np.zeros(g.nnz, np.int32)
    val = np.zeros(g.nnz, np.float32)
    bounds = np.zeros(2 * max(S, 1), np.int32)
    n = lib().orc_col_tile(_i64(g.n_rows), _i64(g.n_cols), _ptr(g.rowptr), _ptr(g.col),
                           _ptr(g.val), _i32(cols_per_partition), _ptr(rp), _ptr(col), _ptr(val),
                           _ptr(bounds))
    assert n == S
    return Graph(g.n_rows, g.n_cols, rp, col, val, S, bounds)


def sample_ab(g: Graph, nsamp, ra=5, rb=7):
    rp = np.zeros(g.n_rows + 1, np.int32)
    col = np.zeros(g.n_rows * nsamp, np.int32)
    val = np.zeros(g.n_rows * nsamp, np.float32)
    rc = lib().orc_sample_ab(_i64(g.n_rows), _ptr(g.rowptr), _ptr(g.col), _ptr(g.val), _i32(nsamp),
                             _i32(ra), _i32(rb), _ptr(rp), _ptr(col), _ptr(val))
    assert rc == 0
    return Graph(g.n_rows, g.n_cols, rp, col, val)


def mask_subgraphs(g: Graph, mask, levels):
    """getMaskSubgraphs levels 0..levels-1 (tests/common.h:21-110)."""
    cur = np.ascontiguousarray(mask, np.int32)
    out = []
    for _ in range(levels):
        rp = np.zeros(g.n_rows + 1, np.int32)
        col = np.zeros(max(g.nnz, 1), np.int32)
        nxt = np.zeros(g.n_rows, np.int32)
        rc = lib().orc_mask_subgraph(_i64(g.n_rows), _ptr(g.rowptr), _ptr(g.col), _ptr(cur),
                                     _ptr(rp), _ptr(col), _ptr(nxt))
        assert rc == 0
        out.append(Graph(g.n_rows, g.n_cols, rp, col[: rp[-1]].copy(), None))
        cur = nxt
    return out


# ---- reference (compiled from /root/reference) ----------------------------------------
def ref_csr_build(n_rows, n_cols, src, dst):
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    rp = np.zeros(n_rows + 1, np.int32)
    col = np.zeros(src.shape[0], np.int32)
    val = np.zeros(src.shape[0], np.float32)
    ref().ref_csr_build(ctypes.c_int(n_rows), ctypes.c_int(n_cols), ctypes.c_int(src.shape[0]),
                        _ptr(src), _ptr(dst), _ptr(rp), _ptr(col), _ptr(val))
    return rp, col, val


def ref_read_mtx(path, cap):
    """The reference's MtxIO::readMtx (src/utils/mtx_io.h:199-499): (n_rows, n_cols, rows,
    cols, vals or None) of the COO entries in file order, mirrors included."""
    rows = np.zeros(cap, np.int32)
    cols = np.zeros(cap, np.int32)
    vals = np.zeros(cap, np.float32)
    nr, nc, nv = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    st = ref().ref_read_mtx(str(path).encode(), ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(nv), _ptr(rows),
                            _ptr(cols), _ptr(vals), ctypes.c_int64(cap))
    if st < 0:
        raise RuntimeError(f"ref_read_mtx: {st}")
    n = nv.value
    return nr.value, nc.value, rows[:n], cols[:n], (vals[:n] if st == 1 else None)


def ref_read_mtx_dense(path, cap):
    """The reference's MtxIO on a dense "array" file (readDM without RNPY): float32 [r, c]."""
    out = np.zeros(cap, np.float32)
    nr, nc = ctypes.c_int64(), ctypes.c_int64()
    st = ref().ref_read_mtx_dense(str(path).encode(), ctypes.byref(nr), ctypes.byref(nc), _ptr(out),
                                  ctypes.c_int64(cap))
    if st < 0:
        raise RuntimeError(f"ref_read_mtx_dense: {st}")
    return out[:nr.value * nc.value].reshape(nr.value, nc.value)


def ref_read_sm_mtx(path, n_rows, cap):
    """The reference's readSM (src/utils/common.h:397-416): MtxIO -> CSRCMatrix::build(CSR);
    (rowptr, col, val or None)."""
    rp = np.zeros(n_rows + 1, np.int32)
    col = np.zeros(cap, np.int32)
    val = np.zeros(cap, np.float32)
    st = ref().ref_read_sm_mtx(str(path).encode(), _ptr(rp), _ptr(col), _ptr(val), ctypes.c_int64(n_rows + 1),
                               ctypes.c_int64(cap))
    if st < 0:
        raise RuntimeError(f"ref_read_sm_mtx: {st}")
    n = int(rp[-1])
    return rp, col[:n], (val[:n] if st == 1 else None)


def ref_gspmm(g: Graph, X, Y=None):
    X = np.ascontiguousarray(X, np.float32)
    val = g.val if g.val is not None else np.ones(g.nnz, np.float32)
    if Y is None:
        Y = np.zeros((g.n_rows, X.shape[1]), np.float32)
    ref().ref_gspmm(ctypes.c_int(g.n_rows), ctypes.c_int(g.n_cols), ctypes.c_int(g.nnz),
                    _ptr(g.rowptr), _ptr(g.col), _ptr(val), _ptr(X), ctypes.c_int(X.shape[1]),
                    _ptr(Y))
    return Y


def ref_col_tile(g: Graph, cols_per_partition, max_seg=4096):
    S = (g.n_cols + cols_per_partition - 1) // cols_per_partition
    val = g.val if g.val is not None else np.ones(g.nnz, np.float32)
    rp = np.zeros((g.n_rows + 1) * max(S, 1), np.int32)
    col = np.zeros(g.nnz, np.int32)
    oval = np.zeros(g.nnz, np.float32)
    bounds = np.zeros(2 * max(S, 1), np.int32)
    n = ref().ref_col_tile(ctypes.c_int(g.n_rows), ctypes.c_int(g.n_cols), ctypes.c_int(g.nnz),
                           _ptr(g.rowptr), _ptr(g.col), _ptr(val), ctypes.c_int(cols_per_partition),
                           ctypes.c_int(max_seg), _ptr(rp), _ptr(col), _ptr(oval), _ptr(bounds))
    assert n == S, (n, S)
    return Graph(g.n_rows, g.n_cols, rp, col, oval, S, bounds)


def ref_sample_ab(g: Graph, nsamp, ra=5, rb=7):
    val = g.val if g.val is not None else np.ones(g.nnz, np.float32)
    rp = np.zeros(g.n_rows + 1, np.int32)
    col = np.zeros(g.n_rows * nsamp, np.int32)
    oval = np.zeros(g.n_rows * nsamp, np.float32)
    ref().ref_sample_ab(ctypes.c_int(g.n_rows), ctypes.c_int(g.n_cols), ctypes.c_int(g.nnz),
                        _ptr(g.rowptr), _ptr(g.col), _ptr(val), ctypes.c_int(nsamp),
                        ctypes.c_int(ra), ctypes.c_int(rb), _ptr(rp), _ptr(col), _ptr(oval))
    return Graph(g.n_rows, g.n_cols, rp, col, oval)


def ref_mask_subgraphs(g: Graph, mask, levels):
    """Reference getMaskSubgraphs: [(fwd rowptr, fwd col, bwd rowptr, bwd col)] per level."""
    n, nnz = g.n_rows, g.nnz
    m = np.ascontiguousarray(mask, np.float32)
    rp = np.zeros(levels * (n + 1), np.int32)
    col = np.zeros(levels * max(nnz, 1), np.int32)
    nv = np.zeros(levels, np.int32)
    trp = np.zeros(levels * (n + 1), np.int32)
    tcol = np.zeros(levels * max(nnz, 1), np.int32)
    ref().ref_mask_subgraphs(ctypes.c_int(n), ctypes.c_int(nnz), _ptr(g.rowptr), _ptr(g.col),
                             _ptr(m), ctypes.c_int(levels), _ptr(rp), _ptr(col), _ptr(nv),
                             _ptr(trp), _ptr(tcol))
    out = []
    for l in range(levels):
        k = int(nv[l])
        out.append((rp[l * (n + 1):(l + 1) * (n + 1)].copy(), col[l * nnz:l * nnz + k].copy(),
                    trp[l * (n + 1):(l + 1) * (n + 1)].copy(), tcol[l * nnz:l * nnz + k].copy()))
    return out


def ref_threads() -> int:
    return int(ref().ref_omp_threads())


def ref_set_threads(n: int) -> None:
    ref().ref_set_threads(ctypes.c_int(int(n)))


def gat_input_layer_ref(rowptr, col, X, W, b, wL, bL, wR, bR, dY, heads, slope=0.2, threads=None, aL=None,
                        aR=None):
    """TEST INFRASTRUCTURE: config 3's first GAT layer as the reference's generated program
    composes it, with its REF backward -- the reference for the input-space layer
    (gala_gat_in_*):
      v1 = X W^T + b                          FFN_OP, torch::nn::Linear (common.h:1188-1242);
                                              fp32 result of a float64 product (the library
                                              GEMM's order is not pinned)
      aL = head_attn(v1, wL, bL)              attnL = ffn(res, out=1) per head (common.h:1248-1260)
      Y, dX_agg, d_aL = orc_gat_ref_layer     K5 ... K8 + aggregation, and its REF backward
                                              (common.h:735-894; aR recomputed from v1, d aR = d aL)
    and the parameter gradients autograd forms through those ops (float64 from the layer's
    fp32 outputs):
      dv1 = dX_agg + d_aL (x) (wL + wR) per head   (HeadAttn / the aR Linear's input gradient)
      dW = dv1^T X, db = sum dv1, d wL = d wR = sum_r d_aL[r, h] v1[r, head h], d bL = d bR = sum d_aL.
    aL / aR [n, heads] (optional): the attention logits to use instead of head_attn(v1) --
    the kernels' own, whose summation order differs from the Linear's: an edge whose logit
    sits at 0 may take the other LeakyReLU slope under a one-ulp change and move its row's
    d_aL by ~ alpha * |d alpha|; the tests check the logits themselves
    against the float64 Linear separately.
    Returns a dict of numpy arrays (Y, daL, aR, dW, db, dwL, dbL, dwR, dbR, v1)."""
    X = np.ascontiguousarray(X, np.float32)
    F, fin = W.shape
    H, D = heads, F // heads
    v1 = (X.astype(np.float64) @ np.asarray(W, np.float64).T + (0 if b is None else np.asarray(b, np.float64)))
    v1 = v1.astype(np.float32)
    aL = head_attn(v1, wL, bL, H) if aL is None else np.ascontiguousarray(aL, np.float32)
    n = len(rowptr) - 1
    if threads:
        set_threads(threads)
    rid = None if aR is None else np.arange(n, dtype=np.int64)
    lay = GatRefLayer(rowptr, col, n, v1, dY, aL, wR, bR, H, slope=slope, row_ids=rid, aR=aR).run()
    daL = lay.daL.astype(np.float64)
    sLR = (np.asarray(wL, np.float64) + np.asarray(wR, np.float64)).reshape(H, D)
    dv1 = lay.dX.astype(np.float64).reshape(n, H, D) + daL[:, :, None] * sLR[None]
    dv1 = dv1.reshape(n, F)
    dW = dv1.T @ X.astype(np.float64)
    db = dv1.sum(0)
    dw = np.einsum("rh,rhd->hd", daL, v1.astype(np.float64).reshape(n, H, D)).reshape(-1)
    return dict(Y=lay.Y, daL=lay.daL, aR=lay.aR, q=lay.q, dW=dW, db=db, dwL=dw, dbL=daL.sum(0), dwR=dw,
                dbR=daL.sum(0), v1=v1)
