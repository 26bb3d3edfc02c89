"""Host-side graph layout (numpy in, numpy out) through the C ABI's OpenMP builders.

Mirrors what the generated program does on the CPU before its H2D copies:
readSM_npy32 -> CSRCMatrix::build (tests/common.h:331-366, src/formats/csrc_matrix.h:148-376),
static_ord_col_breakpoints + ord_col_tiling_torch (src/ops/tiling.h:1594-1608, 222-283),
inplace_sample_graph_ab (src/ops/tiling.h:454-508).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import _abi


def _p(a):
    return None if a is None else a.ctypes.data


@dataclass
class HostGraph:
    n_rows: int
    n_cols: int
    rowptr: np.ndarray           # int32 [(n_rows+1)*n_seg]
    col: np.ndarray              # int32 [nnz]
    val: np.ndarray | None = None
    n_seg: int = 1
    bounds: np.ndarray | None = None  # int32 [2*n_seg] (host, like the reference)
    val_heads: int = 1

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])

    def degrees(self) -> np.ndarray:
        rp = self.rowptr.reshape(self.n_seg, self.n_rows + 1).astype(np.int64)
        return (rp[:, 1:] - rp[:, :-1]).sum(0)


def split_threshold(n_rows: int, nnz: int) -> int:
    """Hub-row threshold of a graph (gala_host_split_threshold: max(1024, 8*ceil(nnz/n))),
    the one definition shared with the C++ mirror and the partitioners."""
    t = int(_abi.lib().gala_host_split_threshold(int(n_rows), int(nnz)))
    _abi.check("gala_host_split_threshold", min(t, 0))
    return t


def csr_build(n_rows: int, n_cols: int, src, dst, return_perm: bool = False):
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    nnz = src.shape[0]
    rowptr = np.empty(n_rows + 1, np.int32)
    col = np.empty(nnz, np.int32)
    perm = np.empty(nnz, np.int32) if return_perm else None
    _abi.call("gala_host_csr_build", n_rows, n_cols, nnz, _p(src), _p(dst), _p(rowptr), _p(col),
              _p(perm))
    g = HostGraph(n_rows, n_cols, rowptr, col)
    return (g, perm) if return_perm else g


def col_breakpoints(n_cols: int, cols_per_partition: int) -> np.ndarray:
    cap = n_cols // max(cols_per_partition, 1) + 2
    out = np.empty(cap, np.int32)
    n = _abi.lib().gala_host_col_breakpoints(n_cols, cols_per_partition, _p(out), cap)
    _abi.check("gala_host_col_breakpoints", 0 if n > 0 else int(n))
    return out[:n].copy()


def col_tile(g: HostGraph, cols_per_partition: int) -> HostGraph:
    assert g.n_seg == 1
    bp = col_breakpoints(g.n_cols, cols_per_partition)
    S = bp.shape[0] - 1
    rp = np.empty((g.n_rows + 1) * S, np.int32)
    col = np.empty(g.nnz, np.int32)
    val = np.empty(g.nnz, np.float32) if g.val is not None else None
    bounds = np.empty(2 * S, np.int32)
    _abi.call("gala_host_col_tile", g.n_rows, _p(g.rowptr), _p(g.col), _p(g.val), S, _p(bp),
              _p(rp), _p(col), _p(val), _p(bounds))
    return HostGraph(g.n_rows, g.n_cols, rp, col, val, S, bounds, g.val_heads)


def sample_ab(g: HostGraph, nsamp: int, ra: int = 5, rb: int = 7) -> HostGraph:
    assert g.n_seg == 1
    rp = np.empty(g.n_rows + 1, np.int32)
    col = np.empty(g.n_rows * nsamp, np.int32)
    val = np.empty(g.n_rows * nsamp, np.float32) if g.val is not None else None
    _abi.call("gala_host_sample_ab", g.n_rows, _p(g.rowptr), _p(g.col), _p(g.val), nsamp, ra, rb,
              _p(rp), _p(col), _p(val))
    return HostGraph(g.n_rows, g.n_cols, rp, col, val)


def transpose(g: HostGraph):
    """CSR of A^T and perm (edge k of A^T is edge perm[k] of A)."""
    assert g.n_seg == 1
    rp = np.empty(g.n_cols + 1, np.int32)
    col = np.empty(g.nnz, np.int32)
    perm = np.empty(g.nnz, np.int32)
    _abi.call("gala_host_csr_transpose", g.n_rows, g.n_cols, _p(g.rowptr), _p(g.col), _p(rp),
              _p(col), _p(perm))
    val = g.val[perm] if g.val is not None else None
    return HostGraph(g.n_cols, g.n_rows, rp, col, val), perm


def mask_subgraphs(g: HostGraph, mask: np.ndarray, levels: int):
    """getMaskSubgraphs (tests/common.h:21-110): level l keeps the rows within l hops
    (through maxAgg over g) of the mask; returns [level 0, ..., level levels-1]."""
    assert g.n_seg == 1
    cur = np.ascontiguousarray(mask, dtype=np.int32)
    out = []
    for _ in range(levels):
        rp = np.empty(g.n_rows + 1, np.int32)
        _abi.call("gala_host_mask_subgraph", g.n_rows, _p(g.rowptr), _p(g.col), _p(cur), _p(rp),
                  None, None)
        col = np.empty(int(rp[-1]), np.int32)
        nxt = np.empty(g.n_rows, np.int32)
        _abi.call("gala_host_mask_subgraph", g.n_rows, _p(g.rowptr), _p(g.col), _p(cur), _p(rp),
                  _p(col), _p(nxt))
        out.append(HostGraph(g.n_rows, g.n_cols, rp, col))
        cur = nxt
    return out


def gen_graph(kind: str, n: int, n_undirected: int, seed: int = 42) -> HostGraph:
    """Deterministic synthetic graph: 'uniform' (random symmetric + self loops), 'rmat', or
    'banded' (every edge's ends at most min(8192, max(16, n/256)) ids apart)."""
    k = {"uniform": 0, "rmat": 1, "banded": 2}[kind]
    m = 2 * n_undirected + n
    src = np.empty(m, np.int32)
    dst = np.empty(m, np.int32)
    _abi.call("gala_host_gen_graph", k, n, n_undirected, seed, _p(src), _p(dst))
    return csr_build(n, n, src, dst)


MTX_FIELDS = ("pattern", "integer", "real", "double")
MTX_SYMMETRY = ("general", "symmetric", "skew-symmetric")


def mtx_info(path: str) -> dict:
    """Header of a Matrix Market file (gala_host_mtx_info)."""
    v = [ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()]
    _abi.call("gala_host_mtx_info", os.fsencode(path), *[ctypes.addressof(x) for x in v])
    return {"n_rows": v[0].value, "n_cols": v[1].value, "nnz": v[2].value, "field": MTX_FIELDS[v[3].value],
            "symmetry": MTX_SYMMETRY[v[4].value], "capacity": v[5].value}


def read_mtx_coo(path: str):
    """(info, rows, cols, vals) of a Matrix Market file: the reference's MtxIO entries
    (src/utils/mtx_io.h:199-499), 0-based, file order, (skew-)symmetric mirrors included;
    vals None for a pattern file."""
    info = mtx_info(path)
    cap = max(info["capacity"], 1)
    rows = np.empty(cap, np.int32)
    cols = np.empty(cap, np.int32)
    vals = np.empty(cap, np.float32)
    n = ctypes.c_int64()
    _abi.call("gala_host_mtx_read", os.fsencode(path), _p(rows), _p(cols), _p(vals), cap, ctypes.addressof(n))
    k = n.value
    return info, rows[:k], cols[:k], (None if info["field"] == "pattern" else vals[:k])


def load_mtx(path: str) -> HostGraph:
    """A Matrix Market graph as the reference's readSM builds it (src/utils/common.h:397-416:
    MtxIO entries -> CSRCMatrix::build(CSR), rows sorted, columns ascending, values carried;
    a pattern file has no values, i.e. an unweighted graph)."""
    info, rows, cols, vals = read_mtx_coo(path)
    g, perm = csr_build(info["n_rows"], info["n_cols"], rows, cols, return_perm=True)
    if vals is not None:
        g.val = np.ascontiguousarray(vals[perm])
    return g


def load_mtx_dense(path: str) -> np.ndarray:
    """A dense Matrix Market "array" file as float32 [rows, cols] (the reference's readDM
    without RNPY, src/utils/common.h:146-183: column-major entries placed row-major)."""
    nr, nc = ctypes.c_int64(), ctypes.c_int64()
    _abi.call("gala_host_mtx_dense_info", os.fsencode(path), ctypes.addressof(nr), ctypes.addressof(nc))
    out = np.empty((nr.value, nc.value), np.float32)
    k = ctypes.c_int64()
    _abi.call("gala_host_mtx_read_dense", os.fsencode(path), _p(out), nr.value, nc.value, ctypes.addressof(k))
    return out


def load_npy_dataset(path: str) -> HostGraph:
    """The reference's on-disk format (scripts/Data/gala_export_npy.py:104-171):
    Adj_src.npy = uint32 [nrows, ncols, src...], Adj_dst.npy = uint32 [dst...]."""
    src = np.load(os.path.join(path, "Adj_src.npy"))
    dst = np.load(os.path.join(path, "Adj_dst.npy"))
    n_rows, n_cols = int(src[0]), int(src[1])
    return csr_build(n_rows, n_cols, src[2:].astype(np.int32), dst.astype(np.int32))
