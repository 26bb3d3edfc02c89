"""CPU: libgala_hip.so loads, exports every entry point include/gala_hip.h declares, and
validates arguments without touching a GPU; the host-side builders are deterministic."""
import ctypes
import os
import re

import numpy as np
import pytest

from gala import _abi, layout
from _graphs import long_row_graph

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gala_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(gala_\w+)\s*\(", text, re.M)))


def test_header_parses():
    syms = declared_symbols()
    assert "gala_spmm_f32" in syms and "gala_host_csr_build" in syms
    assert len(syms) >= 20


def test_library_exports_every_declared_symbol():
    L = _abi.lib()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_ctypes_signatures_cover_header():
    assert set(declared_symbols()) == set(_abi.SIGNATURES)


def test_nm_exports():
    out = os.popen(f"nm -D --defined-only {_abi.LIB_PATH}").read()
    for s in declared_symbols():
        assert re.search(rf"\bT {s}$", out, re.M), s


def test_version_and_status_strings():
    L = _abi.lib()
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "gala_hip.h")).read()
    declared = int(re.search(r"#define GALA_ABI_VERSION (\d+)", hdr).group(1))
    assert L.gala_abi_version() == declared == _abi.ABI_VERSION == 6
    assert L.gala_status_string(0) == b"GALA_OK"
    assert L.gala_status_string(-4) == b"GALA_ERR_GRAPH"


def test_invalid_arguments_rejected_without_gpu():
    L = _abi.lib()
    assert L.gala_spmm_f32(None, None, 0, None, 0, 0, None, None, 0, 0, 0, 0, None) == _abi.GALA_ERR_INVALID_ARG
    c = _abi.gala_csr_t()
    c.n_rows, c.n_cols, c.nnz, c.n_seg = 4, 4, 0, 0  # n_seg 0 invalid
    assert L.gala_spmm_f32(ctypes.byref(c), None, 8, None, 8, 8, None, None, 0, 0, 0, 0, None) == _abi.GALA_ERR_INVALID_ARG
    c.n_seg = 2  # tiled without host bounds
    assert L.gala_degree_f32(ctypes.byref(c), None, 1.0, 0, 0, None) == _abi.GALA_ERR_INVALID_ARG
    c.n_seg = 1
    c.n_rows = 0  # empty graph: nothing to launch, OK even without a device
    assert L.gala_spmm_f32(ctypes.byref(c), None, 8, None, 8, 8, None, None, 0, 0, 0, 0, None) == 0
    assert L.gala_sddvv_f32(ctypes.byref(c), None, None, 1, 7, 0.2, None, None) == _abi.GALA_ERR_INVALID_ARG
    assert L.gala_edge_softmax_fwd_f32(ctypes.byref(c), None, 1, 5, None, None) == _abi.GALA_ERR_INVALID_ARG


def test_host_builders_reject_bad_graphs():
    with pytest.raises(_abi.GalaError):
        layout.csr_build(3, 3, np.array([0, 5], np.int32), np.array([1, 1], np.int32))
    with pytest.raises(_abi.GalaError):
        layout.csr_build(3, 3, np.array([0, 1], np.int32), np.array([1, 3], np.int32))
    g = layout.csr_build(4, 4, np.array([0, 1], np.int32), np.array([1, 2], np.int32))
    with pytest.raises(_abi.GalaError):  # row 2 has degree 0: the reference divides by zero
        layout.sample_ab(g, 3)


def test_generator_deterministic_and_symmetric():
    a = layout.gen_graph("uniform", 3000, 9000, seed=5)
    b = layout.gen_graph("uniform", 3000, 9000, seed=5)
    np.testing.assert_array_equal(a.rowptr, b.rowptr)
    np.testing.assert_array_equal(a.col, b.col)
    assert a.nnz == 2 * 9000 + 3000
    t, _ = layout.transpose(a)  # symmetric: A^T == A
    np.testing.assert_array_equal(t.rowptr, a.rowptr)
    np.testing.assert_array_equal(t.col, a.col)
    r = layout.gen_graph("rmat", 4096, 20000, seed=1)
    deg = r.degrees()
    assert deg.max() > 20 * np.median(deg)  # skewed
    for n in (3000, 5_000_000):             # banded: |u - v| <= min(8192, max(16, n / 256))
        band = min(8192, max(16, n // 256))
        bg = layout.gen_graph("banded", n, 4 * n if n < 10000 else 200_000, seed=2)
        rows = np.repeat(np.arange(n), np.diff(bg.rowptr))
        assert np.abs(rows - bg.col).max() <= band and bg.nnz == 2 * (4 * n if n < 10000 else 200_000) + n
        t, _ = layout.transpose(bg)
        np.testing.assert_array_equal(t.col, bg.col)


def test_transpose_roundtrip():
    rng = np.random.default_rng(0)
    src = rng.integers(0, 50, 400).astype(np.int32)
    dst = rng.integers(0, 70, 400).astype(np.int32)
    g = layout.csr_build(50, 70, src, dst)
    t, perm = layout.transpose(g)
    assert t.n_rows == 70 and t.n_cols == 50
    tt, perm2 = layout.transpose(t)
    np.testing.assert_array_equal(tt.rowptr, g.rowptr)
    np.testing.assert_array_equal(tt.col, g.col)
    rows = np.repeat(np.arange(50), np.diff(g.rowptr))
    np.testing.assert_array_equal(t.col, rows[perm])


def test_col_tile_large_segment_count_and_breakpoints():
    g = layout.gen_graph("uniform", 1000, 4000, seed=2)
    bp = layout.col_breakpoints(1000, 64)
    assert bp[0] == 0 and bp[-1] == 1000 and len(bp) == 17
    t = layout.col_tile(g, 64)
    assert t.n_seg == 16 and t.bounds[-1] == g.nnz
    rp = t.rowptr.reshape(t.n_seg, g.n_rows + 1)
    np.testing.assert_array_equal((rp[:, 1:] - rp[:, :-1]).sum(0), g.degrees())


def test_row_order_exact_above_the_counting_cap():
    """gala_host_row_order: non-increasing degree over the whole order (rows past the 4096
    counting-sort cap sorted exactly, ties by row id), so the rows above any hub threshold
    are exactly its first entries (the REF-order hub kernel's contract)."""
    g = long_row_graph()
    order = np.empty(g.n_rows, np.int32)
    _abi.call("gala_host_row_order", g.n_rows, g.rowptr.ctypes.data, order.ctypes.data)
    deg = np.diff(g.rowptr)
    assert sorted(order.tolist()) == list(range(g.n_rows))
    np.testing.assert_array_equal(order, np.lexsort((np.arange(g.n_rows), -deg)))
    thr = layout.split_threshold(g.n_rows, g.nnz)
    assert thr > 4500 and (deg > thr).sum() == 3
    assert set(order[:3].tolist()) == set(np.flatnonzero(deg > thr).tolist())
