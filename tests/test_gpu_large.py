"""GPU: the 64-bit address path (SURVEY §7 hard part 3: the reference's `row*dcols` is 32-bit
int, cuda.h:309-310, and overflows once N*F >= 2^31 -- ogbn-papers100M at F = 128 is 1.4e10).

* A 17.2 M-row uniform graph at F = 128: X and Y hold 2.2e9 floats each, so every row past
  16.8 M addresses beyond 2^31 elements.  Integer-valued features make the per-row sums
  exact, so 3000 sampled rows (half of them past the 2^31 boundary) must equal a float64
  gather of their neighbours bit for bit, and so must the degree pass.
* Sizes past the int32 index contract are refused with GALA_ERR_UNSUPPORTED before any
  memory is touched (csrc/abi.cpp check_csr), never wrapped.
"""
import ctypes

import numpy as np
import pytest
import torch

from gala import _abi, layout, ops

pytestmark = pytest.mark.gpu


def test_spmm_rows_past_2pow31_elements():
    n, F = 17_200_000, 128
    assert n * F > 2 ** 31
    g = layout.gen_graph("uniform", n, 12_000_000, seed=5)       # E = 41.2 M incl. self loops
    dg = ops.DeviceGraph.from_host(g)
    gen = torch.Generator(device="cuda").manual_seed(7)
    X = torch.randint(-8, 9, (n, F), device="cuda", generator=gen, dtype=torch.int32).float()
    Y = ops.spmm(dg, X)
    deg = ops.degree(dg)
    torch.cuda.synchronize()
    rng = np.random.default_rng(3)
    boundary = (2 ** 31) // F                                    # first row past 2^31 elements
    rows = np.concatenate([rng.integers(0, boundary, 1500), rng.integers(boundary, n, 1500), [n - 1]])
    starts, ends = g.rowptr[rows].astype(np.int64), g.rowptr[rows + 1].astype(np.int64)
    cols = np.concatenate([g.col[s:e] for s, e in zip(starts, ends)]).astype(np.int64)
    Xn = X[torch.from_numpy(cols).cuda()].double().cpu().numpy()
    seg = np.repeat(np.arange(rows.shape[0]), ends - starts)
    ref = np.zeros((rows.shape[0], F))
    np.add.at(ref, seg, Xn)
    got = Y[torch.from_numpy(rows).cuda()].double().cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(deg[torch.from_numpy(rows).cuda()].cpu().numpy(), (ends - starts).astype(np.float32))


def _csr(n_rows, n_cols, nnz):
    c = _abi.gala_csr_t()
    c.n_rows, c.n_cols, c.nnz = n_rows, n_cols, nnz
    c.rowptr, c.col = 0x1000, 0x2000      # never dereferenced: validation refuses first
    c.val, c.val_heads, c.n_seg, c.seg_bounds, c.split, c.val_row_scale = None, 1, 1, None, None, None
    return c


@pytest.mark.parametrize("shape", [(1000, 1000, 2 ** 31), (2 ** 31 - 1, 1000, 10), (1000, 2 ** 31, 10)])
def test_sizes_beyond_int32_are_refused(shape):
    c = _csr(*shape)
    L = _abi.lib()
    st = L.gala_spmm_f32(ctypes.byref(c), 0x3000, 32, 0x4000, 32, 32, None, None, 0, 0, 5, 7, None)
    assert st == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_degree_f32(ctypes.byref(c), 0x4000, 1.0, 0, 0, None) == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_gat_fwd_ex_f32(ctypes.byref(c), 0x1, 0x2, None, None, 0x3, 32, 32, 1, 0.2, 0, 0x4, 32,
                                 None, None, None) == _abi.GALA_ERR_UNSUPPORTED
