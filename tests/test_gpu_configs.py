"""GPU: the BASELINE configs at their own workload sizes, outputs checked against the oracle.

* config 2 -- ogbn-arxiv shape (N = 169 343, E = 1 335 586 stored edges), GCN-2 hidden 128:
  the step's four norm-scaled aggregations (degree, 2 forward, 2 backward; the fused step
  bench.py times), every output row bit-exact against the oracle's chain on the whole graph;
* config 3 -- ogbn-products shape (N = 2 449 029, E = 126 M), the 8-head GAT layer (F = 256,
  REF softmax, source logits recomputed from X): gala_gat_fwd_stats_f32 then
  gala_gat_bwd_stats_f32, Y, dX and d_aL of rows [0, k) against the oracle's pass-by-pass
  REF layer (orc_gat_ref_layer, the composition of the reference's K5-K9 passes) at 1e-4;
* config 4 -- Reddit shape (R-MAT, N = 232 965, E = 114.6 M, max degree ~1 M), kernel-sampled
  SAGE aggregation n = 20 at F = 256: the sampled rows (the first rows and the 64 longest)
  bit-exact against the oracle's sampler (cuda.h:313-321).

Synthetic graphs of the published shapes (no datasets offline), the bench.py generators.
"""
import os

import numpy as np
import pytest
import torch

import oracle as orc
from gala import layout, ops

pytestmark = pytest.mark.gpu

TOL = dict(atol=1e-4, rtol=1e-4)


def _threads():
    orc.set_threads(min(16, len(os.sched_getaffinity(0))))


def _rows_graph(g, rows):
    """The sub-CSR of the given rows (every edge kept, columns global): an oracle graph
    whose row i is g's row rows[i]."""
    rp = g.rowptr.astype(np.int64)
    deg = rp[rows + 1] - rp[rows]
    sp = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(deg, out=sp[1:])
    col = np.concatenate([g.col[rp[r]:rp[r + 1]] for r in rows]) if len(rows) else np.zeros(0, np.int32)
    return orc.Graph(len(rows), g.n_cols, sp.astype(np.int32), np.ascontiguousarray(col, np.int32))


@pytest.mark.timeout(300)
def test_config2_arxiv_gcn2_step_bitexact():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from gala.backend import HipBackend
    _threads()
    F = 128
    g = layout.gen_graph("uniform", 169_343, (1_335_586 - 169_343) // 2, seed=42)
    assert abs(g.nnz - 1_335_586) < 8
    be = HipBackend("cuda")
    agg = bench.OneGpuGCN(g, F, be)
    gen = torch.Generator(device="cuda").manual_seed(1234)
    X = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    dY = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    bufs = [be.empty(g.n_rows, F) for _ in range(4)]
    bench.make_fused_step(agg, X, dY, bufs)()
    og = orc.Graph(g.n_rows, g.n_cols, g.rowptr, g.col)
    norm = orc.degree(og, power=-0.5)
    xh, dyh = X.cpu().numpy(), dY.cpu().numpy()
    H1 = orc.spmm(og, xh, src_scale=norm, dst_scale=norm)
    H2 = orc.spmm(og, H1, src_scale=norm, dst_scale=norm)
    G1 = orc.spmm(og, dyh, src_scale=norm, dst_scale=norm)
    G0 = orc.spmm(og, G1, src_scale=norm, dst_scale=norm)
    for got, want in zip(bufs, (H1, H2, G1, G0)):
        np.testing.assert_array_equal(got.cpu().numpy(), want)


@pytest.mark.timeout(300)
def test_headline_products_gcn2_fused_step_bitexact():
    """The headline workload itself: bench.py's OneGpuGCN + make_fused_step on its uniform
    Products graph (N = 2 449 029, E = 126 167 309, F = 32 -- the graph, width and step the
    BENCH line times), all four outputs (H1, H2, G1, G0) on EVERY row bit-exact against the
    oracle's degree-normed chain (codegen/gala.cu:433-456: norm = deg^-1/2 from the
    degree pass, then norm * A (norm * H) per aggregation)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from gala.backend import HipBackend
    _threads()
    F = 32
    g = bench.products_graph("uniform", 1.0)
    assert (g.n_rows, g.nnz) == (bench.PRODUCTS_N, bench.PRODUCTS_E)
    be = HipBackend("cuda")
    agg = bench.OneGpuGCN(g, F, be)
    gen = torch.Generator(device="cuda").manual_seed(2024)
    X = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    dY = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    bufs = [be.empty(g.n_rows, F) for _ in range(4)]
    step = bench.make_fused_step(agg, X, dY, bufs)
    step()
    step()                                   # a second step overwrites every output alike
    torch.cuda.synchronize()
    og = orc.Graph(g.n_rows, g.n_cols, g.rowptr, g.col)
    norm = orc.degree(og, power=-0.5)
    xh, dyh = X.cpu().numpy(), dY.cpu().numpy()
    H1 = orc.spmm(og, xh, src_scale=norm, dst_scale=norm)
    H2 = orc.spmm(og, H1, src_scale=norm, dst_scale=norm)
    G1 = orc.spmm(og, dyh, src_scale=norm, dst_scale=norm)
    G0 = orc.spmm(og, G1, src_scale=norm, dst_scale=norm)
    for name, got, want in zip(("H1", "H2", "G1", "G0"), bufs, (H1, H2, G1, G0)):
        np.testing.assert_array_equal(got.cpu().numpy(), want, err_msg=name)


def _assert_source_logits(aR, X, wR, bR, H, cols):
    """The kernels' recomputed source logits aR[c] = <X[c, head h], wR_h> + bR[h] against the
    float64 per-head Linear (common.h:1248-1260) on the columns the oracle layer reads, 1e-5."""
    D = X.shape[1] // H
    w = wR.cpu().double().view(H, D)
    b = bR.cpu().double()
    got = aR.view(-1, H)
    for i in range(0, len(cols), 65536):
        c = torch.from_numpy(cols[i:i + 65536]).cuda()
        xc = X[c].cpu().double().view(-1, H, D)
        want = (xc * w[None]).sum(-1) + b[None]
        np.testing.assert_allclose(got[c].cpu().double().numpy(), want.numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.timeout(300)
def test_config3_products_gat8_rows_against_ref_layer():
    _threads()
    H, D = 8, 32
    F = H * D
    g = layout.gen_graph("uniform", 2_449_029, 61_859_140, seed=42)
    assert g.nnz > 120_000_000
    gen = torch.Generator(device="cuda").manual_seed(4321)
    X = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    dY = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    aL = torch.rand((g.n_rows, H), device="cuda", generator=gen) - 0.5
    wR = (torch.rand(F, device="cuda", generator=gen) - 0.5) * 0.2
    bR = (torch.rand(H, device="cuda", generator=gen) - 0.5) * 0.2
    dg = ops.DeviceGraph.from_host(g)
    Y, q, Ym, sma, aR = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
    dX, daL = ops.gat_bwd_stats(dg, aL, aR, dY, q, Y, Ym, sma, heads=H)
    torch.cuda.synchronize()
    k = int(np.searchsorted(g.rowptr, 600_000))          # rows [0, k): ~600 K edges
    # on the kernels' own source logits (the reference's torch Linear order is unpinned; see
    # tests/test_gpu_hub_rows.py)
    ref = orc.GatRefLayer(g.rowptr[:k + 1], g.col[:g.rowptr[k]], k, X.cpu().numpy(), dY.cpu().numpy(),
                          aL.cpu().numpy(), wR.cpu().numpy(), bR.cpu().numpy(), H, row_ids=np.arange(k),
                          aR=aR.view(-1, H).cpu().numpy()).run()
    np.testing.assert_allclose(Y[:k].cpu().numpy(), ref.Y, **TOL)
    np.testing.assert_allclose(dX[:k].cpu().numpy(), ref.dX, **TOL)
    np.testing.assert_allclose(daL.view(-1, H)[:k].cpu().numpy(), ref.daL, **TOL)
    # the aR handed to the oracle is itself checked: the float64 Linear on every column those
    # rows read (and the rows themselves), at size
    _assert_source_logits(aR, X, wR, bR, H, np.unique(np.concatenate([g.col[:g.rowptr[k]], np.arange(k)])))


@pytest.mark.timeout(300)
def test_config4_reddit_kernel_sampled_rows_bitexact():
    _threads()
    F, n = 256, 20
    g = layout.gen_graph("rmat", 232_965, (114_615_892 - 232_965) // 2, seed=42)
    deg = np.diff(g.rowptr.astype(np.int64))
    assert g.nnz > 100_000_000 and deg.max() > 500_000
    gen = torch.Generator(device="cuda").manual_seed(99)
    X = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    dg = ops.DeviceGraph.from_host(g)
    rows = np.unique(np.concatenate([np.arange(3000), np.argsort(deg)[-64:]])).astype(np.int64)
    sub = _rows_graph(g, rows)
    xh = X.cpu().numpy()
    for ra, rb in ((5, 7), (13, 3)):
        Y = ops.spmm(dg, X, nsamp=n, ra=ra, rb=rb).cpu().numpy()
        want = orc.spmm(sub, xh, sample=True, nsamp=n, ra=ra, rb=rb)
        np.testing.assert_array_equal(Y[rows], want)
