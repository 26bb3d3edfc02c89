"""CPU: the host-CPU baselines bench.py reports beside the GPU numbers.

* The SDDMM + edge-softmax baseline (oracle orc_gat_ref_layer, one REF GAT layer forward +
  backward, pass by pass with OpenMP) is the same arithmetic as composing the oracle's
  single-kernel restatements: bit-identical outputs, on the whole graph and on a row sample.
* bench.py's two baseline legs run on a small graph, report the cores they used and label
  their kind ("reference" when oracle/_ref is built, "port" for the GAT restatement).
"""
import os
import sys

import numpy as np
import pytest

import oracle as orc
from _graphs import cora_like, features, powerlaw, to_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _composed(og, aL, aR, X, dY, H):
    """The same layer from the single-kernel restatements (gat_fwd / gat_bwd / spmm)."""
    Y, alpha = orc.gat_fwd(og, aL, aR, X, heads=H)
    _, daL = orc.gat_bwd(og, aL, aR, X, dY, alpha, heads=H)
    gw = orc.Graph(og.n_rows, og.n_cols, og.rowptr, og.col, alpha, 1, None, H)
    dX = orc.spmm(gw, dY)
    return Y, dX, daL.reshape(-1, H), alpha


@pytest.mark.parametrize("H,D", [(1, 32), (4, 8), (8, 32)])
@pytest.mark.parametrize("graph", ["cora", "powerlaw"])
def test_gat_ref_layer_matches_composition(graph, H, D):
    g = cora_like() if graph == "cora" else powerlaw(n=2048, m=12000)
    og = to_oracle(g)
    F = H * D
    X = features(g.n_cols, F, seed=1)
    dY = features(g.n_rows, F, seed=2)
    aL = features(g.n_rows, H, seed=3) * 0.5
    wR = features(1, F, seed=4).ravel() * 0.2
    bR = features(1, H, seed=5).ravel() * 0.1
    layer = orc.GatRefLayer(g.rowptr, g.col, g.n_rows, X, dY, aL, wR, bR, H).run()
    aR = orc.head_attn(X, wR, bR, H)
    np.testing.assert_array_equal(layer.aR, aR)
    Y, dX, daL, alpha = _composed(og, aL, aR, X, dY, H)
    np.testing.assert_array_equal(layer.Y, Y)
    np.testing.assert_array_equal(layer.dX, dX)
    np.testing.assert_array_equal(layer.daL, daL)
    np.testing.assert_array_equal(layer.pa, alpha)
    # the per-head attention Linear against float64
    ref = (X.astype(np.float64).reshape(-1, H, D) * wR.astype(np.float64).reshape(H, D)).sum(-1) + bR
    np.testing.assert_allclose(aR, ref, atol=1e-5, rtol=1e-5)


def test_gat_ref_layer_row_sample():
    """The bench's bounded sample: rows [0, k) give exactly those rows of the full layer."""
    g = cora_like()
    H, F = 2, 16
    X, dY = features(g.n_cols, F, seed=1), features(g.n_rows, F, seed=2)
    aL, wR = features(g.n_rows, H, seed=3), features(1, F, seed=4).ravel()
    full = orc.GatRefLayer(g.rowptr, g.col, g.n_rows, X, dY, aL, wR, None, H).run()
    k = 1000
    part = orc.GatRefLayer(g.rowptr, g.col, k, X, dY, aL, wR, None, H).run()
    assert part.nnz == int(g.rowptr[k])
    for a, b in ((part.Y, full.Y), (part.dX, full.dX), (part.daL, full.daL), (part.q, full.q)):
        np.testing.assert_array_equal(a, b[:k])


def test_bench_baseline_legs_report_cores():
    sys.path.insert(0, ROOT)
    import bench
    from gala import layout
    g = layout.gen_graph("uniform", 3000, 20000, seed=42)
    d = bench.cpu_baseline(g, 32, budget_s=2.0)
    assert d["value"] > 0 and d["cores"] >= 1 and d["kind"] in ("reference", "port")
    assert d["host_cores"]["affinity_cpus"] >= d["cores"]
    if orc.ref_available():
        assert d["kind"] == "reference" and "x86-64-v4" in d["sample"]
    H, F = 8, 256
    X, dY = features(g.n_cols, F, seed=1), features(g.n_rows, F, seed=2)
    aL, wR = features(g.n_rows, H, seed=3), features(1, F, seed=4).ravel()
    b = bench.gat_cpu_baseline(g, X, dY, aL, wR, np.zeros(H, np.float32), H, budget_s=1.0)
    assert b["value"] > 0 and b["kind"] == "port" and b["cores"] >= 1
