"""GPU parity: libgala_hip.so (through the C ABI) vs the oracle on the same seeded inputs.

Bar: bit-exact for SpMM/degree/SDDVV/row-scale (same per-row CSR order and the same
rounding steps as the reference kernels), |err| <= 1e-4 (abs) + 1e-4 (rel) for the
reductions whose order the GPU changes (row-sum, SDDMM dot, softmax, fused GAT).
"""
import numpy as np
import pytest
import torch

import oracle as orc
from gala import _abi, layout, ops
from _graphs import cora_like, edge_values, features, powerlaw, to_oracle, with_empty_rows

pytestmark = pytest.mark.gpu
TOL = dict(atol=1e-4, rtol=1e-4)
DEV = "cuda"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


GRAPHS = {"cora": cora_like, "powerlaw": powerlaw, "empty_rows": with_empty_rows}


@pytest.fixture(scope="module", params=list(GRAPHS))
def graph(request):
    return GRAPHS[request.param]()


@pytest.mark.parametrize("F", [1, 2, 7, 16, 32, 33, 40, 47, 62, 64, 100, 128, 256, 602])
@pytest.mark.parametrize("weighted", [False, True])
def test_spmm_bitexact(graph, F, weighted):
    val = edge_values(graph.nnz) if weighted else None
    X = features(graph.n_cols, F)
    ref = orc.spmm(to_oracle(graph, val), X)
    dg = ops.DeviceGraph.from_host(layout.HostGraph(graph.n_rows, graph.n_cols, graph.rowptr, graph.col, val), split=False)
    Y = host(ops.spmm(dg, dev(X)))
    np.testing.assert_array_equal(Y, ref)


@pytest.mark.parametrize("F", [16, 47])
def test_spmm_reference_gspmm(F):
    """Same numbers as the reference's own CPU gSpMM (pinned by the golden fixtures)."""
    g = cora_like()
    X = features(g.n_cols, F, integer=False)
    dg = ops.DeviceGraph.from_host(g, split=False)
    Y = host(ops.spmm(dg, dev(X)))
    np.testing.assert_array_equal(Y, orc.gspmm(to_oracle(g), X))


def test_spmm_strided_and_accum():
    g = cora_like()
    Xf = features(g.n_cols, 40)
    X = dev(Xf)[:, 4:36]           # ldx = 40, F = 32, 16-B aligned
    Y0 = features(g.n_rows, 48, seed=5)
    Yt = dev(Y0)
    out = Yt[:, 8:40]
    ops.spmm(ops.DeviceGraph.from_host(g, split=False), X, out=out, accum=True)
    ref = orc.spmm(to_oracle(g), Xf[:, 4:36].copy(), Y=Y0[:, 8:40].copy(), accum=True)
    got = host(Yt)
    np.testing.assert_array_equal(got[:, 8:40], ref)
    np.testing.assert_array_equal(got[:, :8], Y0[:, :8])
    np.testing.assert_array_equal(got[:, 40:], Y0[:, 40:])


@pytest.mark.parametrize("F", [32, 47])
def test_spmm_gcn_norm_fused(F):
    g = powerlaw()
    norm = (1.0 / np.sqrt(g.degrees().astype(np.float32))).astype(np.float32)
    X = features(g.n_cols, F)
    ref = orc.spmm(to_oracle(g), X, src_scale=norm, dst_scale=norm)
    dg = ops.DeviceGraph.from_host(g, split=False)
    Y = host(ops.spmm(dg, dev(X), src_scale=dev(norm), dst_scale=dev(norm)))
    np.testing.assert_array_equal(Y, ref)


@pytest.mark.parametrize("F", [1, 3, 32, 47, 100])
def test_row_broadcast_then_spmm_matches_fused(F):
    """norm * A (norm * X) as two kernels == the fused src/dst-scaled SpMM, bit for bit."""
    g = powerlaw()
    norm = (1.0 / np.sqrt(g.degrees().astype(np.float32))).astype(np.float32)
    X = features(g.n_cols, F)
    dg = ops.DeviceGraph.from_host(g, split=False)
    Xs = ops.row_broadcast(dev(norm), dev(X))
    np.testing.assert_array_equal(host(Xs), norm[:, None] * X)
    Y = host(ops.spmm(dg, Xs, dst_scale=dev(norm)))
    np.testing.assert_array_equal(Y, orc.spmm(to_oracle(g), X, src_scale=norm, dst_scale=norm))


@pytest.mark.parametrize("cpp", [900, 1000, 2708])
@pytest.mark.parametrize("F", [1, 32, 100])
def test_spmm_col_tiled(cpp, F):
    g = cora_like()
    t = layout.col_tile(g, cpp)
    X = features(g.n_cols, F)
    ref = orc.spmm(to_oracle(t), X)
    Y = host(ops.spmm(ops.DeviceGraph.from_host(t, split=False), dev(X)))
    np.testing.assert_array_equal(Y, ref)
    # tiled == untiled: segments partition each row's ascending columns in order
    np.testing.assert_array_equal(Y, orc.spmm(to_oracle(g), X))


def test_spmm_many_segments():
    g = cora_like()
    t = layout.col_tile(g, 20)   # 136 segments > 64 per launch
    X = features(g.n_cols, 32)
    Y = host(ops.spmm(ops.DeviceGraph.from_host(t, split=False), dev(X)))
    np.testing.assert_array_equal(Y, orc.spmm(to_oracle(t), X))


@pytest.mark.parametrize("F", [32, 256])
@pytest.mark.parametrize("tiled", [False, True])
def test_spmm_kernel_sampled(F, tiled):
    g = with_empty_rows()
    if tiled:
        g = layout.col_tile(g, 300)
    X = features(g.n_cols, F)
    ref = orc.spmm(to_oracle(g), X, sample=True, nsamp=20, ra=5, rb=7)
    Y = host(ops.spmm(ops.DeviceGraph.from_host(g, split=False), dev(X), nsamp=20, ra=5, rb=7))
    np.testing.assert_array_equal(Y, ref)


def test_spmm_multihead_weights():
    g = cora_like()
    H, D = 4, 8
    val = edge_values(g.nnz, heads=H)
    X = features(g.n_cols, H * D)
    ref = orc.spmm(to_oracle(g, val, heads=H), X)
    dg = ops.DeviceGraph.from_host(g, split=False).with_values(dev(val), val_heads=H)
    np.testing.assert_array_equal(host(ops.spmm(dg, dev(X))), ref)


@pytest.mark.parametrize("power", [1.0, -0.5])
@pytest.mark.parametrize("weighted", [False, True])
def test_degree(graph, power, weighted):
    val = edge_values(graph.nnz) if weighted else None
    ref = orc.degree(to_oracle(graph, val), power=power)
    dg = ops.DeviceGraph.from_host(layout.HostGraph(graph.n_rows, graph.n_cols, graph.rowptr, graph.col, val), split=False)
    got = host(ops.degree(dg, power=power))
    if power == 1.0:
        np.testing.assert_array_equal(got, ref)
    else:
        np.testing.assert_allclose(got, ref, **TOL)


def test_degree_sampled_full_op():
    g = layout.col_tile(cora_like(), 1000)
    got = host(ops.degree(ops.DeviceGraph.from_host(g, split=False), nsamp=20))
    np.testing.assert_array_equal(got, np.full(g.n_rows, 20.0 * g.n_seg, np.float32))


@pytest.mark.parametrize("op", [0, 1, 2])
@pytest.mark.parametrize("heads", [1, 3, 4, 8])
def test_sddvv(graph, op, heads):
    a = features(graph.n_rows, heads, seed=11)
    b = features(graph.n_cols, heads, seed=12)
    ref = orc.sddvv(to_oracle(graph), a, b, heads=heads, op=op, slope=0.2)
    got = host(ops.sddvv(ops.DeviceGraph.from_host(graph, split=False), dev(a), dev(b), op=op, heads=heads, slope=0.2))
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("heads", [1, 3, 8])
def test_row_sum_and_scale(graph, tiled, heads):
    g = layout.col_tile(graph, 1000) if tiled else graph
    v = edge_values(g.nnz, heads=heads, seed=5)
    dg = ops.DeviceGraph.from_host(g, split=False)
    got = host(ops.row_sum(dg, dev(v), heads=heads, eps=1e-12))
    # K7 in the reference's order (cuda.h:505-524): bit-identical, segments and empty rows too
    np.testing.assert_array_equal(got, orc.row_sum(to_oracle(g), v, heads=heads, eps=1e-12))
    out0 = features(g.n_rows, heads, seed=7).ravel()
    acc = dev(out0)
    ops.row_sum(dg, dev(v), heads=heads, eps=1e-12, out=acc, accum=True)
    np.testing.assert_array_equal(host(acc), orc.row_sum(to_oracle(g), v, heads=heads, eps=1e-12,
                                                         out=out0.copy(), accum=True))
    q = features(g.n_rows, heads, seed=6).ravel()
    vv = dev(v)
    ops.row_scale_(dg, dev(q), vv, heads=heads)
    np.testing.assert_array_equal(host(vv), orc.row_scale(to_oracle(g), q, v, heads=heads))


@pytest.mark.parametrize("F,heads", [(1, 1), (16, 1), (32, 1), (33, 1), (47, 1), (62, 1), (100, 1), (256, 8), (64, 2)])
def test_sddmm(graph, F, heads):
    A = features(graph.n_rows, F, seed=21)
    B = features(graph.n_cols, F, seed=22)
    got = host(ops.sddmm(ops.DeviceGraph.from_host(graph, split=False), dev(A), dev(B), heads=heads))
    np.testing.assert_allclose(got, orc.sddmm(to_oracle(graph), A, B, heads=heads), **TOL)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
@pytest.mark.parametrize("heads", [1, 3, 8])
@pytest.mark.parametrize("tiled", [False, True])
def test_edge_softmax(graph, mode, heads, tiled):
    g = layout.col_tile(graph, 1000) if tiled else graph
    s = edge_values(g.nnz, heads=heads, lo=-3, hi=3, seed=8)
    d = edge_values(g.nnz, heads=heads, lo=-1, hi=1, seed=9)
    dg = ops.DeviceGraph.from_host(g, split=False)
    a = host(ops.edge_softmax(dg, dev(s), heads=heads, mode=mode))
    a_ref = orc.softmax_fwd(to_oracle(g), s, heads=heads, mode=mode)
    np.testing.assert_allclose(a, a_ref, **TOL)
    ds = host(ops.edge_softmax_bwd(dg, dev(a_ref), dev(d), heads=heads, mode=mode))
    np.testing.assert_allclose(ds, orc.softmax_bwd(to_oracle(g), a_ref, d, heads=heads, mode=mode), **TOL)


def test_edge_softmax_overflow_clamp():
    """REF mode clamps exp at 1e12 and has no max subtraction (common.h:760-761)."""
    g = cora_like()
    s = edge_values(g.nnz, lo=20, hi=40, seed=8)
    got = host(ops.edge_softmax(ops.DeviceGraph.from_host(g, split=False), dev(s)))
    np.testing.assert_allclose(got, orc.softmax_fwd(to_oracle(g), s), **TOL)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
@pytest.mark.parametrize("F,heads", [(32, 1), (33, 1), (47, 1), (62, 1), (256, 8)])
def test_gat_fused(graph, mode, F, heads):
    aL = features(graph.n_rows, heads, seed=31)
    aR = features(graph.n_cols, heads, seed=32)
    X = features(graph.n_cols, F, seed=33)
    Y_ref, al_ref = orc.gat_fwd(to_oracle(graph), aL, aR, X, heads=heads, slope=0.2, mode=mode)
    Y, al = ops.gat_fwd(ops.DeviceGraph.from_host(graph, split=False), dev(aL), dev(aR), dev(X), heads=heads,
                        slope=0.2, mode=mode, want_alpha=True)
    np.testing.assert_allclose(host(al), al_ref, **TOL)
    np.testing.assert_allclose(host(Y), Y_ref, **TOL)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
@pytest.mark.parametrize("F,heads", [(32, 1), (33, 1), (47, 1), (62, 1), (256, 8), (64, 4)])
@pytest.mark.parametrize("tiled", [False, True])
def test_gat_bwd_fused(graph, mode, F, heads, tiled):
    """Fused d alpha -> softmax bwd -> LeakyReLU bwd -> row sum vs the oracle chain."""
    g = layout.col_tile(graph, 1000) if tiled else graph
    aL = features(g.n_rows, heads, seed=41)
    aR = features(g.n_cols, heads, seed=42)
    X = features(g.n_cols, F, seed=43)
    dY = features(g.n_rows, F, seed=44)
    og = to_oracle(g)
    _, alpha = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=mode)
    dz_ref, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, alpha, heads=heads, slope=0.2, mode=mode)
    daL, dz = ops.gat_bwd(ops.DeviceGraph.from_host(g, split=False), dev(aL), dev(aR), dev(X), dev(dY),
                          dev(alpha), heads=heads, slope=0.2, mode=mode)
    np.testing.assert_allclose(host(daL), daL_ref, **TOL)
    if mode == _abi.GALA_SOFTMAX_FIXED:
        np.testing.assert_allclose(host(dz), dz_ref, **TOL)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
@pytest.mark.parametrize("F", [32, 47, 64])
@pytest.mark.parametrize("tiled", [False, True])
def test_gat_attention_recompute(graph, mode, F, tiled):
    """gala_gat_{fwd,bwd}_attn_f32: aR = X wR + bR recomputed from the gathered rows,
    against the oracle chain on that aR (computed here in float64, rounded to fp32)."""
    g = layout.col_tile(graph, 1000) if tiled else graph
    aL = features(g.n_rows, 1, seed=51)
    X = features(g.n_cols, F, seed=53)
    dY = features(g.n_rows, F, seed=54)
    wR = features(1, F, seed=55).ravel() * 0.5
    bR = np.array([0.1], np.float32)
    aR = (X.astype(np.float64) @ wR.astype(np.float64) + 0.1).astype(np.float32)
    og = to_oracle(g)
    Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=1, slope=0.2, mode=mode)
    dg = ops.DeviceGraph.from_host(g, split=False)
    Y, al = ops.gat_fwd_attn(dg, dev(aL), dev(wR), dev(bR), dev(X), slope=0.2, mode=mode, want_alpha=True)
    np.testing.assert_allclose(host(al), al_ref, **TOL)
    np.testing.assert_allclose(host(Y), Y_ref, **TOL)
    if mode == _abi.GALA_SOFTMAX_REF:
        _, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=1, slope=0.2, mode=mode)
        daL = ops.gat_bwd_attn(dg, dev(aL), dev(wR), dev(bR), dev(X), dev(dY), dev(al_ref), slope=0.2)
        np.testing.assert_allclose(host(daL), daL_ref, **TOL)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
@pytest.mark.parametrize("F,heads", [(32, 1), (47, 1), (256, 8), (64, 4)])
def test_gat_hub_rows_split(mode, F, heads):
    """Hub rows cut into chunks (plan threshold 64, chunks of 32 edges): the fused GAT
    forward / backward combine per-chunk partials (online-softmax merge, ordered sums)."""
    g = powerlaw()
    aL = features(g.n_rows, heads, seed=61)
    aR = features(g.n_cols, heads, seed=62)
    X = features(g.n_cols, F, seed=63)
    dY = features(g.n_rows, F, seed=64)
    og = to_oracle(g)
    Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=mode)
    dz_ref, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=heads, slope=0.2, mode=mode)
    dg = ops.DeviceGraph.from_host(g, split=False)
    dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
    assert dg.split_rows > 10
    Y, al = ops.gat_fwd(dg, dev(aL), dev(aR), dev(X), heads=heads, slope=0.2, mode=mode, want_alpha=True)
    np.testing.assert_allclose(host(al), al_ref, **TOL)
    np.testing.assert_allclose(host(Y), Y_ref, **TOL)
    daL, dz = ops.gat_bwd(dg, dev(aL), dev(aR), dev(X), dev(dY), dev(al_ref), heads=heads, slope=0.2, mode=mode)
    np.testing.assert_allclose(host(daL), daL_ref, **TOL)
    if mode == _abi.GALA_SOFTMAX_FIXED:
        np.testing.assert_allclose(host(dz), dz_ref, **TOL)
    if heads == 1:  # attention recompute on the same split plan
        wR = features(1, F, seed=65).ravel() * 0.5
        bR = np.array([0.1], np.float32)
        aR2 = (X.astype(np.float64) @ wR.astype(np.float64) + 0.1).astype(np.float32)
        Y2_ref, al2_ref = orc.gat_fwd(og, aL, aR2, X, heads=1, slope=0.2, mode=mode)
        Y2, al2 = ops.gat_fwd_attn(dg, dev(aL), dev(wR), dev(bR), dev(X), slope=0.2, mode=mode, want_alpha=True)
        np.testing.assert_allclose(host(al2), al2_ref, **TOL)
        np.testing.assert_allclose(host(Y2), Y2_ref, **TOL)
        if mode == _abi.GALA_SOFTMAX_REF:
            _, daL2_ref = orc.gat_bwd(og, aL, aR2, X, dY, al2_ref, heads=1, slope=0.2, mode=mode)
            daL2 = ops.gat_bwd_attn(dg, dev(aL), dev(wR), dev(bR), dev(X), dev(dY), dev(al2_ref), slope=0.2)
            np.testing.assert_allclose(host(daL2), daL2_ref, **TOL)


@pytest.mark.parametrize("heads", [1, 8])
@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
def test_edge_ops_hub_rows_split(heads, mode):
    """Row-segment edge ops with hub rows cut into chunks (plan threshold 64, 32-edge
    chunks): SDDVV / row-scale per chunk (bit-exact), row sum and softmax fwd/bwd from
    chunk partials combined in order (tolerance)."""
    g = powerlaw()
    og = to_oracle(g)
    dg = ops.DeviceGraph.from_host(g, split=False)
    dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
    a = features(g.n_rows, heads, seed=71)
    b = features(g.n_cols, heads, seed=72)
    np.testing.assert_array_equal(host(ops.sddvv(dg, dev(a), dev(b), op=2, heads=heads, slope=0.2)),
                                  orc.sddvv(og, a, b, heads=heads, op=2, slope=0.2))
    v = edge_values(g.nnz, heads=heads, seed=73)
    # REF order (default): hub rows by k_row_sum_hub's chains, bit-identical; chunked: tolerance
    np.testing.assert_array_equal(host(ops.row_sum(dg, dev(v), heads=heads, eps=1e-12)),
                                  orc.row_sum(og, v, heads=heads, eps=1e-12))
    np.testing.assert_allclose(host(ops.row_sum(dg, dev(v), heads=heads, eps=1e-12, hub="chunked")),
                               orc.row_sum(og, v, heads=heads, eps=1e-12), **TOL)
    vv = dev(v)
    ops.row_scale_(dg, dev(a), vv, heads=heads)
    np.testing.assert_array_equal(host(vv), orc.row_scale(og, a.ravel(), v, heads=heads))
    s = edge_values(g.nnz, heads=heads, lo=-3, hi=3, seed=74)
    d = edge_values(g.nnz, heads=heads, lo=-1, hi=1, seed=75)
    a_ref = orc.softmax_fwd(og, s, heads=heads, mode=mode)
    np.testing.assert_allclose(host(ops.edge_softmax(dg, dev(s), heads=heads, mode=mode)), a_ref, **TOL)
    np.testing.assert_allclose(host(ops.edge_softmax_bwd(dg, dev(a_ref), dev(d), heads=heads, mode=mode)),
                               orc.softmax_bwd(og, a_ref, d, heads=heads, mode=mode), **TOL)


def test_edge_permute():
    g = powerlaw()
    t, perm = layout.transpose(g)
    v = edge_values(g.nnz, heads=2)
    got = host(ops.edge_permute(dev(perm), dev(v), heads=2))
    np.testing.assert_array_equal(got, v.reshape(-1, 2)[perm].ravel())


def test_empty_graph_and_zero_features():
    g = layout.HostGraph(5, 5, np.zeros(6, np.int32), np.zeros(0, np.int32))
    dg = ops.DeviceGraph.from_host(g, split=False)
    Y = host(ops.spmm(dg, torch.ones(5, 8, device=DEV)))
    np.testing.assert_array_equal(Y, np.zeros((5, 8), np.float32))
    np.testing.assert_array_equal(host(ops.degree(dg)), np.zeros(5, np.float32))


def test_invalid_args_fail_loudly():
    g = cora_like()
    dg = ops.DeviceGraph.from_host(g, split=False)
    X = torch.ones(g.n_cols, 8, device=DEV)
    with pytest.raises(_abi.GalaError):
        _abi.call("gala_spmm_f32", dg.csr(), X.data_ptr(), 4, X.data_ptr(), 8, 8, None, None, 0, 0, 0, 0, None)
    with pytest.raises(ValueError):
        ops.spmm(dg, torch.ones(g.n_cols, 8))


# ---- against the reference's own outputs (tests/golden, generated from /root/reference)
import glob as _glob  # noqa: E402
import os as _os  # noqa: E402

_GOLDEN = sorted(_glob.glob(_os.path.join(_os.path.dirname(__file__), "golden", "*.npz")))


@pytest.mark.parametrize("path", _GOLDEN, ids=[_os.path.basename(p)[:-4] for p in _GOLDEN])
def test_spmm_matches_reference_gspmm_fixtures(path):
    fx = dict(np.load(path, allow_pickle=False))
    n = int(fx["n"])
    g = layout.HostGraph(n, n, fx["rowptr"], fx["col"])
    dg = ops.DeviceGraph.from_host(g, split=False)
    for k in [k for k in fx if k.startswith("Y_F") or k.startswith("Yw_F")]:
        F = int(k.split("_F")[1])
        X = dev(np.ascontiguousarray(fx["X"][:, :F]))
        gg = dg if k.startswith("Y_") else dg.with_values(dev(fx["w"]))
        np.testing.assert_array_equal(host(ops.spmm(gg, X)), fx[k], err_msg=k)
    # tiled layouts from ord_col_tiling_torch give the same aggregation
    for k in [k for k in fx if k.startswith("tile") and k.endswith("_rowptr")]:
        cpp = k[4:-len("_rowptr")]
        bounds = fx[f"tile{cpp}_bounds"]
        t = layout.HostGraph(n, n, fx[k], fx[f"tile{cpp}_col"], None, len(bounds) // 2, bounds)
        F = min(int(k2[3:]) for k2 in fx if k2.startswith("Y_F"))
        X = dev(np.ascontiguousarray(fx["X"][:, :F]))
        np.testing.assert_array_equal(host(ops.spmm(ops.DeviceGraph.from_host(t, split=False), X)), fx[f"Y_F{F}"])


# ---- the GCN step's epilogues (gala_spmm_ex_f32, gala_row_broadcast_deg_f32) ---------
@pytest.mark.parametrize("F", [1, 7, 32, 47, 128, 2100])
@pytest.mark.parametrize("kind", ["cora", "hubs", "empty"])
def test_spmm_epilogue_deg_norm_and_next_input(F, kind):
    """The degree norm formed from the rowptr and the next aggregation's pre-scaled input
    written by the SpMM equal the degree pass + pow(-0.5) + ROW_BROADCAST chain bit for bit
    (codegen/gala.cu:433-456), hub rows (both orders), empty rows and F past one launch's
    column block (2100 > 512 float4) included; the oracle pins the chain."""
    g = {"cora": cora_like, "hubs": hub_graph, "empty": with_empty_rows}[kind]()
    # bit patterns: an empty row's norm is inf (as pow(0, -0.5) is), its sums NaN on both paths
    _same = lambda a, b: torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))  # noqa: E731
    dg = ops.DeviceGraph.from_host(g)
    X = dev(features(g.n_cols, F, seed=5))
    norm = ops.degree(dg, power=-0.5)
    np.testing.assert_array_equal(host(norm), orc.degree(to_oracle(g), power=-0.5))
    Xs = ops.row_broadcast(norm, X)
    assert _same(ops.row_broadcast_deg(dg, X), Xs)
    for hub in ("exact", "chunked"):
        Y = ops.spmm(dg, Xs, dst_scale=norm, hub=hub)
        Yn = ops.row_broadcast(norm, Y)
        Y1, Y2 = torch.empty_like(Y), torch.empty_like(Y)
        ops.spmm(dg, Xs, out=Y1, dst_deg=True, out2=Y2, hub=hub)
        assert _same(Y1, Y) and _same(Y2, Yn)
        # a given second scale, and the deg norm without the second output
        s2 = dev(features(g.n_rows, 1, seed=6).ravel())
        ops.spmm(dg, Xs, out=Y1, dst_deg=True, out2=Y2, out2_scale=s2, hub=hub)
        assert _same(Y1, Y) and _same(Y2, ops.row_broadcast(s2, Y))
        assert _same(ops.spmm(dg, Xs, dst_deg=True, hub=hub), Y)
    if kind != "hubs":
        np.testing.assert_array_equal(host(Y1), orc.spmm(to_oracle(g), host(Xs), dst_scale=host(norm)))
    # accumulate with the deg norm: Y += norm * A X
    Y0 = dev(features(g.n_rows, F, seed=8))
    want = ops.spmm(dg, Xs, dst_scale=norm, out=Y0.clone(), accum=True)
    got = ops.spmm(dg, Xs, dst_deg=True, out=Y0.clone(), accum=True)
    assert _same(got, want)
    # refused: the deg norm with a given dst scale, or with kernel sampling
    with pytest.raises(_abi.GalaError):
        ops.spmm(dg, Xs, dst_scale=norm, dst_deg=True)
    with pytest.raises(_abi.GalaError):
        ops.spmm(dg, Xs, dst_deg=True, nsamp=4)
    # refused on a weighted graph (its degree pass sums the values, not the rowptr counts)
    gw = dg.with_values(dev(edge_values(g.nnz)))
    with pytest.raises(_abi.GalaError):
        ops.spmm(gw, Xs, dst_deg=True)
    with pytest.raises(_abi.GalaError):
        ops.row_broadcast_deg(gw, X)


@pytest.mark.parametrize("F", [1, 7, 32, 47, 128, 2100])
@pytest.mark.parametrize("kind", ["cora", "empty", "tiled", "many_segs", "padded"])
def test_spmm_relu_prologue_and_epilogue_match_the_passes(F, kind):
    """gala_spmm_ex_f32's ReLU fields (gcn_aggregate_relu_apply's fused forward and backward)
    against the passes they fold, bit for bit: the source pre * relu(act * X) formed per
    gathered element (gala_row_scale_relu_f32, then the SpMM), and the ReLU backward of the
    result in the store (the SpMM, then gala_relu_scale_backward_f32); each factor absent or
    present, -0 / exact zeros / NaN in X, column segments (136 of them: more than one launch's
    64, so the ReLU backward must wait for the last launch's sums), row-padded operands, F past
    one launch's column block.  Refused on weighted or sampled graphs and with hub rows."""
    g = with_empty_rows() if kind == "empty" else cora_like()
    tile = {"tiled": 900, "many_segs": 20}.get(kind)
    dg = ops.DeviceGraph.from_host(layout.col_tile(g, tile) if tile else g, split=False)
    _same = lambda a, b: torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))  # noqa: E731
    rng = np.random.default_rng(F)
    X = rng.uniform(-1, 1, (g.n_cols, F)).astype(np.float32)
    X[::7, 0] = 0.0
    X[1::11, -1] = -0.0
    X[5, 0] = np.nan
    R = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    if kind == "padded":
        _, Xd = _padded(X, F, 5.0)
        _, Rd = _padded(R, F, 7.0)
    else:
        Xd, Rd = dev(X), dev(R)
    act, pre, post = (dev(rng.uniform(0.1, 2, g.n_rows).astype(np.float32)) for _ in range(3))
    for a, s, d in ((act, pre, post), (None, pre, None), (act, None, post), (None, None, None)):
        if kind == "many_segs":
            d = None  # a dst scale past one launch's segments is refused (test_spmm_many_segments)
        want = ops.spmm(dg, ops.row_scale_relu(Xd, a, s), dst_scale=d)
        got = ops.spmm(dg, Xd, src_scale=s, dst_scale=d, src_relu=True, src_act=a)
        assert _same(got, want), (a is None, s is None, d is None)
        G = ops.spmm(dg, Xd, src_scale=s, dst_scale=d)
        want = ops.relu_scale_backward(Rd, G, a)
        got = ops.spmm(dg, Xd, src_scale=s, dst_scale=d, relu_x=Rd, relu_act=a)
        assert _same(got, want), (a is None, s is None, d is None)
    if kind == "cora":
        with pytest.raises(_abi.GalaError):
            ops.spmm(dg.with_values(dev(edge_values(g.nnz))), Xd, src_relu=True)
        with pytest.raises(_abi.GalaError):
            ops.spmm(dg, Xd, relu_x=Rd, nsamp=3)
        with pytest.raises(_abi.GalaError):
            ops.spmm(ops.DeviceGraph.from_host(hub_graph()), dev(features(hub_graph().n_cols, F)), src_relu=True)


def test_fused_gcn_step_matches_the_chain():
    """bench.py's fused step (the headline workload) against its unfused chain on a graph
    with hub rows and one without: all four outputs bit-identical."""
    import sys
    sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
    import bench
    from gala.backend import HipBackend
    be = HipBackend("cuda")
    for g in (cora_like(), hub_graph()):
        agg = bench.OneGpuGCN(g, 32, be)
        X, dY = dev(features(g.n_rows, 32, seed=1)), dev(features(g.n_rows, 32, seed=2))
        bufs = [be.empty(g.n_rows, 32) for _ in range(4)]
        bench.make_step(agg, X, dY, bufs)()
        want = [b.clone() for b in bufs]
        bench.make_fused_step(agg, X, dY, bufs)()
        for a, b in zip(want, bufs):
            assert torch.equal(a, b)


# ---- hub rows (power-law): split plan ----------------------------------------------------
def hub_graph():
    """R-MAT graph plus a star row of 20k edges and a few mid-size rows."""
    rng = np.random.default_rng(11)
    base = powerlaw(n=6000, m=40000, seed=5)
    rows = np.repeat(np.arange(base.n_rows), np.diff(base.rowptr)).astype(np.int32)
    src = np.concatenate([rows, np.full(20000, 17, np.int32), np.full(3000, 4000, np.int32)])
    dst = np.concatenate([base.col, rng.integers(0, 6000, 23000).astype(np.int32)])
    return layout.csr_build(6000, 6000, src, dst)


def assert_reordered_sum(Y, g, X, val=None, dst_scale=None, Y0=None):
    """Rows the split plan sums in chunks are compared with the exact (float64) sum.

    A chunked fp32 sum of a 20k-edge row differs from the sequential one by rounding alone,
    so the bound scales with the row's L1 mass: |Y - exact| <= 1e-6 * sum|A_e X_j| + 1e-6.
    (The reference's own sequential fp32 sum is no fixed point to compare with at 1e-4: on
    these hub rows it is itself up to 8e-4 from the exact sum, measured on MI355X; both sums
    are within the L1 bound of it.)  This is the GALA_SPMM_HUB_CHUNKED fast mode only: the
    default REF order sums every hub row sequentially, bit for bit.
    """
    import scipy.sparse as sp
    v = np.ones(g.nnz) if val is None else np.asarray(val, np.float64)
    # copies: scipy canonicalises (sums duplicate edges) in place on the arrays it is given
    A = sp.csr_matrix((v, g.col.copy(), g.rowptr.copy()), shape=(g.n_rows, g.n_cols))
    X64 = X.astype(np.float64)
    exact = A @ X64
    mass = abs(A) @ np.abs(X64)
    if dst_scale is not None:
        exact *= dst_scale[:, None]
        mass *= np.abs(dst_scale)[:, None]
    if Y0 is not None:
        exact += Y0
        mass += np.abs(Y0)
    err = np.abs(Y.astype(np.float64) - exact)
    bound = 1e-6 * mass + 1e-6
    assert np.all(err <= bound), f"max err/bound {np.max(err / bound):.3f}"


@pytest.mark.parametrize("F", [1, 32, 47, 256])
@pytest.mark.parametrize("weighted", [False, True])
def test_spmm_split_hub_rows(F, weighted):
    g = hub_graph()
    val = edge_values(g.nnz) if weighted else None
    hg = layout.HostGraph(g.n_rows, g.n_cols, g.rowptr, g.col, val)
    dg = ops.DeviceGraph.from_host(hg)
    assert dg.split_rows >= 2
    X = features(g.n_cols, F)
    ref = orc.spmm(to_oracle(hg), X)
    # REF order (the default): hub rows summed sequentially by k_spmm_hub_exact -- within
    # north_star's 1e-4 of the reference's sequential sum, in fact bit-identical
    Y = host(ops.spmm(dg, dev(X)))
    np.testing.assert_allclose(Y, ref, rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(Y, ref)
    np.testing.assert_array_equal(host(ops.spmm(dg, dev(X), exact=True)), ref)   # GALA_SPMM_EXACT
    # the fast mode: hub rows as chunk partials (reordered sum)
    Yc = host(ops.spmm(dg, dev(X), hub="chunked"))
    assert_reordered_sum(Yc, g, X, val)
    light = np.diff(g.rowptr) <= 1024
    np.testing.assert_array_equal(Yc[light], ref[light])     # other rows: still bit-exact


@pytest.mark.parametrize("F", [1, 32, 47, 256])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("hubs", [False, True])
def test_spmm_row_order_bitexact(F, weighted, hubs):
    """Degree-ordered row schedule (gala_host_row_order), alone and with the hub-row split:
    rows run in another order, each still one sequential pass -> bit-identical (without
    hubs), and the sampled path too."""
    g = powerlaw()
    val = edge_values(g.nnz) if weighted else None
    X = features(g.n_cols, F)
    dg = ops.DeviceGraph.from_host(layout.HostGraph(g.n_rows, g.n_cols, g.rowptr, g.col, val), split=False)
    dg.set_split_plan(g.rowptr, 64 if hubs else 0, chunk=32, row_order=True)
    ref = orc.spmm(to_oracle(g, val), X)
    np.testing.assert_array_equal(host(ops.spmm(dg, dev(X))), ref)   # REF order: hub rows too
    if hubs:
        got = host(ops.spmm(dg, dev(X), hub="chunked"))
        assert_reordered_sum(got, g, X, val)                     # split rows: chunked order
        light = np.diff(g.rowptr) <= 64
        np.testing.assert_array_equal(got[light], ref[light])  # the others: bit-exact
    np.testing.assert_array_equal(host(ops.spmm(dg, dev(X), nsamp=20)),
                                  orc.spmm(to_oracle(g, val), X, sample=True, nsamp=20))


def test_spmm_split_with_norms_and_accum():
    g = hub_graph()
    dg = ops.DeviceGraph.from_host(g)
    norm = (1.0 / np.sqrt(g.degrees().astype(np.float32))).astype(np.float32)
    X = features(g.n_cols, 32)
    Y0 = features(g.n_rows, 32, seed=3)
    ref = orc.spmm(to_oracle(g), X, dst_scale=norm, Y=Y0.copy(), accum=True)
    Yt = dev(Y0)
    ops.spmm(dg, dev(X), dst_scale=dev(norm), out=Yt, accum=True)
    np.testing.assert_array_equal(host(Yt), ref)                # REF order, hub rows included
    Yt = dev(Y0)
    ops.spmm(dg, dev(X), dst_scale=dev(norm), out=Yt, accum=True, hub="chunked")
    light = np.diff(g.rowptr) <= 1024
    np.testing.assert_allclose(host(Yt)[light], ref[light], **TOL)
    assert_reordered_sum(host(Yt), g, X, dst_scale=norm.astype(np.float64), Y0=Y0)
    # accumulate without a dst scale starts from Y (the hub kernel too)
    Yt = dev(Y0)
    ops.spmm(dg, dev(X), out=Yt, accum=True)
    np.testing.assert_array_equal(host(Yt), orc.spmm(to_oracle(g), X, Y=Y0.copy(), accum=True))


@pytest.mark.parametrize("F,heads", [(32, 1), (47, 1), (256, 8)])
def test_sddmm_split_hub_rows(F, heads):
    g = hub_graph()
    dg = ops.DeviceGraph.from_host(g)
    assert dg.split_rows >= 2
    A = features(g.n_rows, F, seed=21)
    B = features(g.n_cols, F, seed=22)
    got = host(ops.sddmm(dg, dev(A), dev(B), heads=heads))
    np.testing.assert_allclose(got, orc.sddmm(to_oracle(g), A, B, heads=heads), **TOL)


# ---- FFN gradients (gala_dense_grad_f32) ---------------------------------------------------
@pytest.mark.parametrize("N,K,M", [(2708, 64, 32), (100000, 100, 32), (50000, 32, 47),
                                   (20000, 602, 256), (33, 7, 1), (1, 1, 1), (0, 16, 8),
                                   # narrow outputs (k_tn_skinny): every KL / CH class
                                   (100000, 32, 1), (100000, 47, 1), (70001, 5, 2), (3000, 16, 3),
                                   (65537, 100, 4), (4099, 256, 1), (50, 129, 4), (0, 47, 1),
                                   # LDS-staged 128 x 128 tiles (k_tn_lds): config 5's layers,
                                   # partial m / k tiles, fewer rows than one stage, a ragged stage
                                   (100000, 128, 128), (40000, 128, 172), (20003, 256, 68),
                                   (5000, 132, 260), (31, 128, 128), (70, 68, 68),
                                   # 192-row m tiles (they pad M less): one, and three with a partial last
                                   (3000, 100, 180), (2000, 72, 540)])
def test_dense_grad_matches_float64(N, K, M):
    """dW = dY^T X, db = sum_n dY: |err| <= 1e-5 * sum_n |dY||X| (fp32 accumulation bound)."""
    rng = np.random.default_rng(N + K + M)
    X = rng.uniform(-1, 1, (N, K)).astype(np.float32)
    dY = rng.uniform(-1, 1, (N, M)).astype(np.float32)
    dW, db = ops.dense_grad(dev(X), dev(dY))
    X64, Y64 = X.astype(np.float64), dY.astype(np.float64)
    want = Y64.T @ X64
    mass = np.abs(Y64).T @ np.abs(X64)
    assert np.all(np.abs(host(dW) - want) <= 1e-5 * mass + 1e-6)
    np.testing.assert_allclose(host(db), Y64.sum(0), atol=1e-5 * max(N, 1), rtol=1e-5)
    # deterministic: the same shapes give the same bits
    dW2, db2 = ops.dense_grad(dev(X), dev(dY))
    np.testing.assert_array_equal(host(dW2), host(dW))
    np.testing.assert_array_equal(host(db2), host(db))


def test_dense_grad_strided_accumulate_and_no_bias():
    rng = np.random.default_rng(5)
    X = rng.uniform(-1, 1, (4000, 40)).astype(np.float32)
    dY = rng.uniform(-1, 1, (4000, 12)).astype(np.float32)
    W0 = rng.uniform(-1, 1, (12, 40)).astype(np.float32)
    dW = dev(W0)
    ops.dense_grad(dev(X), dev(dY), bias=False, dW=dW, accumulate=True)
    np.testing.assert_allclose(host(dW), W0 + dY.astype(np.float64).T @ X, atol=2e-4, rtol=1e-5)


@pytest.mark.parametrize("K,M", [(47, 1), (40, 12)])
def test_dense_grad_row_strides(K, M):
    """Row-padded / strided X and dY (NaN in the skipped columns) with accumulate."""
    rng = np.random.default_rng(K + M)
    N = 30000
    X = rng.uniform(-1, 1, (N, K)).astype(np.float32)
    dY = rng.uniform(-1, 1, (N, M)).astype(np.float32)
    Xb = torch.full((N, K + 5), float("nan"), device=DEV)
    Xb[:, :K] = dev(X)
    Yb = torch.full((N, M + 3), float("nan"), device=DEV)
    Yb[:, :M] = dev(dY)
    W0 = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    dW = dev(W0)
    db = torch.zeros(M, device=DEV)
    ops.dense_grad(Xb[:, :K], Yb[:, :M], dW=dW, db=db, accumulate=True)
    np.testing.assert_allclose(host(dW), W0 + dY.astype(np.float64).T @ X, atol=2e-4, rtol=1e-5)
    np.testing.assert_allclose(host(db), dY.astype(np.float64).sum(0), atol=1e-5 * N, rtol=1e-5)


def _padded(a, F, fill):
    """[N, F] view of an [N, F rounded up to 4] buffer whose padding holds `fill`."""
    Fp = (F + 3) // 4 * 4
    buf = torch.full((a.shape[0], Fp), fill, device=DEV)
    buf[:, :F] = dev(a)
    return buf, buf[:, :F]


@pytest.mark.parametrize("F", [3, 7, 33, 45, 47, 62])
@pytest.mark.parametrize("hubs", [False, True])
def test_padded_rows_float4_path(F, hubs):
    """Row-padded operands (row stride F rounded up to 4, padding = NaN) take the float4
    path with a partial last vector: SpMM (plain and weighted) stays bit-exact, the GAT
    forward / backward (also with attention recompute) and SDDMM stay within TOL, and the
    output padding is never written."""
    g = powerlaw()
    og = to_oracle(g)
    dg = ops.DeviceGraph.from_host(g, split=False)
    if hubs:
        dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
        assert dg.split_rows > 10
    X = features(g.n_cols, F, seed=71)
    _, Xp = _padded(X, F, float("nan"))
    ybuf, Yp = _padded(np.zeros((g.n_rows, F), np.float32), F, 7.0)
    # bit-identical to the unpadded (narrower-vector) launch on the same plan, and bit-exact
    # vs the oracle (hub rows in REF order too)
    def check(Y, val=None):
        np.testing.assert_array_equal(Y, orc.spmm(to_oracle(g, val), X))
    ops.spmm(dg, Xp, out=Yp)
    np.testing.assert_array_equal(host(Yp), host(ops.spmm(dg, dev(X))))
    check(host(Yp))
    val = edge_values(g.nnz, seed=72)
    gw = dg.with_values(dev(val))
    ops.spmm(gw, Xp, out=Yp)
    np.testing.assert_array_equal(host(Yp), host(ops.spmm(gw, dev(X))))
    check(host(Yp), val)
    assert bool(torch.all(ybuf[:, F:] == 7.0))
    for mode in (_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED):
        aL = features(g.n_rows, 1, seed=73)
        aR = features(g.n_cols, 1, seed=74)
        Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=1, slope=0.2, mode=mode)
        Y, al = ops.gat_fwd(dg, dev(aL), dev(aR), Xp, slope=0.2, mode=mode, want_alpha=True)
        assert Y.stride(0) == (F + 3) // 4 * 4
        np.testing.assert_allclose(host(al), al_ref, **TOL)
        np.testing.assert_allclose(host(Y), Y_ref, **TOL)
        dY = features(g.n_rows, F, seed=75)
        _, dYp = _padded(dY, F, float("nan"))
        dz_ref, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=1, slope=0.2, mode=mode)
        daL, dz = ops.gat_bwd(dg, dev(aL), dev(aR), Xp, dYp, dev(al_ref), slope=0.2, mode=mode)
        np.testing.assert_allclose(host(daL), daL_ref, **TOL)
        if mode == _abi.GALA_SOFTMAX_FIXED:
            np.testing.assert_allclose(host(dz), dz_ref, **TOL)
        wR = features(1, F, seed=76).ravel() * 0.5
        bR = np.array([0.1], np.float32)
        aR2 = (X.astype(np.float64) @ wR.astype(np.float64) + 0.1).astype(np.float32)
        Y2_ref, al2_ref = orc.gat_fwd(og, aL, aR2, X, heads=1, slope=0.2, mode=mode)
        Y2, al2 = ops.gat_fwd_attn(dg, dev(aL), dev(wR), dev(bR), Xp, slope=0.2, mode=mode, want_alpha=True)
        np.testing.assert_allclose(host(al2), al2_ref, **TOL)
        np.testing.assert_allclose(host(Y2), Y2_ref, **TOL)
        if mode == _abi.GALA_SOFTMAX_REF:
            _, daL2_ref = orc.gat_bwd(og, aL, aR2, X, dY, al2_ref, heads=1, slope=0.2, mode=mode)
            daL2 = ops.gat_bwd_attn(dg, dev(aL), dev(wR), dev(bR), Xp, dYp, dev(al2_ref), slope=0.2)
            np.testing.assert_allclose(host(daL2), daL2_ref, **TOL)
    A = features(g.n_rows, F, seed=77)
    _, Ap = _padded(A, F, float("nan"))
    np.testing.assert_allclose(host(ops.sddmm(dg, Ap, Xp)), orc.sddmm(og, A, X), **TOL)


def test_pad_rows_helper():
    X = torch.arange(2 * 47, dtype=torch.float32, device=DEV).reshape(2, 47)
    P = ops.pad_rows(X)
    assert P.shape == (2, 47) and P.stride(0) == 48 and torch.equal(P, X)
    assert ops.pad_rows(P) is P


def test_ops_capture_in_hip_graph():
    """The C ABI is stream-ordered with no host synchronisation or allocation inside, so a
    whole GCN + GAT step (hub-row split plan and row order included) captures into one HIP
    graph; replays on new inputs match eager execution bit for bit."""
    g = powerlaw()
    dg = ops.DeviceGraph.from_host(g, split=False)
    dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
    X = dev(features(g.n_cols, 32, seed=81))
    aL = dev(features(g.n_rows, 1, seed=82))
    aR = dev(features(g.n_cols, 1, seed=83))

    def step():
        norm = ops.degree(dg, power=-0.5)
        Y = ops.spmm(dg, ops.row_broadcast(norm, X), dst_scale=norm)
        Yg, al = ops.gat_fwd(dg, aL, aR, X, want_alpha=True)
        s = ops.sddvv(dg, aL, aR, op=2)
        return Y, Yg, al, ops.edge_softmax(dg, s)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up: workspaces allocated outside the capture
        step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        outs = step()
    for seed in (84, 85):
        X.copy_(dev(features(g.n_cols, 32, seed=seed)))
        graph.replay()
        want = step()
        for a, b in zip(outs, want):
            assert torch.equal(a, b)


@pytest.mark.parametrize("F", [1, 7, 32, 47, 128])
@pytest.mark.parametrize("padded", [False, True])
def test_row_scale_relu_matches_torch_chain(F, padded):
    """The GCN ReLU prologue pre * relu(act * X) and its backward are bit-identical to the
    torch ops they replace (mul, relu, mul; relu's threshold_backward, mul backward),
    including -0, NaN and exact zeros, and leave row padding untouched."""
    n = 3000
    rng = np.random.default_rng(F)
    X = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    X[::7, 0] = 0.0
    X[1::11, -1] = -0.0
    X[5, 0] = np.nan
    act = rng.uniform(0.1, 2, n).astype(np.float32)
    pre = rng.uniform(0.1, 2, n).astype(np.float32)
    G = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    if padded:
        xb, Xd = _padded(X, F, 5.0)
        _, Gd = _padded(G, F, 5.0)
    else:
        Xd, Gd = dev(X), dev(G)
    a, p = dev(act), dev(pre)
    for A, P in ((a, p), (None, p), (a, None), (None, None)):
        t = Xd if A is None else A[:, None] * Xd
        want = torch.relu(t) if P is None else P[:, None] * torch.relu(t)
        got = ops.row_scale_relu(Xd, A, P)
        assert torch.equal(torch.nan_to_num(got, nan=123.0), torch.nan_to_num(want, nan=123.0))
        assert torch.equal(torch.signbit(got), torch.signbit(want))
        r = torch.relu(t)
        dt = torch.where(r <= 0, torch.zeros_like(Gd), Gd)
        want_dx = dt if A is None else dt * A[:, None]
        got_dx = ops.relu_scale_backward(Xd, Gd, A)
        assert torch.equal(torch.nan_to_num(got_dx, nan=123.0), torch.nan_to_num(want_dx, nan=123.0))
    if padded:
        assert bool(torch.all(xb[:, F:] == 5.0))


@pytest.mark.parametrize("N,K,M", [(100000, 100, 32), (50000, 32, 47), (50000, 47, 32), (20000, 48, 128),
                                   (7000, 32, 172), (3000, 32, 256), (33, 7, 3), (1, 1, 1), (0, 16, 8),
                                   (4097, 5, 40),
                                   # W^T past 64 KB of LDS (the launch opts in to 160 KB)
                                   (20000, 128, 128), (5000, 100, 160)])
def test_ffn_fwd_matches_float64(N, K, M):
    """Y = X W^T + b on the matrix cores: |err| <= 1e-5 * sum_k |x w| + 1e-6 (fp32 chain)."""
    rng = np.random.default_rng(N + 7 * K + M)
    X = rng.uniform(-1, 1, (N, K)).astype(np.float32)
    W = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    b = rng.uniform(-1, 1, M).astype(np.float32)
    Y = host(ops.ffn_fwd(dev(X), dev(W), dev(b)))
    want = X.astype(np.float64) @ W.astype(np.float64).T + b
    mass = np.abs(X.astype(np.float64)) @ np.abs(W.astype(np.float64)).T + np.abs(b)
    assert np.all(np.abs(Y - want) <= 1e-5 * mass + 1e-6)
    Y2 = host(ops.ffn_fwd(dev(X), dev(W), None))  # no bias, and deterministic
    assert np.all(np.abs(Y2 - (want - b)) <= 1e-5 * mass + 1e-6)


def test_ffn_fwd_strided_and_unsupported():
    rng = np.random.default_rng(3)
    X = rng.uniform(-1, 1, (5000, 47)).astype(np.float32)
    W = rng.uniform(-1, 1, (40, 47)).astype(np.float32)
    Xb = torch.full((5000, 48), float("nan"), device=DEV)
    Xb[:, :47] = dev(X)
    Yb = torch.full((5000, 44), 7.0, device=DEV)
    ops.ffn_fwd(Xb[:, :47], dev(W), out=Yb[:, :40])
    np.testing.assert_allclose(host(Yb[:, :40]), X.astype(np.float64) @ W.T.astype(np.float64), atol=1e-4, rtol=1e-5)
    assert bool(torch.all(Yb[:, 40:] == 7.0))
    with pytest.raises(_abi.GalaError):
        ops.ffn_fwd(dev(rng.uniform(-1, 1, (10, 602)).astype(np.float32)),
                    dev(rng.uniform(-1, 1, (256, 602)).astype(np.float32)))


# ---- factored attention output (p, q) and the head-distributed forward ------------------
@pytest.mark.parametrize("F,heads", [(32, 1), (47, 1), (256, 8), (64, 4), (24, 3), (16, 8), (128, 2), (256, 2)])
@pytest.mark.parametrize("split", [False, True])
def test_gat_factored_alpha_bitexact(F, heads, split):
    """REF mode, gala_gat_fwd_ex_f32 with q_out: alpha_out = p, q_out = 1/(sum + 1e-12),
    and p * q (rounded) is BIT-identical to the materialised alpha of gala_gat_fwd_f32; Y
    is identical too.  The backward on (p, q) equals the backward on alpha bit for bit, and
    so does the dX SpMM over val = p with val_row_scale = q.  Against the oracle within the
    tolerance (hub-row plan included).  The head widths give 1, 2, 4, 8, 16 and 32 lanes per
    head: every DPP lane exchange (lane_xor, group_bcast) and the ds_swizzle / shuffle ones."""
    g = powerlaw()
    aL = features(g.n_rows, heads, seed=71)
    aR = features(g.n_cols, heads, seed=72)
    X = features(g.n_cols, F, seed=73)
    dY = features(g.n_rows, F, seed=74)
    dg = ops.DeviceGraph.from_host(g, split=False)
    if split:
        dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
    Y, al = ops.gat_fwd(dg, dev(aL), dev(aR), dev(X), heads=heads, want_alpha=True)
    Y2, p, q = ops.gat_fwd_ex(dg, dev(aL), dev(X), aR=dev(aR), heads=heads, factored=True)
    assert torch.equal(Y, Y2)
    rows = torch.from_numpy(np.repeat(np.arange(g.n_rows), np.diff(g.rowptr))).to(DEV)
    alpha_f = (p.view(-1, heads) * q.view(-1, heads)[rows]).reshape(-1)
    assert torch.equal(alpha_f, al)
    Y_ref, al_ref = orc.gat_fwd(to_oracle(g), aL, aR, X, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    np.testing.assert_allclose(host(Y2), Y_ref, **TOL)
    np.testing.assert_allclose(host(alpha_f), al_ref, **TOL)
    if 64 % heads == 0:   # the fused backward needs heads | lanes
        d1, _ = ops.gat_bwd(dg, dev(aL), dev(aR), dev(X), dev(dY), al, heads=heads)
        d2, _ = ops.gat_bwd_ex(dg, dev(aL), dev(X), dev(dY), p, q=q, aR=dev(aR), heads=heads)
        assert torch.equal(d1, d2)
    s1 = ops.spmm(dg.with_values(al, val_heads=heads), dev(dY))
    s2 = ops.spmm(dg.with_values(p, val_heads=heads, row_scale=q), dev(dY))
    assert torch.equal(s1, s2)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
@pytest.mark.parametrize("F,heads", [(256, 8), (64, 4), (32, 2), (48, 3), (128, 2), (256, 2), (16, 8)])
def test_gat_multihead_attention_recompute(graph, mode, F, heads):
    """gala_gat_fwd_ex_f32 with aR recomputed per head, aR[j,h] = <X[j, head h], wR[head h]>
    + bR[h] (the multi-head GAT layer's source logit), against the oracle chain on that aR
    (float64, rounded to fp32); REF backward with the same recompute on (p, q)."""
    D = F // heads
    aL = features(graph.n_rows, heads, seed=81)
    X = features(graph.n_cols, F, seed=83)
    dY = features(graph.n_rows, F, seed=84)
    wR = features(1, F, seed=85).ravel() * 0.5
    bR = features(1, heads, seed=86).ravel() * 0.1
    aR = np.stack([X[:, h * D:(h + 1) * D].astype(np.float64) @ wR[h * D:(h + 1) * D].astype(np.float64) + bR[h]
                   for h in range(heads)], 1).astype(np.float32)
    og = to_oracle(graph)
    Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=mode)
    dg = ops.DeviceGraph.from_host(graph, split=False)
    if 64 % heads:      # alpha of heads that do not divide the row group needs aR itself
        with pytest.raises(_abi.GalaError):
            ops.gat_fwd_ex(dg, dev(aL), dev(X), wR=dev(wR), bR=dev(bR), heads=heads, mode=mode, want_alpha=True)
        Y = ops.gat_fwd_ex(dg, dev(aL), dev(X), wR=dev(wR), bR=dev(bR), heads=heads, mode=mode)
        np.testing.assert_allclose(host(Y), Y_ref, **TOL)
        return
    Y, al = ops.gat_fwd_ex(dg, dev(aL), dev(X), wR=dev(wR), bR=dev(bR), heads=heads, mode=mode, want_alpha=True)
    np.testing.assert_allclose(host(al), al_ref, **TOL)
    np.testing.assert_allclose(host(Y), Y_ref, **TOL)
    if mode == _abi.GALA_SOFTMAX_REF and heads in (1, 2, 4, 8):  # fused backward: heads | lanes
        _, p, q = ops.gat_fwd_ex(dg, dev(aL), dev(X), wR=dev(wR), bR=dev(bR), heads=heads, factored=True)
        _, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=heads, slope=0.2, mode=mode)
        daL, _ = ops.gat_bwd_ex(dg, dev(aL), dev(X), dev(dY), p, q=q, wR=dev(wR), bR=dev(bR), heads=heads)
        np.testing.assert_allclose(host(daL), daL_ref, **TOL)


def test_gat_ex_rejects_bad_arguments():
    g = cora_like()
    dg = ops.DeviceGraph.from_host(g, split=False)
    aL, X = dev(features(g.n_rows, 1)), dev(features(g.n_cols, 32))
    with pytest.raises(_abi.GalaError):    # factored output is REF only
        ops.gat_fwd_ex(dg, aL, X, aR=dev(features(g.n_cols, 1)), mode=_abi.GALA_SOFTMAX_FIXED, factored=True)
    with pytest.raises(_abi.GalaError):    # recompute needs wR
        ops.gat_fwd_ex(dg, aL, X)
    with pytest.raises(_abi.GalaError):    # val_row_scale without values
        ops.spmm(ops.DeviceGraph(g.n_rows, g.n_cols, dg.rowptr, dg.col, None, val_row_scale=aL), X)


@pytest.mark.parametrize("F,heads", [(32, 1), (47, 1), (256, 8), (64, 4), (24, 3)])
@pytest.mark.parametrize("layout_", ["plain", "tiled", "split"])
@pytest.mark.parametrize("rc", [False, True])
def test_gat_bwd_fused_recompute(F, heads, layout_, rc):
    """gala_gat_bwd_fused_f32: alpha recomputed from (aL, aR | wR, bR) and the forward's q
    (gala_gat_fwd_ex_f32 with q_out only).  dX is BIT-identical to the SpMM over the
    materialised alpha; d_aL matches the alpha-based fused backward and the oracle within
    the tolerance.  Plain, column-tiled and hub-row-split graphs."""
    if rc and 64 % heads:
        pytest.skip("recompute with heads that do not divide the row group: covered by the forward test")
    g = powerlaw()
    if layout_ == "tiled":
        g = layout.col_tile(g, 1000)
    D = F // heads
    aL = features(g.n_rows, heads, seed=91)
    X = features(g.n_cols, F, seed=93)
    dY = features(g.n_rows, F, seed=94)
    if rc:
        wR = features(1, F, seed=95).ravel() * 0.5
        bR = features(1, heads, seed=96).ravel() * 0.1
        aR = np.stack([X[:, h * D:(h + 1) * D].astype(np.float64) @ wR[h * D:(h + 1) * D].astype(np.float64) + bR[h]
                       for h in range(heads)], 1).astype(np.float32)
        kw = dict(wR=dev(wR), bR=dev(bR))
    else:
        aR = features(g.n_cols, heads, seed=92)
        kw = dict(aR=dev(aR))
    dg = ops.DeviceGraph.from_host(g, split=False)
    if layout_ == "split":
        dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
    Y, q = ops.gat_fwd_ex(dg, dev(aL), dev(X), heads=heads, factored="q", **kw)
    Y2, p, q2 = ops.gat_fwd_ex(dg, dev(aL), dev(X), heads=heads, factored=True, **kw)
    if layout_ == "split" and 8 % heads:
        # alpha_out of heads that do not divide the row group runs hub rows unsplit
        torch.testing.assert_close(Y, Y2, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(q, q2, rtol=1e-5, atol=1e-6)
    else:
        assert torch.equal(Y, Y2) and torch.equal(q, q2)
    dX, daL = ops.gat_bwd_fused(dg, dev(aL), dev(X), dev(dY), q, heads=heads, **kw)
    # the GAT kernels sum hub rows as chunk partials: the SpMM in the same (fast) mode
    dX_ref = ops.spmm(dg.with_values(p, val_heads=heads, row_scale=q), dev(dY), hub="chunked")
    assert torch.equal(dX, dX_ref)
    og = to_oracle(g)
    _, al_ref = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    _, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    np.testing.assert_allclose(host(daL), daL_ref, **TOL)
    with pytest.raises(_abi.GalaError):   # dY[col] needs a square pattern
        rect = ops.DeviceGraph(g.n_rows, g.n_rows + 5, dg.rowptr, dg.col, n_seg=dg.n_seg, bounds=dg.bounds)
        ops.gat_bwd_fused(rect, dev(aL), dev(np.vstack([X, X[:5]])), dev(dY), q, heads=heads, **kw)


@pytest.mark.parametrize("F,heads", [(32, 1), (47, 1), (256, 8), (64, 4), (100, 1), (128, 2), (256, 2)])
@pytest.mark.parametrize("layout_", ["plain", "tiled", "split"])
@pytest.mark.parametrize("rc", [False, True])
def test_gat_row_stats(F, heads, layout_, rc):
    """gala_gat_fwd_stats_f32 / gala_gat_bwd_stats_f32: Y and q BIT-identical to the
    factored forward, dX BIT-identical to the recomputed fused backward (so the RC forward's
    aR_out equals the per-edge recompute), d_aL within the tolerance of the oracle's
    edge-by-edge REF chain; Ym and sma against a float64 restatement."""
    g = powerlaw()
    if layout_ == "tiled":
        g = layout.col_tile(g, 1000)
    D = F // heads
    aL = features(g.n_rows, heads, seed=91)
    X = features(g.n_cols, F, seed=93)
    dY = features(g.n_rows, F, seed=94)
    if rc:
        wR = features(1, F, seed=95).ravel() * 0.5
        bR = features(1, heads, seed=96).ravel() * 0.1
        aR = np.stack([X[:, h * D:(h + 1) * D].astype(np.float64) @ wR[h * D:(h + 1) * D].astype(np.float64) + bR[h]
                       for h in range(heads)], 1).astype(np.float32)
        kw = dict(wR=dev(wR), bR=dev(bR))
    else:
        aR = features(g.n_cols, heads, seed=92)
        kw = dict(aR=dev(aR))
    dg = ops.DeviceGraph.from_host(g, split=False)
    if layout_ == "split":
        dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
    out = ops.gat_fwd_stats(dg, dev(aL), dev(X), heads=heads, want_aR=rc, want_p=True, **kw)
    Y, q, Ym, sma = out[:4]
    pe = out[-1]
    Y0, q0 = ops.gat_fwd_ex(dg, dev(aL), dev(X), heads=heads, factored="q", **kw)
    assert torch.equal(Y, Y0) and torch.equal(q, q0)
    aRd = out[4] if rc else dev(aR)
    if rc:  # the recomputed logits: the float64 Linear within fp32 rounding
        np.testing.assert_allclose(host(aRd).reshape(-1, heads), aR, rtol=1e-5, atol=1e-5)
    # Ym, sma: sum_e m_e alpha_e X[col], sum_e m_e alpha_e (float64 restatement)
    og = to_oracle(g)
    _, al_ref = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    rows = np.repeat(np.arange(g.n_rows), np.diff(g.rowptr[:g.n_rows + 1]).astype(np.int64)) \
        if g.n_seg == 1 else None
    if rows is not None:
        t = aL[rows].astype(np.float64) + aR[g.col].astype(np.float64)
        m = np.where(t > 0, 1.0, 0.2)
        ma = m * al_ref.reshape(-1, heads).astype(np.float64)
        sma_ref = np.zeros((g.n_rows, heads))
        np.add.at(sma_ref, rows, ma)
        Ym_ref = np.zeros((g.n_rows, F))
        np.add.at(Ym_ref, rows, np.repeat(ma, D, axis=1) * X[g.col].astype(np.float64))
        np.testing.assert_allclose(host(sma).reshape(-1, heads), sma_ref, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(host(Ym), Ym_ref, rtol=1e-4, atol=1e-4)
    dX, daL = ops.gat_bwd_stats(dg, dev(aL), aRd, dev(dY), q, Y, Ym, sma, heads=heads)
    dX0, daL0 = ops.gat_bwd_fused(dg, dev(aL), dev(X), dev(dY), q, heads=heads, **kw)
    assert torch.equal(dX, dX0)
    # the forward's p (exp terms in edge order) instead of aR: the same alpha, the same dX
    _, p_ref, _ = ops.gat_fwd_ex(dg, dev(aL), dev(X), heads=heads, factored=True, **kw)
    assert torch.equal(pe, p_ref)
    dXp, daLp = ops.gat_bwd_stats(dg, dev(aL), None, dev(dY), q, Y, Ym, sma, heads=heads, p=pe)
    assert torch.equal(dXp, dX) and torch.equal(daLp, daL)
    _, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    np.testing.assert_allclose(host(daL), daL_ref, **TOL)
    np.testing.assert_allclose(host(daL), host(daL0), **TOL)


def test_gat_row_stats_rejects_bad_arguments():
    g = cora_like()
    dg = ops.DeviceGraph.from_host(g, split=False)
    aL, X = dev(features(g.n_rows, 1)), dev(features(g.n_cols, 32))
    aR = dev(features(g.n_cols, 1))
    with pytest.raises(_abi.GalaError):    # a rectangular pattern: no dY[col] / own-row logits
        rect = ops.DeviceGraph(g.n_rows, g.n_rows + 5, dg.rowptr, dg.col)
        ops.gat_fwd_stats(rect, aL, dev(features(g.n_rows + 5, 32)), aR=dev(features(g.n_rows + 5, 1)))
    with pytest.raises(_abi.GalaError):    # aR_out only with the recompute
        ops.gat_fwd_stats(dg, aL, X, aR=aR, want_aR=True)
    Y, q, Ym, sma = ops.gat_fwd_stats(dg, aL, X, aR=aR)
    with pytest.raises(_abi.GalaError):    # the backward reads aR explicitly
        ops.gat_bwd_stats(dg, aL, None, dev(features(g.n_rows, 32)), q, Y, Ym, sma)


@pytest.mark.parametrize("F,heads", [(256, 8), (47, 1), (64, 4), (24, 3), (100, 1)])
def test_head_attn(F, heads):
    """gala_head_attn_f32 within fp32 rounding of the CPU twin's sequential chain (lane
    chains + a butterfly; F = 47 and 100 on a power of two of lanes with the ones past D
    idle); its backward bit-exact against float32 numpy (one product, one sum)."""
    N = 3001
    X = features(N, F, seed=71)
    w = features(1, F, seed=72).ravel()
    b = features(1, heads, seed=73).ravel()
    D = F // heads
    out = ops.head_attn(dev(X), dev(w), dev(b), heads=heads)
    ref = np.empty((N, heads), np.float32)
    _abi.call_cpu("gala_head_attn_f32", N, F, heads, X.ctypes.data, F, w.ctypes.data, b.ctypes.data,
                  ref.ctypes.data, None)
    np.testing.assert_allclose(host(out), ref, rtol=1e-5, atol=1e-5)
    g = features(N, heads, seed=74)
    m = np.repeat(g, D, axis=1) * w[None, :]
    assert np.array_equal(host(ops.head_attn_bwd(dev(g), dev(w), heads=heads)), m)
    dX0 = features(N, F, seed=75)
    assert np.array_equal(host(ops.head_attn_bwd(dev(g), dev(w), heads=heads, dX=dev(dX0))), dX0 + m)


@pytest.mark.parametrize("F,heads", [(32, 1), (256, 8), (64, 4)])
@pytest.mark.parametrize("split", [False, True])
def test_gat_row_stats_aR_from_self_loop(F, heads, split):
    """The statistics forward takes each row's own recomputed source logit (aR_out) from
    the row's self-loop edge instead of re-reading X[row]; rows without a self-loop (and hub
    rows) read X[row].  Both paths must give the same bits: a graph with every self-loop and
    the same graph with the self-loops of every other row removed give identical aR_out,
    and the backward over either stays bit-identical to the per-edge recompute."""
    g1 = powerlaw()
    rows = np.repeat(np.arange(g1.n_rows), np.diff(g1.rowptr).astype(np.int64))
    loops = rows == g1.col
    assert np.array_equal(np.unique(rows[loops]), np.arange(g1.n_rows))   # every row has a self-loop
    keep = ~(loops & (rows % 2 == 0))
    g2 = layout.csr_build(g1.n_rows, g1.n_cols, rows[keep].astype(np.int32), g1.col[keep])
    X = dev(features(g1.n_cols, F, seed=93))
    dY = dev(features(g1.n_rows, F, seed=94))
    aL = dev(features(g1.n_rows, heads, seed=91))
    kw = dict(wR=dev(features(1, F, seed=95).ravel() * 0.5), bR=dev(features(1, heads, seed=96).ravel() * 0.1))
    aRs = []
    for g in (g1, g2):
        dg = ops.DeviceGraph.from_host(g, split=False)
        if split:
            dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
        Y, q, Ym, sma, aRo = ops.gat_fwd_stats(dg, aL, X, heads=heads, want_aR=True, **kw)
        dX, _ = ops.gat_bwd_stats(dg, aL, aRo, dY, q, Y, Ym, sma, heads=heads)
        dX0, _ = ops.gat_bwd_fused(dg, aL, X, dY, q, heads=heads, **kw)
        assert torch.equal(dX, dX0)
        aRs.append(aRo)
    assert torch.equal(aRs[0], aRs[1])


def _split_by_column(g, keep):
    sel = keep(g.col)
    rp = np.concatenate([[0], np.cumsum(sel)])[g.rowptr].astype(np.int32)
    return layout.HostGraph(g.n_rows, g.n_cols, rp, g.col[sel].astype(np.int32))


@pytest.mark.parametrize("F,heads", [(32, 1), (47, 1), (256, 8), (64, 4)])
@pytest.mark.parametrize("rc", [False, True])
def test_gat_continue_matches_one_pass(F, heads, rc):
    """gala_gat_fwd_continue_f32: the even columns' partials (gala_gat_fwd_partial_stats_f32 /
    GALA_GAT_PARTIAL), then the odd columns continued from them in place -- hub rows cut into
    chunks on both halves (threshold 64, 32-edge chunks: the fixup starts from the partials)
    -- equal the one-pass statistics forward and the plain REF forward to fp32 rounding."""
    g = powerlaw()
    aL = dev(features(g.n_rows, heads, seed=71))
    X = dev(features(g.n_cols, F, seed=73))
    wR = dev(features(1, F, seed=74).ravel() * 0.5)
    bR = dev(features(1, heads, seed=75).ravel())
    aR = None if rc else ops.head_attn(X, wR, bR, heads=heads)
    kw = {"wR": wR, "bR": bR} if rc else {}
    dg = ops.DeviceGraph.from_host(g)
    want = ops.gat_fwd_stats(dg, aL, X, aR=aR, heads=heads, **kw)[:4]
    halves = []
    for keep in (lambda c: c % 2 == 0, lambda c: c % 2 == 1):
        h = _split_by_column(g, keep)
        d = ops.DeviceGraph.from_host(h, split=False)
        d.set_split_plan(h.rowptr, 64, chunk=32, row_order=True)
        assert d.split_rows > 5
        halves.append(d)
    U, S, Um, M = ops.gat_fwd_partial_stats(halves[0], aL, X, aR=aR, heads=heads, **kw)
    got = ops.gat_fwd_continue(halves[1], aL, X, U, S, aR=aR, heads=heads, Um0=Um, M0=M, **kw)
    assert got[0].data_ptr() == U.data_ptr() and got[3].data_ptr() == M.data_ptr()   # in place
    for a, b in zip(got, want):
        torch.testing.assert_close(a.reshape(-1), b.reshape(-1), rtol=2e-5, atol=1e-6)
    # three ranges, the middle one continued unnormalised (GALA_GAT_PARTIAL)
    thirds = [ops.DeviceGraph.from_host(_split_by_column(g, lambda c, r=r: c % 3 == r)) for r in range(3)]
    U, S, Um, M = ops.gat_fwd_partial_stats(thirds[0], aL, X, aR=aR, heads=heads, **kw)
    ops.gat_fwd_continue(thirds[1], aL, X, U, S, aR=aR, heads=heads, Um0=Um, M0=M, partial=True, **kw)
    got = ops.gat_fwd_continue(thirds[2], aL, X, U, S, aR=aR, heads=heads, Um0=Um, M0=M, **kw)
    for a, b in zip(got, want):
        torch.testing.assert_close(a.reshape(-1), b.reshape(-1), rtol=2e-5, atol=1e-6)
    Ar = aR if aR is not None else ops.head_attn(X, wR, bR, heads=heads)
    Y, s = ops.gat_fwd_partial(halves[0], aL, X, aR=Ar, heads=heads)
    Y, q = ops.gat_fwd_continue(halves[1], aL, X, Y, s, aR=Ar, heads=heads)
    torch.testing.assert_close(Y, want[0], rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(q.reshape(-1), want[1].reshape(-1), rtol=2e-5, atol=0.0)


@pytest.mark.parametrize("F,heads", [(32, 1), (47, 1), (256, 8), (64, 4)])
@pytest.mark.parametrize("split", [False, True])
def test_gat_bwd_stats_linear_bitexact(F, heads, split):
    """gala_gat_bwd_stats_linear_f32: the attention Linear's dX term folded into the statistics
    backward's store equals gala_gat_bwd_stats_f32 followed by gala_head_attn_bwd_f32
    accumulating into dX, bit for bit -- hub rows included (the fixup adds it), d_aL
    unchanged."""
    g = powerlaw()
    aL = dev(features(g.n_rows, heads, seed=81))
    X = dev(features(g.n_cols, F, seed=82))
    dY = dev(features(g.n_rows, F, seed=83))
    wR = dev(features(1, F, seed=84).ravel() * 0.5)
    bR = dev(features(1, heads, seed=85).ravel())
    dg = ops.DeviceGraph.from_host(g, split=False)
    if split:
        dg.set_split_plan(g.rowptr, 64, chunk=32, row_order=True)
    Y, q, Ym, sma, aR = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=heads, want_aR=True)
    dX0, daL0 = ops.gat_bwd_stats(dg, aL, aR, dY, q, Y, Ym, sma, heads=heads)
    ops.head_attn_bwd(daL0.view(-1, heads), wR, heads=heads, dX=dX0, n_rows=g.n_rows)
    dX1, daL1 = ops.gat_bwd_stats(dg, aL, aR, dY, q, Y, Ym, sma, heads=heads, wR=wR)
    assert torch.equal(daL1, daL0)
    assert torch.equal(dX1, dX0)
