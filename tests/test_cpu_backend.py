"""CPU: the host-CPU backend libgala_cpu.so (include/gala_cpu.h)
against the oracle, through its C ABI (host pointers).

Bar, as for the HIP library: bit-exact for SpMM / degree / SDDVV / row-scale /
row-broadcast / edge permutation (same per-row CSR order and rounding steps as the
reference kernels), |err| <= 1e-4 (abs) + 1e-4 (rel) for the reductions (row-sum, SDDMM,
softmax, fused GAT forward / backward, dense gradients).
"""
import ctypes

import numpy as np
import pytest

import oracle as orc
from gala import _abi, layout
from _graphs import cora_like, edge_values, features, powerlaw, to_oracle, with_empty_rows

TOL = dict(atol=1e-4, rtol=1e-4)
GRAPHS = {"cora": cora_like, "powerlaw": powerlaw, "empty_rows": with_empty_rows}


@pytest.fixture(scope="module", params=list(GRAPHS))
def graph(request):
    return GRAPHS[request.param]()


def P(a):
    return None if a is None else a.ctypes.data


class HostCsr:
    """gala_csr_t over numpy arrays (kept alive with the struct)."""

    def __init__(self, g: layout.HostGraph, val=None, heads=1):
        self.g, self.val = g, (None if val is None else np.ascontiguousarray(val, np.float32))
        c = _abi.gala_csr_t()
        c.n_rows, c.n_cols, c.nnz = g.n_rows, g.n_cols, g.nnz
        c.rowptr, c.col, c.val = P(g.rowptr), P(g.col), P(self.val)
        c.val_heads, c.n_seg = heads, g.n_seg
        c.seg_bounds = None if g.bounds is None else g.bounds.ctypes.data
        c.split = None
        self.c = c

    @property
    def ref(self):
        return ctypes.byref(self.c)


def spmm_cpu(g, X, val=None, heads=1, src=None, dst=None, Y=None, accum=False, nsamp=None):
    F = X.shape[1]
    Y = np.zeros((g.n_rows, F), np.float32) if Y is None else Y
    flags = (_abi.GALA_SPMM_ACCUM if accum else 0) | (_abi.GALA_SPMM_SAMPLE if nsamp is not None else 0)
    A = HostCsr(g, val, heads)
    _abi.call_cpu("gala_spmm_f32", A.ref, P(X), F, P(Y), F, F, P(src), P(dst), flags, nsamp or 0, 5, 7, None)
    return Y


def test_exports_every_operator():
    L = _abi.cpu_lib()
    for fn in _abi.CPU_OPS:
        assert hasattr(L, _abi.cpu_name(fn)), fn
    hdr = open(_abi.os.path.join(_abi._HERE, "..", "..", "include", "gala_cpu.h")).read()
    for fn in _abi.CPU_OPS:
        assert _abi.cpu_name(fn) + "(" in hdr, fn


@pytest.mark.parametrize("F", [1, 7, 32, 47, 100])
@pytest.mark.parametrize("weighted", [False, True])
def test_spmm_bitexact(graph, F, weighted):
    val = edge_values(graph.nnz) if weighted else None
    X = features(graph.n_cols, F)
    np.testing.assert_array_equal(spmm_cpu(graph, X, val), orc.spmm(to_oracle(graph, val), X))


def test_spmm_scales_accum_tiled_sampled():
    g = cora_like()
    X = features(g.n_cols, 32)
    n = features(g.n_rows, 1, seed=3).ravel() + 2.0
    Y0 = features(g.n_rows, 32, seed=4)
    got = spmm_cpu(g, X, src=n, dst=n, Y=Y0.copy(), accum=True)
    np.testing.assert_array_equal(got, orc.spmm(to_oracle(g), X, src_scale=n, dst_scale=n, Y=Y0.copy(), accum=True))
    t = layout.col_tile(g, 1000)
    np.testing.assert_array_equal(spmm_cpu(t, X), orc.spmm(to_oracle(t), X))
    np.testing.assert_array_equal(spmm_cpu(t, X, nsamp=20), orc.spmm(to_oracle(t), X, sample=True, nsamp=20))


def test_spmm_multihead_weights():
    g = powerlaw()
    val = edge_values(g.nnz, heads=4)
    X = features(g.n_cols, 64)
    np.testing.assert_array_equal(spmm_cpu(g, X, val, heads=4), orc.spmm(to_oracle(g, val, heads=4), X))


@pytest.mark.parametrize("power", [1.0, -0.5])
@pytest.mark.parametrize("weighted", [False, True])
def test_degree(graph, power, weighted):
    val = edge_values(graph.nnz) if weighted else None
    out = np.empty(graph.n_rows, np.float32)
    _abi.call_cpu("gala_degree_f32", HostCsr(graph, val).ref, P(out), power, 0, 0, None)
    np.testing.assert_array_equal(out, orc.degree(to_oracle(graph, val), power=power))


@pytest.mark.parametrize("op", [0, 1, 2])
@pytest.mark.parametrize("heads", [1, 3, 8])
def test_sddvv(graph, op, heads):
    a = features(graph.n_rows, heads, seed=11)
    b = features(graph.n_cols, heads, seed=12)
    out = np.empty(graph.nnz * heads, np.float32)
    _abi.call_cpu("gala_sddvv_f32", HostCsr(graph).ref, P(a), P(b), heads, op, 0.2, P(out), None)
    np.testing.assert_array_equal(out, orc.sddvv(to_oracle(graph), a, b, heads=heads, op=op, slope=0.2))


@pytest.mark.parametrize("heads", [1, 8])
def test_row_sum_scale_broadcast(graph, heads):
    t = layout.col_tile(graph, 1000)
    v = edge_values(t.nnz, heads=heads, seed=5)
    out = np.empty(t.n_rows * heads, np.float32)
    _abi.call_cpu("gala_row_sum_f32", HostCsr(t).ref, P(v), heads, 1e-12, P(out), 0, None)
    np.testing.assert_allclose(out, orc.row_sum(to_oracle(t), v, heads=heads, eps=1e-12), **TOL)
    q = features(t.n_rows, heads, seed=6).ravel()
    vv = v.copy()
    _abi.call_cpu("gala_row_scale_f32", HostCsr(t).ref, P(q), heads, P(vv), None)
    np.testing.assert_array_equal(vv, orc.row_scale(to_oracle(t), q, v, heads=heads))
    X = features(graph.n_rows, 13)
    s = features(graph.n_rows, 1).ravel()
    Y = np.empty_like(X)
    _abi.call_cpu("gala_row_broadcast_f32", graph.n_rows, 13, P(s), P(X), 13, P(Y), 13, None)
    np.testing.assert_array_equal(Y, (s[:, None] * X).astype(np.float32))


@pytest.mark.parametrize("F,heads", [(1, 1), (32, 1), (47, 1), (256, 8), (12, 3)])
def test_sddmm(graph, F, heads):
    A = features(graph.n_rows, F, seed=21)
    B = features(graph.n_cols, F, seed=22)
    out = np.empty(graph.nnz * heads, np.float32)
    _abi.call_cpu("gala_sddmm_dot_f32", HostCsr(graph).ref, P(A), F, P(B), F, F, heads, P(out), None)
    np.testing.assert_allclose(out, orc.sddmm(to_oracle(graph), A, B, heads=heads), **TOL)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
@pytest.mark.parametrize("heads", [1, 3])
def test_edge_softmax(graph, mode, heads):
    g = layout.col_tile(graph, 1000)
    s = edge_values(g.nnz, heads=heads, lo=-3, hi=3, seed=8)
    d = edge_values(g.nnz, heads=heads, lo=-1, hi=1, seed=9)
    a = np.empty_like(s)
    _abi.call_cpu("gala_edge_softmax_fwd_f32", HostCsr(g).ref, P(s), heads, mode, P(a), None)
    a_ref = orc.softmax_fwd(to_oracle(g), s, heads=heads, mode=mode)
    np.testing.assert_allclose(a, a_ref, **TOL)
    ds = np.empty_like(s)
    _abi.call_cpu("gala_edge_softmax_bwd_f32", HostCsr(g).ref, P(a_ref), P(d), heads, mode, P(ds), None)
    np.testing.assert_allclose(ds, orc.softmax_bwd(to_oracle(g), a_ref, d, heads=heads, mode=mode), **TOL)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
@pytest.mark.parametrize("F,heads", [(32, 1), (47, 1), (64, 4)])
def test_gat_fwd_bwd(graph, mode, F, heads):
    aL = features(graph.n_rows, heads, seed=31)
    aR = features(graph.n_cols, heads, seed=32)
    X = features(graph.n_cols, F, seed=33)
    dY = features(graph.n_rows, F, seed=34)
    og = to_oracle(graph)
    Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=mode)
    Y = np.empty((graph.n_rows, F), np.float32)
    al = np.empty(graph.nnz * heads, np.float32)
    _abi.call_cpu("gala_gat_fwd_f32", HostCsr(graph).ref, P(aL), P(aR), P(X), F, F, heads, 0.2, mode,
                  P(Y), F, P(al), None)
    np.testing.assert_allclose(al, al_ref, **TOL)
    np.testing.assert_allclose(Y, Y_ref, **TOL)
    dz_ref, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=heads, slope=0.2, mode=mode)
    dz = np.empty(graph.nnz * heads, np.float32)
    daL = np.empty(graph.n_rows * heads, np.float32)
    _abi.call_cpu("gala_gat_bwd_f32", HostCsr(graph).ref, P(aL), P(aR), P(X), F, P(dY), F, F, heads, 0.2,
                  mode, P(al_ref), P(dz), P(daL), None)
    np.testing.assert_allclose(daL, daL_ref, **TOL)
    np.testing.assert_allclose(dz, dz_ref, **TOL)


@pytest.mark.parametrize("mode", [_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED])
def test_gat_attention_recompute(graph, mode):
    F = 47
    aL = features(graph.n_rows, 1, seed=51)
    X = features(graph.n_cols, F, seed=53)
    dY = features(graph.n_rows, F, seed=54)
    wR = features(1, F, seed=55).ravel() * 0.5
    bR = np.array([0.1], np.float32)
    aR = (X.astype(np.float64) @ wR.astype(np.float64) + 0.1).astype(np.float32)
    og = to_oracle(graph)
    Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=1, slope=0.2, mode=mode)
    Y = np.empty((graph.n_rows, F), np.float32)
    al = np.empty(graph.nnz, np.float32)
    _abi.call_cpu("gala_gat_fwd_attn_f32", HostCsr(graph).ref, P(aL), P(wR), P(bR), P(X), F, F, 0.2, mode,
                  P(Y), F, P(al), None)
    np.testing.assert_allclose(al, al_ref, **TOL)
    np.testing.assert_allclose(Y, Y_ref, **TOL)
    if mode == _abi.GALA_SOFTMAX_REF:
        _, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=1, slope=0.2, mode=mode)
        daL = np.empty(graph.n_rows, np.float32)
        _abi.call_cpu("gala_gat_bwd_attn_f32", HostCsr(graph).ref, P(aL), P(wR), P(bR), P(X), F, P(dY), F, F,
                      0.2, P(al_ref), P(daL), None)
        np.testing.assert_allclose(daL, daL_ref, **TOL)


@pytest.mark.parametrize("F,heads,rc", [(32, 1, False), (47, 1, True), (64, 4, False), (64, 4, True)])
def test_gat_row_stats(graph, F, heads, rc):
    """gala_cpu_gat_{fwd,bwd}_stats_f32: Y within tolerance of the oracle, dX = A_alpha dY,
    d_aL from the row statistics within tolerance of the oracle's edge-by-edge chain."""
    D = F // heads
    aL = features(graph.n_rows, heads, seed=61)
    X = features(graph.n_cols, F, seed=63)
    dY = features(graph.n_rows, F, seed=64)
    if rc:
        wR = features(1, F, seed=65).ravel() * 0.5
        bR = features(1, heads, seed=66).ravel() * 0.1
        aR = np.stack([X[:, h * D:(h + 1) * D].astype(np.float64) @ wR[h * D:(h + 1) * D].astype(np.float64) + bR[h]
                       for h in range(heads)], 1).astype(np.float32)
    else:
        wR = bR = None
        aR = features(graph.n_cols, heads, seed=62)
    og = to_oracle(graph)
    Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    n = graph.n_rows
    Y, Ym = np.empty((n, F), np.float32), np.empty((n, F), np.float32)
    q, sma = np.empty(n * heads, np.float32), np.empty(n * heads, np.float32)
    aR_out = np.empty(n * heads, np.float32) if rc else None
    pe = np.empty(graph.nnz * heads, np.float32)
    _abi.call_cpu("gala_gat_fwd_stats_f32", HostCsr(graph).ref, P(aL), None if rc else P(aR), P(wR), P(bR), P(X),
                  F, F, heads, 0.2, P(Y), F, P(q), P(Ym), F, P(sma), P(aR_out), P(pe), None)
    np.testing.assert_allclose(Y, Y_ref, **TOL)
    aRx = aR_out if rc else aR
    if rc:
        np.testing.assert_allclose(aR_out.reshape(n, heads), aR, rtol=1e-5, atol=1e-5)
    _, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    dX, daL = np.empty((n, F), np.float32), np.empty(n * heads, np.float32)
    _abi.call_cpu("gala_gat_bwd_stats_f32", HostCsr(graph).ref, P(aL), P(aRx), None, P(dY), F, F, heads, 0.2, P(q),
                  P(Y), F, P(Ym), F, P(sma), P(dX), F, P(daL), None)
    np.testing.assert_allclose(daL, daL_ref, **TOL)
    # alpha from the forward's p instead of aR: the same dX
    dXp = np.empty((n, F), np.float32)
    _abi.call_cpu("gala_gat_bwd_stats_f32", HostCsr(graph).ref, P(aL), None, P(pe), P(dY), F, F, heads, 0.2, P(q),
                  P(Y), F, P(Ym), F, P(sma), P(dXp), F, P(daL), None)
    assert np.array_equal(dXp, dX)
    gw = orc.Graph(og.n_rows, og.n_cols, og.rowptr, og.col, al_ref, og.n_seg, og.bounds, heads)
    np.testing.assert_allclose(dX, orc.spmm(gw, dY), **TOL)


@pytest.mark.parametrize("F,heads", [(256, 8), (47, 1), (64, 4), (24, 3)])
def test_head_attn(F, heads):
    """gala_cpu_head_attn_f32 against a float64 restatement; its backward bit-exact (one
    product and one sum per element, float32 numpy rounds the same way)."""
    N = 1000
    X = features(N, F, seed=71)
    w = features(1, F, seed=72).ravel()
    b = features(1, heads, seed=73).ravel()
    D = F // heads
    out = np.empty((N, heads), np.float32)
    _abi.call_cpu("gala_head_attn_f32", N, F, heads, P(X), F, P(w), P(b), P(out), None)
    ref = (X.astype(np.float64).reshape(N, heads, D) * w.astype(np.float64).reshape(1, heads, D)).sum(2) + b
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)
    g = features(N, heads, seed=74)
    dX = np.empty((N, F), np.float32)
    _abi.call_cpu("gala_head_attn_bwd_f32", N, F, heads, P(g), P(w), P(dX), F, 0, None)
    m = np.repeat(g, D, axis=1) * w[None, :]
    assert np.array_equal(dX, m)
    dX0 = features(N, F, seed=75)
    dX = dX0.copy()
    _abi.call_cpu("gala_head_attn_bwd_f32", N, F, heads, P(g), P(w), P(dX), F, 1, None)
    assert np.array_equal(dX, dX0 + m)


def test_edge_permute_and_dense_grad():
    g = powerlaw()
    t, perm = layout.transpose(g)
    v = edge_values(g.nnz, heads=2)
    out = np.empty_like(v)
    _abi.call_cpu("gala_edge_permute_f32", P(perm), P(v), g.nnz, 2, P(out), None)
    np.testing.assert_array_equal(out, v.reshape(-1, 2)[perm].ravel())
    N, K, M = 20000, 33, 17
    X = features(N, K, seed=1)
    dY = features(N, M, seed=2)
    ws_b = _abi.cpu_lib().gala_cpu_dense_grad_workspace(N, K, M)
    ws = np.empty(max(ws_b // 4, 1), np.float32)
    dW = np.empty((M, K), np.float32)
    db = np.empty(M, np.float32)
    _abi.call_cpu("gala_dense_grad_f32", N, K, M, P(X), K, P(dY), M, P(dW), P(db), 0, P(ws), ws_b, None)
    np.testing.assert_allclose(dW, dY.astype(np.float64).T @ X.astype(np.float64), atol=1e-3, rtol=1e-4)
    np.testing.assert_allclose(db, dY.astype(np.float64).sum(0), atol=1e-3, rtol=1e-4)


def test_status_codes_match_the_hip_abi():
    g = cora_like()
    A = HostCsr(g)
    X = features(g.n_cols, 4)
    Y = np.empty((g.n_rows, 4), np.float32)
    L = _abi.cpu_lib()
    assert L.gala_cpu_spmm_f32(A.ref, P(X), 4, P(Y), 4, -1, None, None, 0, 0, 5, 7, None) == _abi.GALA_ERR_INVALID_ARG
    assert L.gala_cpu_spmm_f32(A.ref, P(X), 4, P(Y), 4, 4, None, None, 0x80, 0, 5, 7, None) == _abi.GALA_ERR_INVALID_ARG
    assert L.gala_cpu_edge_softmax_fwd_f32(A.ref, P(X), 1, 7, P(Y), None) == _abi.GALA_ERR_INVALID_ARG
    bad = HostCsr(layout.col_tile(g, 1000))
    bad.g.bounds[1] = g.nnz + 5
    assert L.gala_cpu_spmm_f32(bad.ref, P(X), 4, P(Y), 4, 4, None, None, 0, 0, 5, 7, None) == _abi.GALA_ERR_GRAPH
    # the rowptr-count degree norm is refused on a weighted graph (its degree sums the values)
    W = HostCsr(g, val=edge_values(g.nnz))
    epi = _abi.gala_spmm_epilogue_t()
    epi.dst_deg_rsqrt = 1
    assert L.gala_cpu_spmm_ex_f32(W.ref, P(X), 4, P(Y), 4, 4, None, None, 0, 0, 5, 7, ctypes.byref(epi),
                                  None) == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_cpu_row_broadcast_deg_f32(W.ref, 4, P(X), 4, P(Y), 4, None) == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_cpu_row_broadcast_deg_f32(A.ref, 4, P(X), 4, P(Y), 4, None) == _abi.GALA_OK


def test_row_scale_relu_and_backward_match_numpy():
    """pre * relu(act * X) and act * (relu(act * X) <= 0 ? 0 : G), bit for bit (float32 numpy
    with the same rounding steps; torch.relu's GPU semantics: -0 -> +0, NaN passes)."""
    rng = np.random.default_rng(3)
    n, F = 500, 13
    X = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    X[::5, 0] = -0.0
    X[3, 2] = np.nan
    act = rng.uniform(0.1, 2, n).astype(np.float32)
    pre = rng.uniform(0.1, 2, n).astype(np.float32)
    G = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    Y = np.empty_like(X)
    _abi.call_cpu("gala_row_scale_relu_f32", n, F, P(act), P(pre), P(X), F, P(Y), F, None)
    t = act[:, None] * X
    r = np.where((t > 0) | np.isnan(t), t, np.float32(0))
    np.testing.assert_array_equal(Y, pre[:, None] * r)
    assert np.array_equal(np.signbit(Y), np.signbit(pre[:, None] * r))
    dX = np.empty_like(X)
    _abi.call_cpu("gala_relu_scale_backward_f32", n, F, P(act), P(X), F, P(G), F, P(dX), F, None)
    np.testing.assert_array_equal(dX, np.where(r <= 0, np.float32(0), G) * act[:, None])


@pytest.mark.parametrize("tiled", [0, 900, 20])
def test_spmm_relu_prologue_and_epilogue_match_the_passes(tiled):
    """gala_spmm_ex_f32's ReLU fields against the passes they fold, bit for bit: the source
    pre * relu(act * X) (gala_row_scale_relu_f32, then the SpMM) and the ReLU backward of the
    result (the SpMM, then gala_relu_scale_backward_f32), one segment and column-tiled;
    refusals on weighted / sampled graphs and for src_act without src_relu."""
    g = cora_like()
    A = HostCsr(layout.col_tile(g, tiled) if tiled else g)  # 20: 136 segments
    n, F = g.n_rows, 13
    rng = np.random.default_rng(8)
    X = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    X[::7, 0] = 0.0
    act = rng.uniform(0.1, 2, n).astype(np.float32)
    pre = rng.uniform(0.1, 2, n).astype(np.float32)
    post = rng.uniform(0.1, 2, n).astype(np.float32)
    Rx = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    L = _abi.cpu_lib()
    for a, s in ((act, pre), (None, pre), (act, None), (None, None)):
        H = np.empty_like(X)
        _abi.call_cpu("gala_row_scale_relu_f32", n, F, P(a), P(s), P(X), F, P(H), F, None)
        want = np.empty_like(X)
        _abi.call_cpu("gala_spmm_f32", A.ref, P(H), F, P(want), F, F, None, P(post), 0, 0, 5, 7, None)
        epi = _abi.gala_spmm_epilogue_t()
        epi.src_relu, epi.src_act = 1, P(a)
        got = np.empty_like(X)
        _abi.call_cpu("gala_spmm_ex_f32", A.ref, P(X), F, P(got), F, F, P(s), P(post), 0, 0, 5, 7,
                      ctypes.byref(epi), None)
        np.testing.assert_array_equal(got, want)
        G = np.empty_like(X)
        _abi.call_cpu("gala_spmm_f32", A.ref, P(X), F, P(G), F, F, P(s), P(post), 0, 0, 5, 7, None)
        _abi.call_cpu("gala_relu_scale_backward_f32", n, F, P(a), P(Rx), F, P(G), F, P(want), F, None)
        epi = _abi.gala_spmm_epilogue_t()
        epi.relu_x, epi.ldrx, epi.relu_act = P(Rx), F, P(a)
        _abi.call_cpu("gala_spmm_ex_f32", A.ref, P(X), F, P(got), F, F, P(s), P(post), 0, 0, 5, 7,
                      ctypes.byref(epi), None)
        np.testing.assert_array_equal(got, want)
    epi = _abi.gala_spmm_epilogue_t()
    epi.src_relu = 1
    W = HostCsr(g, val=edge_values(g.nnz))
    assert L.gala_cpu_spmm_ex_f32(W.ref, P(X), F, P(got), F, F, None, None, 0, 0, 5, 7, ctypes.byref(epi),
                                  None) == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_cpu_spmm_ex_f32(A.ref, P(X), F, P(got), F, F, None, None, _abi.GALA_SPMM_SAMPLE, 3, 5, 7,
                                  ctypes.byref(epi), None) == _abi.GALA_ERR_UNSUPPORTED
    epi = _abi.gala_spmm_epilogue_t()
    epi.src_act = P(act)
    assert L.gala_cpu_spmm_ex_f32(A.ref, P(X), F, P(got), F, F, None, None, 0, 0, 5, 7, ctypes.byref(epi),
                                  None) == _abi.GALA_ERR_INVALID_ARG
    epi = _abi.gala_spmm_epilogue_t()
    epi.relu_x, epi.ldrx = P(Rx), F - 1
    assert L.gala_cpu_spmm_ex_f32(A.ref, P(X), F, P(got), F, F, None, None, 0, 0, 5, 7, ctypes.byref(epi),
                                  None) == _abi.GALA_ERR_INVALID_ARG


@pytest.mark.parametrize("seed", range(24))
def test_random_case(seed):
    """Seeded random sweep of the host backend (the GPU suite runs the same generator through
    libgala_hip.so): random / R-MAT / empty-row / hub graphs, widths, 1-8 heads, strided
    operands; bit-exact degree / SpMM / tiled SpMM, TOL for the reductions and GAT."""
    import test_gpu_fuzz as fz
    rng = np.random.default_rng(5000 + seed)
    g = fz._graph(rng)
    og = to_oracle(g)
    heads = int(rng.choice([1, 1, 2, 4, 8]))
    D = int(rng.choice([1, 2, 4, 8, 16, 32])) if heads > 1 else int(rng.integers(1, 120))
    F = heads * D
    ld = F + int(rng.integers(0, 5))  # strided rows
    X = np.zeros((g.n_cols, ld), np.float32)
    X[:, :F] = rng.uniform(-1, 1, (g.n_cols, F))
    Xc = np.ascontiguousarray(X[:, :F])
    deg = np.empty(g.n_rows, np.float32)
    _abi.call_cpu("gala_degree_f32", HostCsr(g).ref, P(deg), 1.0, 0, 0, None)
    np.testing.assert_array_equal(deg, orc.degree(og))
    Y = np.full((g.n_rows, ld), 7.0, np.float32)
    _abi.call_cpu("gala_spmm_f32", HostCsr(g).ref, P(X), ld, P(Y), ld, F, None, None, 0, 0, 5, 7, None)
    np.testing.assert_array_equal(Y[:, :F], orc.spmm(og, Xc))
    assert np.all(Y[:, F:] == 7.0)
    if g.n_cols > 1:
        tg = layout.col_tile(g, int(rng.integers(1, g.n_cols)))
        np.testing.assert_array_equal(spmm_cpu(tg, Xc), orc.spmm(to_oracle(tg), Xc))
    if g.nnz == 0:
        return
    s = rng.uniform(-3, 3, g.nnz * heads).astype(np.float32)
    for mode in (_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED):
        a = np.empty_like(s)
        _abi.call_cpu("gala_edge_softmax_fwd_f32", HostCsr(g).ref, P(s), heads, mode, P(a), None)
        np.testing.assert_allclose(a, orc.softmax_fwd(og, s, heads=heads, mode=mode), **TOL)
    aL = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    aR = rng.uniform(-1, 1, (g.n_cols, heads)).astype(np.float32)
    dY = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    out = np.empty(g.nnz * heads, np.float32)
    _abi.call_cpu("gala_sddmm_dot_f32", HostCsr(g).ref, P(dY), F, P(X), ld, F, heads, P(out), None)
    np.testing.assert_allclose(out, orc.sddmm(og, dY, Xc, heads=heads), **TOL)
    for mode in (_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED):
        Y_ref, al_ref = orc.gat_fwd(og, aL, aR, Xc, heads=heads, slope=0.2, mode=mode)
        Yg = np.empty((g.n_rows, F), np.float32)
        al = np.empty(g.nnz * heads, np.float32)
        _abi.call_cpu("gala_gat_fwd_f32", HostCsr(g).ref, P(aL), P(aR), P(X), ld, F, heads, 0.2, mode,
                      P(Yg), F, P(al), None)
        np.testing.assert_allclose(al, al_ref, **TOL)
        np.testing.assert_allclose(Yg, Y_ref, **TOL)
        dz_ref, daL_ref = orc.gat_bwd(og, aL, aR, Xc, dY, al_ref, heads=heads, slope=0.2, mode=mode)
        dz = np.empty(g.nnz * heads, np.float32)
        daL = np.empty(g.n_rows * heads, np.float32)
        _abi.call_cpu("gala_gat_bwd_f32", HostCsr(g).ref, P(aL), P(aR), P(X), ld, P(dY), F, F, heads, 0.2,
                      mode, P(al_ref), P(dz), P(daL), None)
        np.testing.assert_allclose(daL, daL_ref, **TOL)
        if mode == _abi.GALA_SOFTMAX_FIXED:
            np.testing.assert_allclose(dz, dz_ref, **TOL)


def test_partial_stats_own_vertex_logits():
    """gala_cpu_gat_fwd_partial_stats_ex_f32: with self_col the recomputed logits of the own
    vertices are written (the vertex cut's backward reuses them); aR_out without self_col is
    refused for a partial pattern."""
    import torch
    from gala import vertex_cut as vc
    from gala.backend import CpuBackend
    g = powerlaw(n=1500, m=9000)
    H, F = 2, 16
    rng = np.random.default_rng(8)
    X = torch.from_numpy(rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32))
    aL = torch.from_numpy(rng.uniform(-1, 1, (g.n_rows, H)).astype(np.float32))
    wR = torch.from_numpy(rng.uniform(-0.5, 0.5, F).astype(np.float32))
    bR = torch.from_numpy(rng.uniform(-0.5, 0.5, H).astype(np.float32))
    be = CpuBackend()
    want = be.head_attn(X, wR, bR, H)        # the CPU twin recomputes with the same dot
    for exchange in ("dense", "sparse"):
        for p in range(3):
            pt = vc.vertex_cut_partition(g, p, 3, chunks=2, exchange=exchange)
            own = slice(pt.r0, pt.r0 + pt.n)
            got = torch.full((pt.n, H), float("nan"))
            hs = pt.sparse.send_graphs if exchange == "sparse" else pt.chunk_graphs
            for k, h in enumerate(hs):
                cg = be.graph(h)
                U, Um = torch.empty((h.n_rows, F)), torch.empty((h.n_rows, F))
                S, M = torch.empty(h.n_rows * H), torch.empty(h.n_rows * H)
                al = torch.zeros((h.n_rows, H))
                be.gat_partial_stats(cg, al, None, X[own].contiguous(), H, 0.2, U, S, Um, M, wR=wR, bR=bR,
                                     self_col=torch.from_numpy(pt.self_cols(k)), aR_out=got)
            np.testing.assert_allclose(got.numpy(), want[own].numpy(), rtol=1e-6, atol=1e-6)
    with pytest.raises(_abi.GalaError):
        cg = be.graph(pt.sparse.send_graphs[0])
        n0 = pt.sparse.send_graphs[0].n_rows
        _abi.call_cpu("gala_gat_fwd_partial_stats_ex_f32", cg.csr(), torch.zeros(n0 * H).data_ptr(), None,
                      wR.data_ptr(), bR.data_ptr(), X[own].contiguous().data_ptr(), F, F, H, 0.2,
                      torch.empty(n0, F).data_ptr(), F, torch.empty(n0 * H).data_ptr(), torch.empty(n0, F).data_ptr(),
                      F, torch.empty(n0 * H).data_ptr(), None, torch.empty(pt.n * H).data_ptr(), None)


def _split_by_column(g, keep):
    """The edges of g whose column satisfies keep(col), as a CSR over the same rows / columns."""
    sel = keep(g.col)
    rp = np.concatenate([[0], np.cumsum(sel)])[g.rowptr].astype(np.int32)
    return layout.HostGraph(g.n_rows, g.n_cols, rp, g.col[sel].astype(np.int32))


@pytest.mark.parametrize("rc", [False, True])
@pytest.mark.parametrize("which", ["powerlaw", "empty_rows"])
def test_gat_continue_matches_one_pass(rc, which):
    """gala_cpu_gat_fwd_continue_f32: partials over the even columns, then the odd columns
    continued from them in place, equal the one-pass statistics forward (Y, q, Ym, sma) and
    the plain REF forward to fp32 rounding; a half-given statistics pair is refused."""
    import torch
    from gala.backend import CpuBackend
    g = powerlaw(n=1500, m=9000) if which == "powerlaw" else with_empty_rows()
    H, F = 2, 16
    rng = np.random.default_rng(5)
    t = lambda a: torch.from_numpy(a.astype(np.float32))  # noqa: E731
    X, aL = t(rng.uniform(-1, 1, (g.n_rows, F))), t(rng.uniform(-1, 1, (g.n_rows, H)))
    wR, bR = t(rng.uniform(-0.5, 0.5, F)), t(rng.uniform(-0.5, 0.5, H))
    be = CpuBackend()
    aR = None if rc else be.head_attn(X, wR, bR, H)
    kw = {"wR": wR, "bR": bR} if rc else {}
    full = be.graph(g)
    want = be.gat_stats_table(full, aL, aR, X, H, 0.2, None, None, **kw)
    g0, g1 = (be.graph(_split_by_column(g, f)) for f in (lambda c: c % 2 == 0, lambda c: c % 2 == 1))
    U, Um, S, M = torch.empty((g.n_rows, F)), torch.empty((g.n_rows, F)), torch.empty(g.n_rows * H), \
        torch.empty(g.n_rows * H)
    be.gat_partial_stats(g0, aL, aR, X, H, 0.2, U, S, Um, M, **kw)
    got = be.gat_continue(g1, aL, aR, X, H, 0.2, U, S, Um, M, **kw)
    for a, b in zip(got, want):
        np.testing.assert_allclose(a.numpy().reshape(-1), b.numpy().reshape(-1), rtol=2e-5, atol=1e-6)
    Ar = aR if aR is not None else be.head_attn(X, wR, bR, H)
    Y, s = torch.empty((g.n_rows, F)), torch.empty(g.n_rows * H)
    be.gat_partial(g0, aL, Ar, X, H, 0.2, Y, s)
    Y, q = be.gat_continue(g1, aL, Ar, X, H, 0.2, Y, s)
    np.testing.assert_allclose(Y.numpy(), want[0].numpy(), rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(q.numpy(), want[1].numpy().reshape(-1), rtol=2e-5, atol=0)
    # three ranges: the middle one continued unnormalised (GALA_GAT_PARTIAL), the last normalises
    g3 = [be.graph(_split_by_column(g, lambda c, r=r: c % 3 == r)) for r in range(3)]
    U, S, Um, M = be.gat_partial_stats(g3[0], aL, aR, X, H, 0.2, U, S, Um, M, **kw)
    be.gat_continue(g3[1], aL, aR, X, H, 0.2, U, S, Um, M, partial=True, **kw)
    got = be.gat_continue(g3[2], aL, aR, X, H, 0.2, U, S, Um, M, **kw)
    for a, b in zip(got, want):
        np.testing.assert_allclose(a.numpy().reshape(-1), b.numpy().reshape(-1), rtol=2e-5, atol=1e-6)
    with pytest.raises(_abi.GalaError):
        _abi.call_cpu("gala_gat_fwd_continue_f32", g1.csr(), aL.data_ptr(), Ar.data_ptr(), None, None,
                      X.data_ptr(), F, F, H, 0.2, 0, U.data_ptr(), F, S.data_ptr(), None, 0, None, U.data_ptr(), F,
                      S.data_ptr(), Um.data_ptr(), F, M.data_ptr(), None)


def test_gat_bwd_stats_linear_matches_two_passes():
    """gala_cpu_gat_bwd_stats_linear_f32: the statistics backward with the attention Linear's
    dX term folded in equals gala_cpu_gat_bwd_stats_ex_f32 followed by
    gala_cpu_head_attn_bwd_f32 (d_aL identical, dX to one rounding); a missing wR is refused."""
    import torch
    from gala.backend import CpuBackend
    g = powerlaw(n=1500, m=9000)
    H, F = 4, 32
    rng = np.random.default_rng(12)
    t = lambda a: torch.from_numpy(a.astype(np.float32))  # noqa: E731
    X, aL, dY = t(rng.uniform(-1, 1, (g.n_rows, F))), t(rng.uniform(-1, 1, (g.n_rows, H))), \
        t(rng.uniform(-1, 1, (g.n_rows, F)))
    wR, bR = t(rng.uniform(-0.5, 0.5, F)), t(rng.uniform(-0.5, 0.5, H))
    be = CpuBackend()
    cg = be.graph(g)
    aR = be.head_attn(X, wR, bR, H)
    Y, q, Ym, sma = be.gat_stats_table(cg, aL, aR, X, H, 0.2, None, None)
    dX0, daL0 = be.gat_bwd_stats_table(cg, aL, aR, dY, None, q, Y, Ym, sma, H, 0.2)
    be.head_attn_bwd(daL0.view(-1, H), wR, H, dX0)
    dX1, daL1 = be.gat_bwd_stats_table(cg, aL, aR, dY, None, q, Y, Ym, sma, H, 0.2, wR=wR)
    np.testing.assert_array_equal(daL1.numpy(), daL0.numpy())
    np.testing.assert_allclose(dX1.numpy(), dX0.numpy(), rtol=1e-6, atol=1e-7)
    with pytest.raises(_abi.GalaError):
        _abi.call_cpu("gala_gat_bwd_stats_linear_f32", cg.csr(), aL.data_ptr(), aR.data_ptr(), None, dY.data_ptr(),
                      F, None, F, H, 0.2, q.data_ptr(), Y.data_ptr(), F, Ym.data_ptr(), F, sma.data_ptr(), None,
                      dX1.data_ptr(), F, daL1.data_ptr(), None)
