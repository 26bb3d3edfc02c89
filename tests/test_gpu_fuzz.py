"""GPU: seeded random parity sweep over the operator surface (tuning-independent corners).

Every case draws a graph (directed random rows with a chosen mean degree, optionally an
R-MAT graph, a block of empty rows, a hub row longer than the split threshold), a width F,
a head count, row padding, edge weights, a hub-row split plan with small chunks and column
tiling, then checks the HIP path against the oracle:

* bit-exact: degree, SpMM without hub chunks, the SpMM's GCN epilogue (deg norm from the
  rowptr, the next input beside the output), row-scale / row-broadcast;
* reordered sums (hub chunks, the GALA_SPMM_HUB_CHUNKED fast mode; the default REF order
  is bit-exact): within the worst-case fp32 summation bound of the row,
  |err| <= (deg + 1) 2^-24 sum|a x| + 1e-6 per entry;
* TOL (1e-4 abs + rel): SDDMM, edge softmax fwd / bwd, fused GAT forward / backward, the
  REF row-statistics backward's d_aL (its Y / q / dX bit-equal to the fused path's).
"""
import os

import numpy as np
import pytest
import torch

import oracle as orc
from gala import _abi, layout, ops
from _graphs import to_oracle

pytestmark = pytest.mark.gpu
TOL = dict(atol=1e-4, rtol=1e-4)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _graph(rng):
    kind = rng.choice(["random", "rmat", "empty_rows", "hub"])
    n = int(rng.integers(1, 2500))
    if kind == "rmat" and n >= 64:
        return layout.gen_graph("rmat", n, int(rng.integers(n, 12 * n)), seed=int(rng.integers(1 << 30)))
    deg = float(rng.uniform(0, 40))
    m = int(deg * n)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    if kind == "empty_rows":
        src = src % max(1, n // 3)
    if kind == "hub":
        hub = np.full(int(rng.integers(300, 3000)), int(rng.integers(0, n)))
        src = np.concatenate([src, hub])
        dst = np.concatenate([dst, rng.integers(0, n, hub.shape[0])])
    return layout.csr_build(n, n, src.astype(np.int32), dst.astype(np.int32))


def _padded(a, fill=np.nan):
    F = a.shape[1]
    buf = torch.full((a.shape[0], (F + 3) // 4 * 4), float(fill), device="cuda")
    buf[:, :F] = _dev(a)
    return buf[:, :F]


def _reordered_ok(Y, g, X, val=None):
    import scipy.sparse as sp
    v = np.ones(g.nnz) if val is None else val.astype(np.float64)
    A = sp.csr_matrix((v, g.col.copy(), g.rowptr.copy()), shape=(g.n_rows, g.n_cols))
    exact = A @ X.astype(np.float64)
    mass = abs(A) @ np.abs(X.astype(np.float64))
    # worst-case bound of any fp32 summation order over a row of n terms: n * 2^-24 * sum|a x|
    n = np.diff(g.rowptr).astype(np.float64)[:, None]
    assert np.all(np.abs(Y.astype(np.float64) - exact) <= (n + 1) * 2.0**-24 * mass + 1e-6)


@pytest.mark.parametrize("seed", range(int(os.environ.get("GALA_FUZZ_CASES", "96"))))
def test_random_case(seed):
    rng = np.random.default_rng(1000 + seed)
    g = _graph(rng)
    og = to_oracle(g)
    heads = int(rng.choice([1, 1, 2, 4, 8]))
    # multi-head widths: per-head lane counts are powers of two (the fused kernels' layout)
    F = heads * int(rng.choice([1, 2, 4, 8, 16, 32])) if heads > 1 else int(rng.integers(1, 300))
    pad = heads == 1 and F % 4 != 0 and bool(rng.integers(0, 2))
    vec = 4 if (F % 4 == 0 or pad) else (2 if F % 2 == 0 else 1)
    edge_ok = -(-F // vec) <= 64  # SDDMM / GAT row groups span at most one wave
    split = bool(rng.integers(0, 2)) and g.nnz > 0
    dg = ops.DeviceGraph.from_host(g, split=False)
    if split:
        dg.set_split_plan(g.rowptr, int(rng.integers(8, 200)), chunk=int(rng.choice([16, 32, 512])),
                          row_order=bool(rng.integers(0, 2)))
    chunked = dg.split_rows > 0
    X = rng.uniform(-1, 1, (g.n_cols, F)).astype(np.float32)
    Xd = _padded(X) if pad else _dev(X)

    # degree: exact counts
    np.testing.assert_array_equal(_host(ops.degree(dg)), orc.degree(og))
    # SpMM, plain and weighted (one weight per edge)
    val = rng.uniform(0, 1, g.nnz).astype(np.float32)
    for w in (None, val):
        gd = dg if w is None else dg.with_values(_dev(w))
        # REF order (default): bit-exact, hub rows included
        np.testing.assert_array_equal(_host(ops.spmm(gd, Xd)), orc.spmm(og if w is None else to_oracle(g, w), X))
        if chunked:   # the fast mode: hub rows as chunk partials
            _reordered_ok(_host(ops.spmm(gd, Xd, hub="chunked")), g, X, w)
    # the GCN epilogue (gala_spmm_ex_f32): the dst norm deg^-0.5 formed from the rowptr, the next
    # aggregation's input Y2 = fl(norm * Y) beside Y -- the degree pass + ROW_BROADCAST chain
    # of the oracle bit for bit (an empty row: inf norm, NaN row on both sides)
    norm = orc.degree(og, power=-0.5)
    want = orc.spmm(og, X, dst_scale=norm)
    Y1 = torch.empty((g.n_rows, F), device="cuda")
    Y2 = torch.empty((g.n_rows, F), device="cuda")
    ops.spmm(dg, Xd, out=Y1, dst_deg=True, out2=Y2)
    np.testing.assert_array_equal(_host(Y1), want)
    np.testing.assert_array_equal(_host(Y2), (norm[:, None] * want).astype(np.float32))
    # column-tiled layout (no split plan): segments summed in order, bit-exact
    if g.n_cols > 1 and not chunked:
        tg = layout.col_tile(g, int(rng.integers(1, g.n_cols)))
        np.testing.assert_array_equal(_host(ops.spmm(ops.DeviceGraph.from_host(tg, split=False), _dev(X))),
                                      orc.spmm(to_oracle(tg), X))
    if g.nnz == 0:
        return
    s = rng.uniform(-3, 3, g.nnz * heads).astype(np.float32)
    d = rng.uniform(-1, 1, g.nnz * heads).astype(np.float32)
    for mode in (_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED):
        a_ref = orc.softmax_fwd(og, s, heads=heads, mode=mode)
        np.testing.assert_allclose(_host(ops.edge_softmax(dg, _dev(s), heads=heads, mode=mode)), a_ref, **TOL)
        np.testing.assert_allclose(_host(ops.edge_softmax_bwd(dg, _dev(a_ref), _dev(d), heads=heads, mode=mode)),
                                   orc.softmax_bwd(og, a_ref, d, heads=heads, mode=mode), **TOL)
    if not edge_ok:
        return
    # SDDMM, edge softmax, fused GAT (REF and FIXED)
    A = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    Ad = _padded(A) if pad else _dev(A)
    np.testing.assert_allclose(_host(ops.sddmm(dg, Ad, Xd, heads=heads)), orc.sddmm(og, A, X, heads=heads), **TOL)
    aL = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    aR = rng.uniform(-1, 1, (g.n_cols, heads)).astype(np.float32)
    for mode in (_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED):
        Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=mode)
        Yg, al = ops.gat_fwd(dg, _dev(aL), _dev(aR), Xd, heads=heads, slope=0.2, mode=mode, want_alpha=True)
        np.testing.assert_allclose(_host(al), al_ref, **TOL)
        np.testing.assert_allclose(_host(Yg), Y_ref, **TOL)
        dz_ref, daL_ref = orc.gat_bwd(og, aL, aR, X, A, al_ref, heads=heads, slope=0.2, mode=mode)
        daL, dz = ops.gat_bwd(dg, _dev(aL), _dev(aR), Xd, Ad, _dev(al_ref), heads=heads, slope=0.2, mode=mode)
        np.testing.assert_allclose(_host(daL), daL_ref, **TOL)
        if mode == _abi.GALA_SOFTMAX_FIXED:
            np.testing.assert_allclose(_host(dz), dz_ref, **TOL)
    # REF row statistics (the graphs are square): Y / q bit-equal to the q-only forward, dX to
    # the fused backward, the same dX from the parked p, d_aL within TOL of the oracle chain
    Ys, q, Ym, sma, pe = ops.gat_fwd_stats(dg, _dev(aL), Xd, aR=_dev(aR), heads=heads, want_p=True)
    Y0, q0 = ops.gat_fwd_ex(dg, _dev(aL), Xd, aR=_dev(aR), heads=heads, factored="q")
    assert torch.equal(Ys, Y0) and torch.equal(q, q0)
    dX, daL = ops.gat_bwd_stats(dg, _dev(aL), _dev(aR), Ad, q, Ys, Ym, sma, heads=heads)
    dX0, _ = ops.gat_bwd_fused(dg, _dev(aL), Xd, Ad, q, aR=_dev(aR), heads=heads)
    assert torch.equal(dX, dX0)
    dXp, daLp = ops.gat_bwd_stats(dg, _dev(aL), None, Ad, q, Ys, Ym, sma, heads=heads, p=pe)
    assert torch.equal(dXp, dX) and torch.equal(daLp, daL)
    _, al_ref = orc.gat_fwd(og, aL, aR, X, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    _, daL_ref = orc.gat_bwd(og, aL, aR, X, A, al_ref, heads=heads, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
    np.testing.assert_allclose(_host(daL), daL_ref, **TOL)
    gw = orc.Graph(og.n_rows, og.n_cols, og.rowptr, og.col, al_ref, og.n_seg, og.bounds, heads)
    np.testing.assert_allclose(_host(dX), orc.spmm(gw, A), **TOL)
    # per-head attention logits and their input gradient
    wA = rng.uniform(-1, 1, F).astype(np.float32)
    bA = rng.uniform(-1, 1, heads).astype(np.float32)
    ref = (X.astype(np.float64).reshape(-1, heads, F // heads) * wA.reshape(1, heads, -1)).sum(2) + bA
    np.testing.assert_allclose(_host(ops.head_attn(Xd, _dev(wA), _dev(bA), heads=heads)), ref, rtol=1e-5, atol=1e-5)
    gA = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    np.testing.assert_array_equal(_host(ops.head_attn_bwd(_dev(gA), _dev(wA), heads=heads)),
                                  np.repeat(gA, F // heads, axis=1) * wA[None, :])


@pytest.mark.parametrize("seed", range(int(os.environ.get("GALA_FUZZ_CASES", "96")) // 2))
def test_random_case_more_ops(seed):
    """The rest of the surface on the same random graphs: kernel-sampled and multi-head
    weighted SpMM with norms (bit-exact), the attention-recompute GAT kernels, the ReLU
    prologue (bit-exact vs the torch chain), FFN forward / gradients (fp32 bounds)."""
    rng = np.random.default_rng(77000 + seed)
    g = _graph(rng)
    og = to_oracle(g)
    dg = ops.DeviceGraph.from_host(g, split=False)
    F = int(rng.integers(1, 130))
    X = rng.uniform(-1, 1, (g.n_cols, F)).astype(np.float32)
    # kernel sampling (a6): nsamp draws per non-empty row, (ra * j + rb) mod deg
    ns, ra, rb = int(rng.integers(1, 30)), int(rng.integers(1, 50)), int(rng.integers(0, 50))
    np.testing.assert_array_equal(_host(ops.spmm(dg, _dev(X), nsamp=ns, ra=ra, rb=rb)),
                                  orc.spmm(og, X, sample=True, nsamp=ns, ra=ra, rb=rb))
    # multi-head weights with src / dst norms
    H = int(rng.choice([1, 2, 4]))
    D = int(rng.choice([1, 4, 8, 16]))
    Xh = rng.uniform(-1, 1, (g.n_cols, H * D)).astype(np.float32)
    val = rng.uniform(0, 1, g.nnz * H).astype(np.float32)
    sn = rng.uniform(0.1, 1, g.n_cols).astype(np.float32)
    dn = rng.uniform(0.1, 1, g.n_rows).astype(np.float32)
    got = _host(ops.spmm(dg.with_values(_dev(val), val_heads=H), _dev(Xh), src_scale=_dev(sn), dst_scale=_dev(dn)))
    np.testing.assert_array_equal(got, orc.spmm(to_oracle(g, val, H), Xh, src_scale=sn, dst_scale=dn))
    # ReLU prologue: pre * relu(act * X) and its backward vs the torch chain, bit for bit
    Xd, Gd = _dev(X), _dev(rng.uniform(-1, 1, (g.n_cols, F)).astype(np.float32))
    act, pre = _dev(rng.uniform(0.1, 2, g.n_cols).astype(np.float32)), _dev(rng.uniform(0.1, 2, g.n_cols).astype(np.float32))
    t = act[:, None] * Xd
    assert torch.equal(ops.row_scale_relu(Xd, act, pre), pre[:, None] * torch.relu(t))
    assert torch.equal(ops.relu_scale_backward(Xd, Gd, act),
                       torch.where(torch.relu(t) <= 0, torch.zeros_like(Gd), Gd) * act[:, None])
    # attention recompute (one head): aR = X wR + bR inside the kernels
    if g.nnz and F <= 64:
        aL = rng.uniform(-1, 1, (g.n_rows, 1)).astype(np.float32)
        wR = (rng.uniform(-1, 1, F) * 0.5).astype(np.float32)
        bR = np.array([0.1], np.float32)
        aR = (X.astype(np.float64) @ wR.astype(np.float64) + 0.1).astype(np.float32)
        for mode in (_abi.GALA_SOFTMAX_REF, _abi.GALA_SOFTMAX_FIXED):
            Y_ref, al_ref = orc.gat_fwd(og, aL, aR, X, heads=1, slope=0.2, mode=mode)
            Y, al = ops.gat_fwd_attn(dg, _dev(aL), _dev(wR), _dev(bR), _dev(X), slope=0.2, mode=mode, want_alpha=True)
            np.testing.assert_allclose(_host(al), al_ref, **TOL)
            np.testing.assert_allclose(_host(Y), Y_ref, **TOL)
        dY = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
        _, al_ref = orc.gat_fwd(og, aL, aR, X, heads=1, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
        _, daL_ref = orc.gat_bwd(og, aL, aR, X, dY, al_ref, heads=1, slope=0.2, mode=_abi.GALA_SOFTMAX_REF)
        daL = ops.gat_bwd_attn(dg, _dev(aL), _dev(wR), _dev(bR), _dev(X), _dev(dY), _dev(al_ref), slope=0.2)
        np.testing.assert_allclose(_host(daL), daL_ref, **TOL)
    # FFN: forward (where supported) and weight / bias gradients
    N, K, M = g.n_cols, F, int(rng.integers(1, 70))
    W = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    b = rng.uniform(-1, 1, M).astype(np.float32)
    want = X.astype(np.float64) @ W.T.astype(np.float64) + b
    mass = np.abs(X.astype(np.float64)) @ np.abs(W.T.astype(np.float64)) + np.abs(b)
    try:
        Y = _host(ops.ffn_fwd(_dev(X), _dev(W), _dev(b)))
        assert np.all(np.abs(Y - want) <= (K + 1) * 2.0**-24 * mass + 1e-6)
    except _abi.GalaError as e:
        assert e.status == _abi.GALA_ERR_UNSUPPORTED
    dY = rng.uniform(-1, 1, (N, M)).astype(np.float32)
    dW, db = ops.dense_grad(_dev(X), _dev(dY))
    gw = dY.astype(np.float64).T @ X.astype(np.float64)
    gm = np.abs(dY.astype(np.float64)).T @ np.abs(X.astype(np.float64))
    assert np.all(np.abs(_host(dW) - gw) <= (N + 1) * 2.0**-24 * gm + 1e-6)
    np.testing.assert_allclose(_host(db), dY.astype(np.float64).sum(0), atol=(N + 1) * 2.0**-24 * N + 1e-6)


@pytest.mark.parametrize("seed", range(int(os.environ.get("GALA_FUZZ_CASES", "96")) // 4))
def test_random_case_halo_table(seed):
    """The table-indexed statistics pair (gala_gat_{fwd,bwd}_stats_ex_f32) on a random row
    partition of a random graph: each rank's rows over its gathered table equal the one-GPU
    pair's rows bit for bit (Y, q, Ym, sma, the recomputed own logits, dX, d_aL), with the
    whole graph's hub-row plan (small chunks) or none."""
    from gala import dist as gdist
    rng = np.random.default_rng(7000 + seed)
    g = _graph(rng)
    if g.n_rows < 2:
        return
    heads = int(rng.choice([1, 2, 4, 8]))
    D = int(rng.choice([4, 8, 16, 32]))
    F = heads * D
    world = int(rng.integers(1, 5))
    halo = str(rng.choice(["p2p", "dense"]))
    aL = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    X = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    dY = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    wR = _dev(rng.uniform(-0.5, 0.5, F).astype(np.float32))
    bR = _dev(rng.uniform(-0.5, 0.5, heads).astype(np.float32))
    thr = int(rng.choice([0, 64]))
    dg = ops.DeviceGraph.from_host(g, split=thr if thr else False)
    try:
        Y1, q1, Ym1, sma1, aR1 = ops.gat_fwd_stats(dg, _dev(aL), _dev(X), wR=wR, bR=bR, heads=heads, want_aR=True)
    except _abi.GalaError:      # head widths the statistics kernels refuse (D/VEC not a power of two)
        return
    dX1, daL1 = ops.gat_bwd_stats(dg, _dev(aL), aR1, _dev(dY), q1, Y1, Ym1, sma1, heads=heads)
    for p in range(world):
        pt = gdist.partition_graph(g, p, world, halo_mode=halo)
        own = slice(pt.r0, pt.r0 + pt.n)
        x2g = torch.from_numpy(np.maximum(pt.xs_to_global(), 0)).cuda()
        Xs, dYs = _dev(X)[x2g].contiguous(), _dev(dY)[x2g].contiguous()
        x0 = pt.own_offset()
        gp = ops.DeviceGraph.from_host(pt.graph, split=thr if thr else False)
        sc = torch.arange(x0, x0 + pt.n, dtype=torch.int32, device="cuda")
        As = torch.zeros((pt.n_cols, heads), device="cuda")
        Y, q, Ym, sma = ops.gat_fwd_stats(gp, _dev(aL[own]), Xs, wR=wR, bR=bR, heads=heads, self_col=sc, aR_out=As)
        assert torch.equal(Y, Y1[own]) and torch.equal(Ym, Ym1[own])
        assert torch.equal(q.view(-1, heads), q1.view(-1, heads)[own])
        assert torch.equal(sma.view(-1, heads), sma1.view(-1, heads)[own])
        assert torch.equal(As[x0:x0 + pt.n], aR1.view(-1, heads)[own])
        dX, daL = ops.gat_bwd_stats(gp, _dev(aL[own]), aR1.view(-1, heads)[x2g].contiguous(), dYs, q, Y, Ym, sma,
                                    heads=heads, dY_rows=dYs[x0:x0 + pt.n])
        assert torch.equal(dX, dX1[own]) and torch.equal(daL.view(-1, heads), daL1.view(-1, heads)[own])
