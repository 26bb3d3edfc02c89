"""CPU: the multi-head GAT layer in input space (gala_gat_in_*), host backend.

The layer v1 = X W^T + b -> aL / aR = per-head attention Linears of v1 -> the REF GAT
aggregation, and its REF backward down to the parameters, against the oracle's composition
of the reference's passes (oracle.gat_input_layer_ref: orc_gat_ref_layer on the fp32 Linear
output, gradients assembled the way autograd composes Ffn / HeadAttn / GatAggregateFfn).
libgala_cpu.so's twins run the GPU kernels' formulation -- the per-head aggregates of the
INPUT rows projected per row, the weight gradient regrouped over the transposed pattern --
so this checks the algebra on the host; tests/test_gpu_gat_input.py checks the gfx950
kernels the same way (and against these twins).
"""
import ctypes

import numpy as np
import pytest
import torch

import oracle as orc
from gala import _abi, layout
from _graphs import with_empty_rows
from test_cpu_backend import P, HostCsr

TOL = dict(atol=1e-4, rtol=1e-4)


def layer_inputs(n, fin, heads, D, seed):
    rng = np.random.default_rng(seed)
    F = heads * D
    X = rng.uniform(-1, 1, (n, fin)).astype(np.float32)
    W = (rng.uniform(-1, 1, (F, fin)) / np.sqrt(fin)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, F).astype(np.float32)
    wL, wR = (rng.uniform(-0.3, 0.3, F).astype(np.float32) for _ in range(2))
    bL, bR = (rng.uniform(-0.1, 0.1, heads).astype(np.float32) for _ in range(2))
    dY = rng.uniform(-1, 1, (n, F)).astype(np.float32)
    return X, W, b, wL, bL, wR, bR, dY


def compose(W, b, wL, bL, wR, bR, heads):
    from gala import ops
    t = [torch.from_numpy(a) for a in (W, b, wL, bL, wR, bR)]
    u, c = ops.gat_in_compose(*t, heads)
    return u.numpy(), c.numpy()


def cpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads, slope=0.2, order=None, order_t=None, relu=False):
    """The host twins composed as the mirror's GatInputLayer composes the GPU ops (the
    backward over the transposed pattern: g itself when it is symmetric)."""
    n, fin = X.shape
    F = W.shape[0]
    D = F // heads
    u, c = compose(W, b, wL, bL, wR, bR, heads)
    xext = np.zeros((n, 128), np.float32)
    _abi.call_cpu("gala_gat_in_prep_f32", n, fin, P(X), fin, heads, P(u), P(c), P(xext), None)
    A = HostCsr(g)
    Y, Ym = np.empty((n, F), np.float32), np.empty((n, F), np.float32)
    q, sma = np.empty((n, heads), np.float32), np.empty((n, heads), np.float32)
    _abi.call_cpu("gala_gat_in_fwd_f32", A.ref, P(order), fin, heads, D, slope, P(xext), P(W), fin, P(b), P(Y), P(Ym), F,
                  P(q), P(sma), _abi.GALA_GAT_IN_RELU if relu else 0, None)
    daL = np.empty((n, heads), np.float32)
    M = np.empty((heads, D, fin + 1), np.float32)
    wsb = _abi.cpu_lib().gala_cpu_gat_in_bwd_workspace(heads)
    ws = np.empty(wsb // 4, np.float32)
    gT, _ = layout.transpose(g)
    AT = HostCsr(gT)
    _abi.call_cpu("gala_gat_in_bwd_f32", AT.ref, P(order_t), fin, heads, D, slope, P(xext), P(dY), P(Y), P(Ym), F, P(sma),
                  P(daL), P(M), P(ws), wsb, _abi.GALA_GAT_IN_RELU if relu else 0, None)
    Gw, Gb = np.empty((heads, fin), np.float32), np.empty(heads, np.float32)
    gwb = _abi.cpu_lib().gala_cpu_dense_grad_workspace(n, fin, heads)
    gws = np.empty(max(gwb // 4, 1), np.float32)
    _abi.call_cpu("gala_dense_grad_f32", n, fin, heads, P(X), fin, P(daL), heads, P(Gw), P(Gb), 0, P(gws), gwb, None)
    sLR = (wL + wR).reshape(heads, D).astype(np.float64)
    dW = (M[:, :, :fin] + sLR[:, :, None] * Gw[:, None, :]).reshape(F, fin)
    db = (M[:, :, fin] + sLR * Gb[:, None]).reshape(F)
    dw = (W.reshape(heads, D, fin) * Gw[:, None, :]).sum(2) + b.reshape(heads, D) * Gb[:, None]
    return dict(Y=Y, q=q, daL=daL, dW=dW, db=db, dwL=dw.reshape(-1), dbL=Gb, xext=xext)


def own_logits(xext, heads):
    """aL, aR [n, heads] from the extended rows (slots 99 + 4h, 67 + 4h)."""
    return (xext[:, [99 + 4 * h for h in range(heads)]], xext[:, [67 + 4 * h for h in range(heads)]])


def ref_on_own_logits(g, got, X, W, b, wL, bL, wR, bR, dY, heads, relu=False):
    """The oracle's layer on the kernels' own attention logits, after checking those against
    the float64 attention Linears of the float64 Linear output (1e-5): a logit at the
    LeakyReLU kink takes the other slope under a one-ulp change."""
    F = W.shape[0]
    D = F // heads
    aL, aR = own_logits(got["xext"], heads)
    v1 = X.astype(np.float64) @ W.astype(np.float64).T + b.astype(np.float64)
    v1 = v1.reshape(-1, heads, D)
    np.testing.assert_allclose(aL, (v1 * wL.reshape(heads, D)).sum(-1) + bL, atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(aR, (v1 * wR.reshape(heads, D)).sum(-1) + bR, atol=1e-5, rtol=1e-5)
    if relu:   # torch's threshold_backward on the layer's output (the kernels' own relu(Y) > 0)
        dY = np.where(got["Y"] > 0, dY, np.float32(0)).astype(np.float32)
    ref = orc.gat_input_layer_ref(g.rowptr, g.col, X, W, b, wL, bL, wR, bR, dY, heads, aL=aL, aR=aR)
    if relu:
        ref["Y"] = np.maximum(ref["Y"], 0)
    return ref


def grad_close(got, want, name):
    want = np.asarray(want, np.float64)
    tol = 1e-4 * np.abs(want).max() + 1e-6
    err = np.abs(np.asarray(got, np.float64) - want).max()
    assert err <= tol, (name, err, tol)


@pytest.mark.parametrize("fin,heads,D", [(100, 8, 32), (37, 4, 16), (20, 2, 32), (100, 1, 32)])
def test_input_space_layer_matches_the_reference_chain(fin, heads, D):
    g = layout.gen_graph("uniform", 1500, 9000, seed=7)
    X, W, b, wL, bL, wR, bR, dY = layer_inputs(g.n_rows, fin, heads, D, seed=fin + heads)
    got = cpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads)
    ref = ref_on_own_logits(g, got, X, W, b, wL, bL, wR, bR, dY, heads)
    np.testing.assert_allclose(got["Y"], ref["Y"], **TOL)
    np.testing.assert_allclose(got["q"], ref["q"], rtol=1e-4)
    # with the program's ReLU fused (forward store, backward mask)
    gr = cpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads, relu=True)
    rr = ref_on_own_logits(g, gr, X, W, b, wL, bL, wR, bR, dY, heads, relu=True)
    np.testing.assert_allclose(gr["Y"], rr["Y"], **TOL)
    np.testing.assert_allclose(gr["daL"], rr["daL"], **TOL)
    for k in ("dW", "db", "dwL", "dbL"):
        grad_close(gr[k], rr[k], k + "_relu")
    np.testing.assert_allclose(got["daL"], ref["daL"], **TOL)
    for k in ("dW", "db", "dwL", "dbL"):
        grad_close(got[k], ref[k], k)
    # the extended rows: the features, the ones column, aR (against the oracle's aR of v1)
    xe = got["xext"]
    np.testing.assert_array_equal(xe[:, :min(fin, 64)], X[:, :min(fin, 64)])
    assert (xe[:, 112] == 1.0).all()


def test_input_space_layer_power_law_and_empty_rows():
    """A non-symmetric graph with empty rows (q = 1e12, Y = 0): the backward walks the
    transposed pattern."""
    g = with_empty_rows()
    fin, heads, D = 48, 8, 16
    X, W, b, wL, bL, wR, bR, dY = layer_inputs(g.n_rows, fin, heads, D, seed=3)
    got = cpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads)
    ref = ref_on_own_logits(g, got, X, W, b, wL, bL, wR, bR, dY, heads)
    np.testing.assert_allclose(got["Y"], ref["Y"], **TOL)
    np.testing.assert_allclose(got["daL"], ref["daL"], **TOL)
    for k in ("dW", "db", "dwL", "dbL"):
        grad_close(got[k], ref[k], k)


def test_input_space_refusals():
    g = layout.gen_graph("uniform", 100, 300, seed=1)
    A = HostCsr(g)
    X = np.zeros((100, 128), np.float32)
    xext = np.zeros((100, 128), np.float32)
    W = np.zeros((256, 128), np.float32)
    Y = np.zeros((100, 256), np.float32)
    q = np.zeros((100, 8), np.float32)
    L = _abi.cpu_lib()
    # fin > 100, D not in {4, 8, 16, 32}, more than 8 heads: unsupported (callers keep the chain)
    assert L.gala_cpu_gat_in_fwd_f32(A.ref, None, 101, 8, 32, 0.2, P(xext), P(W), 128, None, P(Y), P(Y), 256, P(q), P(q),
                                     0, None) == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_cpu_gat_in_fwd_f32(A.ref, None, 100, 8, 24, 0.2, P(xext), P(W), 128, None, P(Y), P(Y), 256, P(q), P(q),
                                     0, None) == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_cpu_gat_in_prep_f32(100, 101, P(X), 128, 8, P(W), P(W), P(xext), None) == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_cpu_gat_in_prep_f32(100, 100, P(X), 99, 8, P(W), P(W), P(xext), None) == _abi.GALA_ERR_INVALID_ARG
    t = HostCsr(layout.col_tile(g, 40))
    assert L.gala_cpu_gat_in_fwd_f32(t.ref, None, 100, 8, 32, 0.2, P(xext), P(W), 128, None, P(Y), P(Y), 256, P(q), P(q),
                                     0, None) == _abi.GALA_ERR_UNSUPPORTED
    assert L.gala_cpu_gat_in_bwd_workspace(9) < 0


def test_mirror_op_on_host_tensors_equals_the_three_op_chain():
    """The mirror's gat_input_layer_apply with the graph on the host (libgala_cpu.so's twins)
    against ffn_apply -> head_attn_apply -> gat_aggregate_ffn_apply with autograd; a
    non-symmetric pattern (the backward builds and walks its transpose)."""
    import gala
    E = gala.torch_ext()
    for g in (layout.gen_graph("uniform", 1200, 8000, seed=4), with_empty_rows()):
        E.slots_clear()
        off, cols = torch.from_numpy(g.rowptr), torch.from_numpy(g.col)
        vals = torch.ones(g.nnz)
        E.slots_push(off, cols, vals, None, 1, False)
        E.slots_push(off, cols, vals, None, 1, False)
        fin, H, D = 48, 4, 16
        X, W, b, wL, bL, wR, bR, dY = layer_inputs(g.n_rows, fin, H, D, seed=11)
        params = [torch.from_numpy(a).requires_grad_() for a in (W, b, wL.reshape(1, -1), bL, wR.reshape(1, -1), bR)]
        x = torch.from_numpy(X)
        assert E.gat_input_layer_eligible(x, params[0], 0, H, 0)
        for relu in (False, True):
            for p in params:
                p.grad = None
            Y = E.gat_input_layer_apply(x, *params, 0, 0.2, 0, relu)
            Y.backward(torch.from_numpy(dY))
            got = [Y.detach().numpy()] + [p.grad.numpy().copy() for p in params]
            for p in params:
                p.grad = None
            v1 = E.ffn_apply(x, params[0], params[1])
            aL = E.head_attn_apply(v1, params[2], params[3])
            Y0 = E.gat_aggregate_ffn_apply(aL, v1, params[4], params[5], 0, 0.2, 0)
            if relu:
                Y0 = torch.relu(Y0)
            Y0.backward(torch.from_numpy(dY))
            want = [Y0.detach().numpy()] + [p.grad.numpy() for p in params]
            np.testing.assert_allclose(got[0], want[0], **TOL)
            for name, a, w in zip(("W", "b", "wL", "bL", "wR", "bR"), got[1:], want[1:]):
                grad_close(a, w, f"{name} relu={relu}")
    E.slots_clear()
