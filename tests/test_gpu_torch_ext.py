"""GPU: the C++/libtorch mirror of the emitted operator API (host/gala_torch.cpp).

The generated GCN forward of codegen/gala.cu:423-459 and the GAT chain of
src/codegen/common.h:622-894 are rebuilt from the mirrored functions and checked against
an independent float64 torch formulation (tolerance 1e-4, the north_star bar).
"""
import numpy as np
import pytest
import torch

import oracle as orc
from gala import layout
from _graphs import cora_like, features, powerlaw, to_oracle

pytestmark = pytest.mark.gpu
TOL = dict(atol=1e-4, rtol=1e-4)


@pytest.fixture(scope="module")
def E():
    import gala
    return gala.torch_ext()


def dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return t if dtype is None else t.to(dtype)


def push_graph(E, g: layout.HostGraph, weighted=False, with_transpose=False):
    """Slots 0 (forward) and 1 (backward) like the generated dataPrep (cuda.h:1196-1257)."""
    E.slots_clear()
    off, cols = dev(g.rowptr), dev(g.col)
    vals = torch.ones(g.nnz, device="cuda")
    bounds = None if g.n_seg == 1 else torch.from_numpy(g.bounds)
    E.slots_push(off, cols, vals, bounds, g.n_seg, weighted)
    if with_transpose:
        t, perm = layout.transpose(g)
        E.slots_push(dev(t.rowptr), dev(t.col), torch.ones(t.nnz, device="cuda"), None, 1, weighted)
        E.slots_set_transpose_perm(1, dev(perm))
    else:
        E.slots_push(off, cols, vals, bounds, g.n_seg, weighted)
    return off, cols, vals, bounds


def coo(g):
    rows = np.repeat(np.arange(g.n_rows), np.diff(g.rowptr))
    return torch.from_numpy(rows).long(), torch.from_numpy(g.col.astype(np.int64))


def test_emitted_functions_tiled(E):
    g = layout.col_tile(cora_like(), 1000)
    off, cols, vals, bounds = push_graph(E, g)
    X = features(g.n_cols, 47)
    Y = E.aggregate_node_mul_sum_call(dev(X), off, cols, vals, bounds, g.n_seg)
    np.testing.assert_array_equal(Y.cpu().numpy(), orc.spmm(to_oracle(g), X))
    v = features(g.nnz, 1, seed=3).ravel()
    r = E.node_spmv_backward_of_sddmm_nln(off, cols, dev(v), bounds, g.n_rows, g.n_seg)
    np.testing.assert_allclose(r.cpu().numpy().ravel(), orc.row_sum(to_oracle(g), v), **TOL)
    q = features(g.n_rows, 1, seed=4)
    vv = dev(v)
    out = E.inplace_softmax_sddvv(dev(q), off, cols, vv, bounds, g.n_rows, g.n_seg)
    assert out.data_ptr() == vv.data_ptr()  # in place, returns value_graph
    np.testing.assert_array_equal(vv.cpu().numpy(), orc.row_scale(to_oracle(g), q.ravel(), v))
    a, b = features(g.n_rows, 1, seed=5), features(g.n_cols, 1, seed=6)
    s = E.edge_sddvv(dev(a), dev(b), off, cols, vals, bounds, g.n_rows, g.n_seg)
    np.testing.assert_array_equal(s.cpu().numpy(), orc.sddvv(to_oracle(g), a, b, op=0))
    m = E.aggregate_edge_mul(dev(a), dev(b), off, cols, vals, bounds, g.n_seg)
    np.testing.assert_array_equal(m.cpu().numpy(), orc.sddvv(to_oracle(g), a, b, op=1))
    A2, B2 = features(g.n_rows, 32, seed=7), features(g.n_cols, 32, seed=8)
    d = E.edge_sddmm(dev(A2), dev(B2), off, cols, vals, bounds, g.n_rows, g.n_seg)
    np.testing.assert_allclose(d.cpu().numpy(), orc.sddmm(to_oracle(g), A2, B2), **TOL)


@pytest.mark.parametrize("tile", [300, 1000])
def test_tiled_spmm_on_merged_rows_equals_segment_walk(E, tile):
    """A registered tiled graph's unweighted SpMM runs on the slot's merged rows (segments
    concatenated per row, with the merged graph's hub-row plan); an unregistered copy of the
    same tensors takes the kernel's segment walk.  Both equal the oracle bit for bit."""
    g = layout.col_tile(powerlaw(), tile)
    assert g.n_seg > 1
    off, cols, vals, bounds = push_graph(E, g)
    X = dev(features(g.n_cols, 32))
    want = orc.spmm(to_oracle(g), X.cpu().numpy())
    merged = E.aggregate_node_mul_sum_call(X, off, cols, vals, bounds, g.n_seg)
    walked = E.aggregate_node_mul_sum_call(X, off.clone(), cols.clone(), vals, bounds, g.n_seg)
    np.testing.assert_array_equal(merged.cpu().numpy(), want)
    np.testing.assert_array_equal(walked.cpu().numpy(), want)
    ones = torch.ones(g.n_rows, 1, device="cuda")
    deg = E.aggregate_node_mul_sum_direct_call(ones, off, cols, vals, bounds, g.n_seg)
    np.testing.assert_array_equal(deg.cpu().numpy().ravel(), np.diff(powerlaw().rowptr).astype(np.float32))


def test_gcn2_generated_forward_backward(E):
    """codegen/gala.cu:423-459 step through the mirror vs float64 torch.sparse."""
    g = powerlaw()
    off, cols, vals, _ = push_graph(E, g)
    N, Fin, H, C = g.n_rows, 100, 32, 47
    torch.manual_seed(0)
    fc0 = torch.nn.Linear(Fin, H).cuda()
    fc1 = torch.nn.Linear(H, C).cuda()
    X = dev(features(N, Fin))

    ones = torch.ones(N, 1, device="cuda")
    degrees = E.aggregate_node_mul_sum_direct_call(ones, off, cols, vals)
    norm = torch.pow(degrees, -0.5)
    res = fc0(X)
    res = norm * res
    res = E.aggregate_node_mul_sum_apply(res, 0)
    res = norm * res
    res = torch.relu(res)
    res = norm * res
    res = E.aggregate_node_mul_sum_apply(res, 0)
    res = norm * res
    out = fc1(res)
    out.square().sum().backward()

    # float64 reference with the same parameters
    r, c = coo(g)
    A = torch.sparse_coo_tensor(torch.stack([r, c]), torch.ones(len(r), dtype=torch.float64), (N, N))
    W0 = fc0.weight.detach().cpu().double().requires_grad_()
    b0 = fc0.bias.detach().cpu().double().requires_grad_()
    W1 = fc1.weight.detach().cpu().double().requires_grad_()
    b1 = fc1.bias.detach().cpu().double().requires_grad_()
    deg = torch.sparse.sum(A, 1).to_dense()[:, None]
    n64 = deg.pow(-0.5)
    h = X.cpu().double() @ W0.T + b0
    h = n64 * torch.sparse.mm(A, n64 * h)
    h = n64 * torch.sparse.mm(A, n64 * torch.relu(h))
    o = h @ W1.T + b1
    o.square().sum().backward()
    np.testing.assert_array_equal(degrees.cpu().numpy().ravel(), deg.numpy().ravel())
    np.testing.assert_allclose(out.detach().cpu().numpy(), o.detach().numpy(), **TOL)
    np.testing.assert_allclose(fc0.weight.grad.cpu().numpy(), W0.grad.numpy(), atol=1e-3, rtol=1e-4)
    np.testing.assert_allclose(fc1.weight.grad.cpu().numpy(), W1.grad.numpy(), atol=1e-3, rtol=1e-4)


def test_gcn_aggregate_fused_equals_reference_chain(E):
    g = cora_like()
    off, cols, vals, _ = push_graph(E, g)
    X = dev(features(g.n_rows, 32))
    norm = E.degree_norm(off)
    ref = norm * E.aggregate_node_mul_sum_call(norm * X, off, cols, vals)
    got = E.gcn_aggregate(X, norm.view(-1), off, cols)
    np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("graph", ["cora", "powerlaw_dense"])
def test_gcn_aggregate_relu_equals_unfused_chain(E, graph):
    """post * A (pre * relu(act * X)) with its backward, against the same chain of torch ops
    around the plain aggregation, bit for bit: on Cora (4.9 edges per row: the backward's
    post * dY rides in the SpMM as its source scale) and on a graph of 40 edges per row (the
    row-broadcast pass)."""
    g = cora_like() if graph == "cora" else layout.gen_graph("uniform", 3000, 60000, 3)
    push_graph(E, g)
    N = g.n_rows
    torch.manual_seed(1)
    norm = torch.rand(N, 1, device="cuda") + 0.5
    act = torch.rand(N, 1, device="cuda") + 0.5
    # (on Cora the ReLU rides in the SpMM as its prologue, and on both graphs the ReLU
    # backward as its epilogue: gala_spmm_ex_f32's src_relu / relu_x; absent factors and a
    # width that is not a multiple of 4 take the same kernels' other variants)
    for F, a, pre, post in ((32, act, norm, norm), (32, None, norm, None), (47, act, None, norm),
                            (5, None, None, None)):
        X0 = torch.randn(N, F, device="cuda")
        X0[::9, 0] = 0.0
        dY = torch.randn(N, F, device="cuda")
        X1 = X0.clone().requires_grad_()
        Y1 = E.gcn_aggregate_relu_apply(X1, a, pre, post, 0)
        Y1.backward(dY)
        X2 = X0.clone().requires_grad_()
        h = torch.relu(X2 if a is None else a * X2)
        Y2 = E.aggregate_node_mul_sum_apply(h if pre is None else pre * h, 0)
        if post is not None:
            Y2 = post * Y2
        Y2.backward(dY)
        np.testing.assert_array_equal(Y1.detach().cpu().numpy(), Y2.detach().cpu().numpy())
        np.testing.assert_array_equal(X1.grad.cpu().numpy(), X2.grad.cpu().numpy())


@pytest.mark.parametrize("graph", ["cora", "powerlaw_dense"])
def test_gcn_aggregate_apply_equals_unfused_chain(E, graph):
    """post * A (pre * X) with its backward (the first GCN layer's fused op), against torch
    ops around the plain aggregation, bit for bit: on Cora (4.9 edges per row: pre * X and
    the backward's post * dY ride in the SpMM as its source scale) and at 40 edges per row
    (the row-broadcast passes); pre alone and pre + post."""
    g = cora_like() if graph == "cora" else layout.gen_graph("uniform", 3000, 60000, 3)
    push_graph(E, g)
    N = g.n_rows
    torch.manual_seed(2)
    norm = torch.rand(N, 1, device="cuda") + 0.5
    post = torch.rand(N, 1, device="cuda") + 0.5
    X0 = torch.randn(N, 32, device="cuda")
    dY = torch.randn(N, 32, device="cuda")
    for p in (None, post):
        X1 = X0.clone().requires_grad_()
        Y1 = E.gcn_aggregate_apply(X1, norm, p, 0)
        Y1.backward(dY)
        X2 = X0.clone().requires_grad_()
        Y2 = E.aggregate_node_mul_sum_apply(norm * X2, 0)
        if p is not None:
            Y2 = p * Y2
        Y2.backward(dY)
        np.testing.assert_array_equal(Y1.detach().cpu().numpy(), Y2.detach().cpu().numpy())
        np.testing.assert_array_equal(X1.grad.cpu().numpy(), X2.grad.cpu().numpy())


def _gat_unfused_ref(E, aL, aR, X, li=0):
    """The reference's emitted GAT chain (common.h:622-894) through the mirror."""
    s = E.aggregate_edge_sum_apply(aL, aR, li)
    s = torch.nn.functional.leaky_relu(s, 0.2)
    attn = E.non_lnr_op_softmax_apply(s, li)
    return E.aggregate_node_mul_sum_attn_apply(X, attn, li)


@pytest.mark.parametrize("F", [32, 47])
def test_gat_fused_ref_mode_matches_unfused_chain(E, F):
    g = cora_like()
    push_graph(E, g)
    N = g.n_rows
    aL0, aR0, X0 = features(N, 1, seed=1), features(N, 1, seed=2), features(N, F, seed=3)
    outs, grads = [], []
    for fused in (False, True):
        aL = dev(aL0).requires_grad_()
        aR = dev(aR0).requires_grad_()
        X = dev(X0).requires_grad_()
        Y = E.gat_aggregate_apply(aL, aR, X, 0, 0.2, 0) if fused else _gat_unfused_ref(E, aL, aR, X)
        (Y * torch.linspace(-1, 1, F, device="cuda")).sum().backward()
        outs.append(Y.detach().cpu().numpy())
        grads.append([t.grad.cpu().numpy() for t in (aL, aR, X)])
    np.testing.assert_allclose(outs[1], outs[0], **TOL)
    for a, b in zip(grads[1], grads[0]):
        np.testing.assert_allclose(a, b, atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("heads,D", [(1, 32), (4, 16)])
def test_gat_fused_fixed_mode_true_gradients(E, heads, D):
    """FIXED mode: numerically stable softmax and the exact (transposed) gradients,
    checked against float64 torch autograd."""
    g = powerlaw(n=1500, m=9000)
    push_graph(E, g, with_transpose=True)
    N, F = g.n_rows, heads * D
    aL0, aR0, X0 = features(N, heads, seed=1), features(N, heads, seed=2), features(N, F, seed=3)
    aL = dev(aL0).requires_grad_()
    aR = dev(aR0).requires_grad_()
    X = dev(X0).requires_grad_()
    Y = E.gat_aggregate_apply(aL, aR, X, 0, 0.2, 1)
    w = torch.linspace(-1, 1, F, device="cuda")
    (Y * w).sum().backward()

    r, c = coo(g)
    l64 = torch.from_numpy(aL0).double().requires_grad_()
    r64 = torch.from_numpy(aR0).double().requires_grad_()
    x64 = torch.from_numpy(X0).double().requires_grad_()
    z = torch.nn.functional.leaky_relu(l64[r] + r64[c], 0.2)            # [E, H]
    m = torch.full((N, heads), -torch.inf, dtype=torch.float64).scatter_reduce(
        0, r[:, None].expand(-1, heads), z, "amax")
    p = torch.exp(z - m[r])
    den = torch.zeros(N, heads, dtype=torch.float64).index_add(0, r, p)
    alpha = p / den[r]
    msg = alpha[:, :, None] * x64[c].view(-1, heads, D)
    Y64 = torch.zeros(N, heads, D, dtype=torch.float64).index_add(0, r, msg).view(N, F)
    (Y64 * w.cpu().double()).sum().backward()
    np.testing.assert_allclose(Y.detach().cpu().numpy(), Y64.detach().numpy(), **TOL)
    np.testing.assert_allclose(X.grad.cpu().numpy(), x64.grad.numpy(), **TOL)
    np.testing.assert_allclose(aL.grad.cpu().numpy(), l64.grad.numpy(), atol=1e-4, rtol=1e-3)
    np.testing.assert_allclose(aR.grad.cpu().numpy(), r64.grad.numpy(), atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("F", [32, 47])
def test_gat_ffn_recompute_matches_explicit_attention(E, mode, F):
    """gat_aggregate_ffn_apply (aR = Linear(X) recomputed in the kernels) against
    gat_aggregate_apply on aR = torch Linear(X): output and the gradients of aL, X and the
    attention Linear (through aR), within fp32 tolerance."""
    g = powerlaw(n=1500, m=9000)
    push_graph(E, g, with_transpose=(mode == 1))
    N = g.n_rows
    aL0, X0 = features(N, 1, seed=1), features(N, F, seed=3)
    lin0 = torch.nn.Linear(F, 1).cuda()
    outs, grads = [], []
    for ffn in (False, True):
        aL = dev(aL0).requires_grad_()
        X = dev(X0).requires_grad_()
        lin = torch.nn.Linear(F, 1).cuda()
        lin.load_state_dict(lin0.state_dict())
        if ffn:
            Y = E.gat_aggregate_ffn_apply(aL, X, lin.weight, lin.bias, 0, 0.2, mode)
        else:
            Y = E.gat_aggregate_apply(aL, lin(X), X, 0, 0.2, mode)
        (Y * torch.linspace(-1, 1, F, device="cuda")).sum().backward()
        outs.append(Y.detach().cpu().numpy())
        grads.append([t.grad.cpu().numpy() for t in (aL, X, lin.weight, lin.bias)])
    np.testing.assert_allclose(outs[1], outs[0], **TOL)
    for a, b in zip(grads[1], grads[0]):
        np.testing.assert_allclose(a, b, atol=1e-4, rtol=1e-3)


def test_errors_are_exceptions_not_exit(E):
    g = cora_like()
    off, cols, vals, _ = push_graph(E, g)
    # a host tensor against a device graph: an error, never a silent copy or CPU fallback
    with pytest.raises(RuntimeError, match="is on cpu but the graph is on cuda"):
        E.aggregate_node_mul_sum_call(torch.ones(g.n_rows, 4), off, cols, vals)
    with pytest.raises(RuntimeError, match="slot"):
        E.aggregate_node_mul_sum_apply(torch.ones(g.n_rows, 4, device="cuda"), 7)


def test_ffn_apply_matches_linear(E):
    """ffn_apply: at::linear's forward bit for bit; gradients vs float64 autograd."""
    torch.manual_seed(0)
    lin = torch.nn.Linear(100, 32).cuda()
    X = torch.rand(50000, 100, device="cuda") - 0.5
    X.requires_grad_(True)
    Y = E.ffn_apply(X, lin.weight, lin.bias)
    assert torch.equal(Y, lin(X))
    g = torch.rand_like(Y) - 0.5
    Y.backward(g)
    X64, W64 = X.detach().double().cpu(), lin.weight.detach().double().cpu()
    g64 = g.double().cpu()
    np.testing.assert_allclose(lin.weight.grad.cpu().numpy(), (g64.T @ X64).numpy(), atol=1e-3, rtol=1e-4)
    np.testing.assert_allclose(lin.bias.grad.cpu().numpy(), g64.sum(0).numpy(), atol=1e-3, rtol=1e-4)
    np.testing.assert_allclose(X.grad.cpu().numpy(), (g64 @ W64).numpy(), atol=1e-4, rtol=1e-4)
    # no bias
    Z = E.ffn_apply(X.detach(), lin.weight, None)
    assert torch.equal(Z, torch.nn.functional.linear(X.detach(), lin.weight))
