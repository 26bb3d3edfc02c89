"""GPU: the multi-head GAT layer in input space (gala_gat_in_*, csrc/gat_input.hip).

Config 3's layer 1 (Products: fin = 100 -> 8 heads of 32) as the reference's generated program
computes it -- FFN_OP, the per-head attention Linears, the REF edge chain and aggregation,
and the REF backward down to the parameters -- against the oracle's pass-by-pass composition
(oracle.gat_input_layer_ref over orc_gat_ref_layer): forward Y, d_aL and every parameter
gradient within 1e-4 (gradients: 1e-4 of the tensor's largest entry, the refgen tests'
tolerance), on small graphs (symmetric, and non-symmetric with the transposed pattern) and
on the Products shape at full size (N = 2 449 029, E = 126 167 309).  The mirror's
gat_input_layer_apply against the three ops it replaces (ffn_apply -> head_attn_apply ->
gat_aggregate_ffn_apply) with autograd.
"""
import os

import numpy as np
import pytest
import torch

import oracle as orc
from gala import layout, ops
from _graphs import with_empty_rows
from test_gat_input_cpu import cpu_layer, grad_close, layer_inputs, ref_on_own_logits

pytestmark = pytest.mark.gpu
TOL = dict(atol=1e-4, rtol=1e-4)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def gpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads, gT=None, relu=False, order=None, tmode=False):
    dg = ops.DeviceGraph.from_host(g, split=False)
    dgT = None if gT is None else ops.DeviceGraph.from_host(gT, split=False)
    od = None if order is None else dev(order)
    out = ops.gat_input_layer(dg, dev(X), dev(W), dev(b), dev(wL), dev(bL), dev(wR), dev(bR), heads,
                              dY=dev(dY), gT=dgT, relu=relu, order=od, order_t=od, tmode=tmode)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items() if v is not None and k != "T"}


def check_against_ref(got, ref):
    np.testing.assert_allclose(got["Y"], ref["Y"], **TOL)
    np.testing.assert_allclose(got["q"], ref["q"], rtol=1e-4)
    np.testing.assert_allclose(got["daL"], ref["daL"], **TOL)
    for k in ("dW", "db", "dwL", "dbL", "dwR", "dbR"):
        grad_close(got[k], ref[k], k)


@pytest.mark.parametrize("fin,heads,D", [(100, 8, 32), (37, 4, 16), (20, 2, 32), (100, 1, 32), (64, 8, 8),
                                         (48, 8, 4), (100, 3, 4)])
def test_input_space_kernels_against_the_reference_chain(fin, heads, D):
    g = layout.gen_graph("uniform", 3000, 40000, seed=7)
    X, W, b, wL, bL, wR, bR, dY = layer_inputs(g.n_rows, fin, heads, D, seed=fin + heads)
    got = gpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads)
    ref = ref_on_own_logits(g, got, X, W, b, wL, bL, wR, bR, dY, heads)
    check_against_ref(got, ref)
    # the fused ReLU, rows taken in descending-degree order
    gr = gpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads, relu=True, order=ops.degree_order(g.rowptr))
    rr = ref_on_own_logits(g, gr, X, W, b, wL, bL, wR, bR, dY, heads, relu=True)
    check_against_ref(gr, rr)
    # T mode (gala_gat_in_{fwd,bwd}_t_f32: the backward's aggregates formed by the forward)
    gt = gpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads, relu=True, order=ops.degree_order(g.rowptr), tmode=True)
    rt = ref_on_own_logits(g, gt, X, W, b, wL, bL, wR, bR, dY, heads, relu=True)
    check_against_ref(gt, rt)
    # the host twins run the same sums in the same order (exp aside)
    host = cpu_layer(g, X, W, b, wL, bL, wR, bR, dY, heads)
    np.testing.assert_allclose(got["Y"], host["Y"], atol=2e-6, rtol=2e-6)
    np.testing.assert_allclose(got["daL"], host["daL"], atol=2e-6, rtol=2e-6)
    np.testing.assert_allclose(got["dW"], host["dW"], atol=1e-5 * np.abs(host["dW"]).max())


def test_input_space_kernels_non_symmetric_and_empty_rows():
    g = with_empty_rows()
    gT, _ = layout.transpose(g)
    X, W, b, wL, bL, wR, bR, dY = layer_inputs(g.n_rows, 100, 8, 32, seed=5)
    got = gpu_layer(g, X, W, b, wL, bL, wR, bR, dY, 8, gT=gT)
    ref = ref_on_own_logits(g, got, X, W, b, wL, bL, wR, bR, dY, 8)
    check_against_ref(got, ref)
    deg = np.diff(g.rowptr)
    assert (deg == 0).any() and np.all(got["Y"][deg == 0] == 0) and np.all(got["q"][deg == 0] == np.float32(1e12))
    # T mode on the symmetrised graph (its empty rows and heavy row kept)
    src = np.repeat(np.arange(g.n_rows, dtype=np.int32), np.diff(g.rowptr))
    n2 = g.n_rows + 50   # 50 isolated rows: empty in T mode's q pass and walk
    gs = layout.csr_build(n2, n2, np.concatenate([src, g.col]), np.concatenate([g.col, src]))
    X2, W2, b2, wL2, bL2, wR2, bR2, dY2 = layer_inputs(gs.n_rows, 100, 8, 32, seed=6)
    gt = gpu_layer(gs, X2, W2, b2, wL2, bL2, wR2, bR2, dY2, 8, tmode=True)
    rt = ref_on_own_logits(gs, gt, X2, W2, b2, wL2, bL2, wR2, bR2, dY2, 8)
    check_against_ref(gt, rt)
    assert np.all(gt["Y"][g.n_rows:] == 0) and np.all(gt["q"][g.n_rows:] == np.float32(1e12))


def test_input_space_refused_shapes():
    from gala import _abi
    g = layout.gen_graph("uniform", 200, 800, seed=1)
    X, W, b, wL, bL, wR, bR, dY = layer_inputs(g.n_rows, 100, 8, 32, seed=1)
    Wbad = dev(np.zeros((8 * 24, 100), np.float32))
    dg = ops.DeviceGraph.from_host(g, split=False)
    xext = torch.zeros(g.n_rows, 128, device="cuda")
    with pytest.raises(_abi.GalaError):   # D = 24 (the projection takes 4, 8, 16, 32)
        ops.gat_in_fwd(dg, xext, Wbad, None, 8, 100)
    with pytest.raises(_abi.GalaError):   # hub rows: the statistics pair keeps those graphs
        dh = ops.DeviceGraph.from_host(g)
        dh.set_split_plan(g.rowptr, 4, chunk=4)
        ops.gat_in_fwd(dh, xext, dev(W), dev(b), 8, 100)


@pytest.fixture(scope="module")
def E():
    import gala
    return gala.torch_ext()


@pytest.mark.parametrize("symmetric", [False, True])
def test_mirror_op_equals_the_three_op_chain(E, symmetric):
    """gat_input_layer_apply (the one autograd op galac / HIPGenerator emit for config 3's layer
    1) against ffn_apply -> head_attn_apply -> gat_aggregate_ffn_apply on the same slot: Y and
    every parameter gradient within 1e-4; the input gets no gradient (the dataset's features).
    On a symmetric pattern (an undirected program's graph) the op runs in T mode
    (gala_gat_in_{fwd,bwd}_t_f32), else the backward walks the transposed pattern."""
    g = layout.gen_graph("uniform", 4000, 50000, seed=3)
    if symmetric:
        src = np.repeat(np.arange(g.n_rows, dtype=np.int32), np.diff(g.rowptr))
        g = layout.csr_build(g.n_rows, g.n_rows, np.concatenate([src, g.col]), np.concatenate([g.col, src]))
    E.slots_clear()
    off, cols = dev(g.rowptr), dev(g.col)
    vals = torch.ones(g.nnz, device="cuda")
    E.slots_push(off, cols, vals, None, 1, False)
    E.slots_push(off, cols, vals, None, 1, False)
    fin, H, D = 100, 8, 32
    X, W, b, wL, bL, wR, bR, dY = layer_inputs(g.n_rows, fin, H, D, seed=9)
    params = [dev(a).requires_grad_() for a in (W, b, wL.reshape(1, -1), bL, wR.reshape(1, -1), bR)]
    x = dev(X)
    assert E.gat_input_layer_eligible(x, params[0], 0, H, 0)
    for relu in (False, True):
        for p in params:
            p.grad = None
        Y = E.gat_input_layer_apply(x, *params, 0, 0.2, 0, relu)
        Y.backward(dev(dY))
        got = [Y.detach().cpu().numpy()] + [p.grad.cpu().numpy() for p in params]
        for p in params:
            p.grad = None
        v1 = E.ffn_apply(x, params[0], params[1])
        aL = E.head_attn_apply(v1, params[2], params[3])
        Y0 = E.gat_aggregate_ffn_apply(aL, v1, params[4], params[5], 0, 0.2, 0)
        if relu:
            Y0 = torch.relu(Y0)
        Y0.backward(dev(dY))
        want = [Y0.detach().cpu().numpy()] + [p.grad.cpu().numpy() for p in params]
        np.testing.assert_allclose(got[0], want[0], **TOL)
        for name, a, w in zip(("W", "b", "wL", "bL", "wR", "bR"), got[1:], want[1:]):
            grad_close(a, w, f"{name} relu={relu}")
    # an input that needs a gradient keeps the chain
    assert not E.gat_input_layer_eligible(x.clone().requires_grad_(), params[0], 0, H, 0)


@pytest.mark.timeout(900)
def test_config3_products_input_layer_against_the_reference_chain():
    """Config 3's layer 1 at the Products shape (N = 2 449 029, E = 126 167 309 stored edges,
    fin = 100 -> 8 x 32): every output row of Y, d_aL, and all parameter gradients against
    the oracle's pass-by-pass REF layer over the fp32 Linear output."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    orc.set_threads(min(16, len(os.sched_getaffinity(0))))
    g = bench.products_graph("uniform", 1.0)
    assert (g.n_rows, g.nnz) == (bench.PRODUCTS_N, bench.PRODUCTS_E)
    fin, H, D = 100, 8, 32
    X, W, b, wL, bL, wR, bR, dY = layer_inputs(g.n_rows, fin, H, D, seed=2024)
    # as the program runs it: the ReLU fused, rows in descending-degree order
    got = gpu_layer(g, X, W, b, wL, bL, wR, bR, dY, H, relu=True, order=ops.degree_order(g.rowptr), tmode=True)
    ref = ref_on_own_logits(g, got, X, W, b, wL, bL, wR, bR, dY, H, relu=True)
    check_against_ref(got, ref)
