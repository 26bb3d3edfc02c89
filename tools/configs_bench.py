#!/usr/bin/env python3
"""Per-config hot-path timings for BASELINE.json's other configs (not the headline line).

  arxiv   ogbn-arxiv-shaped GCN-2, hidden 128: N=169,343, E=1,335,586 stored edges,
          4 norm-scaled F=128 aggregations per step (same step definition as bench.py)
  gat     ogbn-products-shaped GAT layer, 8 heads x D=32 (F=256) and 1 head x D=47:
          fused forward (logits + LeakyReLU + edge softmax + aggregation) and the
          autograd backward (REF chain and FIXED exact gradients)
  reddit  Reddit-shaped GraphSAGE aggregation with kernel sampling sample(20):
          N=232,965, E=114,615,892 (R-MAT power law), F=256, nsamp=20, ra=5, rb=7
  papers  one GPU's shard of the 8-way ogbn-papers100M partition, GCN-3 at F=128
  papers_full  (not in the default set) the whole Papers100M shape on one GPU, F=128
Prints one JSON line per measurement (median of HIP-event timed reps).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
import gala  # noqa: E402
from gala import layout, ops  # noqa: E402


def timeit(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)) / 1e3


def emit(**kw):
    print(json.dumps(kw), flush=True)


def gcn_step(name, hg, F, aggs=4):
    dg = ops.DeviceGraph.from_host(hg)
    N, E = hg.n_rows, hg.nnz
    X = torch.rand((N, F), device="cuda") * 2 - 1
    bufs = [torch.empty_like(X) for _ in range(aggs + 1)]

    def step():
        norm = ops.degree(dg, power=-0.5)
        src = X
        for dst in bufs[1:]:
            ops.row_broadcast(norm, src, out=bufs[0])
            ops.spmm(dg, bufs[0], dst_scale=norm, out=dst)
            src = dst
    t = timeit(step)
    # the same step replayed from one HIP graph (launch overhead off the timeline)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    tg = timeit(graph.replay)
    emit(config=name, op=f"gcn_step_{aggs}_aggregations_hip_graph", ms=tg * 1e3, edges_per_s=aggs * E / tg)
    norm = ops.degree(dg, power=-0.5)
    tk = timeit(lambda: ops.spmm(dg, bufs[0], dst_scale=norm, out=bufs[1]), reps=20)
    alg = 4 * (N + 1) + 4 * E + 8 * N * F + 4 * N
    emit(config=name, op=f"gcn_step_{aggs}_aggregations", ms=t * 1e3, edges_per_s=aggs * E / t, N=N, E=E, F=F)
    emit(config=name, op="spmm_kernel", ms=tk * 1e3, edges_per_s=E / tk, alg_GBps=alg / tk / 1e9,
         roofline_frac=alg / tk / 8e12)


def gat(hg):
    E_ = gala.torch_ext()
    N, E = hg.n_rows, hg.nnz
    off = torch.from_numpy(hg.rowptr).cuda()
    cols = torch.from_numpy(hg.col).cuda()
    t0 = time.time()
    tg, perm = layout.transpose(hg)
    print(f"transpose {time.time()-t0:.1f}s", file=sys.stderr, flush=True)
    # layer slot 0 (REF): backward slot = the forward graph (undirected, as gala.cu registers
    # it); layer slot 1 (FIXED): backward slot = the transpose + its edge permutation
    E_.slots_clear()
    E_.slots_push(off, cols, None, None, 1, False)
    E_.slots_push(off, cols, None, None, 1, False)
    E_.slots_push(off, cols, None, None, 1, False)
    E_.slots_push(torch.from_numpy(tg.rowptr).cuda(), torch.from_numpy(tg.col).cuda(), None, None, 1, False)
    E_.slots_set_transpose_perm(3, torch.from_numpy(perm).cuda())
    dg = ops.DeviceGraph.from_host(hg)
    for heads, D in ((8, 32), (1, 47), (1, 32)):
        F = heads * D
        aL = torch.rand((N, heads), device="cuda")
        aR = torch.rand((N, heads), device="cuda")
        X = torch.rand((N, F), device="cuda")
        tf = timeit(lambda: ops.gat_fwd(dg, aL, aR, X, heads=heads, want_alpha=True), reps=5)
        emit(config="products_gat", op="gat_fwd_fused", heads=heads, D=D, ms=tf * 1e3, edges_per_s=E / tf)
        for mode in (0, 1):
            l = aL.clone().requires_grad_()
            r = aR.clone().requires_grad_()
            x = X.clone().requires_grad_()

            def fb():
                Y = E_.gat_aggregate_apply(l, r, x, mode, 0.2, mode)
                Y.backward(torch.ones_like(Y))
            t = timeit(fb, reps=5, warm=2)
            emit(config="products_gat", op="gat_layer_fwd_bwd", mode=["REF", "FIXED"][mode], heads=heads,
                 D=D, ms=t * 1e3, edges_per_s=E / t)
        if heads == 1:
            # the DSL's layer: attnR = Linear(X) recomputed inside the kernels
            wR = torch.rand(F, device="cuda") - 0.5
            bR = torch.zeros(1, device="cuda")
            emit(config="products_gat", op="gat_fwd_attn", heads=1, D=D,
                 ms=timeit(lambda: ops.gat_fwd_attn(dg, aL, wR, bR, X, want_alpha=True), reps=5) * 1e3)
            al1 = torch.rand(E, device="cuda")
            emit(config="products_gat", op="gat_bwd_attn", heads=1, D=D,
                 ms=timeit(lambda: ops.gat_bwd_attn(dg, aL, wR, bR, X, X, al1), reps=5) * 1e3)
            for mode in (0, 1):
                l = aL.clone().requires_grad_()
                x = X.clone().requires_grad_()
                lin = torch.nn.Linear(F, 1).cuda()

                def fbf():
                    Y = E_.gat_aggregate_ffn_apply(l, x, lin.weight, lin.bias, mode, 0.2, mode)
                    Y.backward(torch.ones_like(Y))
                t = timeit(fbf, reps=5, warm=2)
                emit(config="products_gat", op="gat_layer_ffn_fwd_bwd", mode=["REF", "FIXED"][mode], heads=1,
                     D=D, ms=t * 1e3, edges_per_s=E / t)
        s = torch.rand(E * heads, device="cuda")
        emit(config="products_gat", op="sddvv_lrelu", heads=heads,
             ms=timeit(lambda: ops.sddvv(dg, aL, aR, op=2, heads=heads)) * 1e3)
        emit(config="products_gat", op="edge_softmax_fwd", heads=heads,
             ms=timeit(lambda: ops.edge_softmax(dg, s, heads=heads)) * 1e3)
        emit(config="products_gat", op="edge_softmax_bwd", heads=heads,
             ms=timeit(lambda: ops.edge_softmax_bwd(dg, s, s, heads=heads)) * 1e3)
        for mode in (0, 1):
            emit(config="products_gat", op="gat_bwd_fused", mode=["REF", "FIXED"][mode], heads=heads, F=F,
                 ms=timeit(lambda: ops.gat_bwd(dg, aL, aR, X, X, s, heads=heads, mode=mode)) * 1e3)
        emit(config="products_gat", op="sddmm", heads=heads, F=F,
             ms=timeit(lambda: ops.sddmm(dg, X, X, heads=heads)) * 1e3)
        gw = dg.with_values(s, val_heads=heads)
        emit(config="products_gat", op="weighted_spmm", heads=heads, F=F,
             ms=timeit(lambda: ops.spmm(gw, X)) * 1e3)


def reddit(hg):
    dg = ops.DeviceGraph.from_host(hg)
    N, E = hg.n_rows, hg.nnz
    deg = hg.degrees()
    F = 256
    X = torch.rand((N, F), device="cuda")
    t = timeit(lambda: ops.spmm(dg, X, nsamp=20, ra=5, rb=7))
    alg = 4 * (N + 1) + 4 * N * 20 + 8 * N * F
    emit(config="reddit_sage", op="spmm_kernel_sampled_n20", ms=t * 1e3, sampled_edges_per_s=N * 20 / t,
         alg_GBps=alg / t / 1e9, roofline_frac=alg / t / 8e12, deg_max=int(deg.max()), deg_mean=float(deg.mean()))
    t = timeit(lambda: ops.spmm(dg, X), reps=3, warm=1)
    emit(config="reddit_sage", op="spmm_full_F256", ms=t * 1e3, edges_per_s=E / t)


def papers_full():
    """The whole ogbn-papers100M shape (111 M vertices, 1.73 B edges, F = 128) resident on ONE
    MI355X: X and Y are 57 GB each.  Integer-valued features make the sum order-free, so
    2000 sampled rows are checked exactly against a float64 gather of the same rows."""
    n = 111_059_956
    t0 = time.time()
    hg = layout.gen_graph("uniform", n, (1_726_745_828 - n) // 2, seed=42)
    print(f"graph built {time.time()-t0:.1f}s N={hg.n_rows} E={hg.nnz}", file=sys.stderr, flush=True)
    dg = ops.DeviceGraph.from_host(hg)
    N, E, F = hg.n_rows, hg.nnz, 128
    X = torch.randint(-8, 9, (N, F), device="cuda", dtype=torch.float32)
    Y = torch.empty_like(X)
    t = timeit(lambda: ops.spmm(dg, X, out=Y), reps=5, warm=1)
    print(f"spmm timed {time.time()-t0:.1f}s", file=sys.stderr, flush=True)
    rng = np.random.default_rng(7)
    rows = np.sort(rng.choice(N, 2000, replace=False))
    worst = 0.0
    for r in rows:
        c = torch.from_numpy(hg.col[hg.rowptr[r]:hg.rowptr[r + 1]].astype(np.int64)).cuda()
        ref = X.index_select(0, c).double().sum(0)
        worst = max(worst, float((Y[r].double() - ref).abs().max()))
    alg = 4 * (N + 1) + 4 * E + 8 * N * F
    emit(config="papers100M_full_1gpu", op="spmm_kernel", ms=t * 1e3, edges_per_s=E / t, alg_GBps=alg / t / 1e9,
         roofline_frac=alg / t / 8e12, gather_GB=E * F * 4 / 1e9, N=N, E=E, F=F,
         max_mem_GB=torch.cuda.max_memory_allocated() / 1e9, sampled_rows_max_abs_err=worst)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="arxiv,gat,reddit,papers")
    a = ap.parse_args()
    w = a.which.split(",")
    if "arxiv" in w:
        gcn_step("arxiv_gcn", layout.gen_graph("uniform", 169_343, (1_335_586 - 169_343) // 2, seed=42), 128)
    if "gat" in w:
        gat(layout.gen_graph("uniform", 2_449_029, 61_859_140, seed=42))
    if "reddit" in w:
        reddit(layout.gen_graph("rmat", 232_965, (114_615_892 - 232_965) // 2, seed=42))
    if "papers" in w:
        # config 5, one GPU's share of the 8-way vertex partition of ogbn-papers100M
        # (N = 111,059,956 / 8, E = 1,726,745,828 / 8), GCN-3 at F = 128: 3 forward + 3
        # backward aggregations per step (the cut-edge halo exchange needs the 8 ranks)
        n = 111_059_956 // 8
        gcn_step("papers100M_shard_of_8", layout.gen_graph("uniform", n, (1_726_745_828 // 8 - n) // 2, seed=42),
                 128, aggs=6)
    if "papers_full" in w:
        papers_full()


if __name__ == "__main__":
    main()
