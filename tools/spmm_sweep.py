#!/usr/bin/env python3
"""Kernel-level timing sweep on the GPU box (tuning aid, not a test).

Times gala ops on a Products-shaped graph with HIP events (median of reps) and prints
one JSON line per case: ms, edges/s, algorithmic GB/s.
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
from gala import layout, ops  # noqa: E402


def timeit(fn, reps=10, warm=2):
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
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="uniform")
    ap.add_argument("--n", type=int, default=2_449_029)
    ap.add_argument("--u", type=int, default=61_859_140)
    ap.add_argument("--F", default="8,16,32,64,128")
    ap.add_argument("--ops", default="spmm,spmm_scaled,degree,sddvv,softmax,sddmm,gat")
    ap.add_argument("--band", type=int, default=4096, help="banded graph: neighbour offset bound")
    ap.add_argument("--sort-rows", action="store_true")
    ap.add_argument("--pad", action="store_true", help="row-padded X / Y (stride F rounded up to 4)")
    args = ap.parse_args()
    t0 = time.time()
    if args.graph == "banded":  # locality: every neighbour within +-band of its row
        rng = np.random.default_rng(42)
        m = 2 * args.u
        src = rng.integers(0, args.n, m, dtype=np.int64)
        dst = np.clip(src + rng.integers(-args.band, args.band + 1, m), 0, args.n - 1)
        ids = np.arange(args.n, dtype=np.int64)
        hg = layout.csr_build(args.n, args.n, np.concatenate([src, ids]).astype(np.int32),
                              np.concatenate([dst, ids]).astype(np.int32))
    else:
        hg = layout.gen_graph(args.graph, args.n, args.u, seed=42)
    if args.sort_rows:  # experiment: rows relabelled by descending degree (stable)
        deg = np.diff(hg.rowptr)
        order = np.argsort(-deg, kind="stable")
        rp = np.zeros(hg.n_rows + 1, np.int64)
        rp[1:] = np.cumsum(deg[order])
        starts = hg.rowptr[:-1][order].astype(np.int64)
        idx = np.repeat(starts - rp[:-1], deg[order]) + np.arange(hg.nnz)
        hg = layout.HostGraph(hg.n_rows, hg.n_cols, rp.astype(np.int32), hg.col[idx])
    print(f"graph built {time.time()-t0:.1f}s N={hg.n_rows} E={hg.nnz}", file=sys.stderr, flush=True)
    dg = ops.DeviceGraph.from_host(hg)
    N, E = hg.n_rows, hg.nnz
    todo = args.ops.split(",")
    norm = ops.degree(dg, power=-0.5)
    for F in [int(f) for f in args.F.split(",")]:
        X = torch.rand((N, F), device="cuda") * 2 - 1
        if args.pad:
            X = ops.pad_rows(X)
        Y = ops.spmm(dg, X)
        base = 4 * (N + 1) + 4 * E + 8 * N * F
        if "spmm" in todo:
            ms = timeit(lambda: ops.spmm(dg, X, out=Y))
            print(json.dumps({"op": "spmm", "F": F, "ms": ms, "edges_per_s": E / ms * 1e3, "alg_GBps": base / ms / 1e6}), flush=True)
        if "spmm_scaled" in todo:
            ms = timeit(lambda: ops.spmm(dg, X, src_scale=norm, dst_scale=norm, out=Y))
            print(json.dumps({"op": "spmm_scaled", "F": F, "ms": ms, "edges_per_s": E / ms * 1e3, "alg_GBps": (base + 8 * N) / ms / 1e6}), flush=True)
        if "gat" in todo:
            aL = torch.rand(N, device="cuda")
            aR = torch.rand(N, device="cuda")
            ms = timeit(lambda: ops.gat_fwd(dg, aL, aR, X))
            print(json.dumps({"op": "gat_fwd", "F": F, "ms": ms, "edges_per_s": E / ms * 1e3, "alg_GBps": (base + 8 * N) / ms / 1e6}), flush=True)
        if "sddmm" in todo:
            ms = timeit(lambda: ops.sddmm(dg, X, X))
            print(json.dumps({"op": "sddmm", "F": F, "ms": ms, "edges_per_s": E / ms * 1e3, "alg_GBps": (4 * (N + 1) + 8 * E + 8 * N * F) / ms / 1e6}), flush=True)
    if "rocsparse" in todo:
        # vendor reference point: torch.sparse CSR matmul -> hipSPARSE/rocSPARSE SpMM
        A = torch.sparse_csr_tensor(dg.rowptr, dg.col, torch.ones(E, device="cuda"), size=(N, N))
        for F in [int(f) for f in args.F.split(",")]:
            X = torch.rand((N, F), device="cuda")
            try:
                ms = timeit(lambda: torch.sparse.mm(A, X), reps=5)
                print(json.dumps({"op": "rocsparse_spmm", "F": F, "ms": ms, "edges_per_s": E / ms * 1e3}), flush=True)
            except Exception as e:
                print(json.dumps({"op": "rocsparse_spmm", "F": F, "error": repr(e)[:200]}), flush=True)
    if "degree" in todo:
        ms = timeit(lambda: ops.degree(dg, power=-0.5))
        print(json.dumps({"op": "degree", "ms": ms, "alg_GBps": (4 * (N + 1) + 4 * N) / ms / 1e6}), flush=True)
    if "sddvv" in todo:
        a = torch.rand(N, device="cuda")
        ms = timeit(lambda: ops.sddvv(dg, a, a))
        print(json.dumps({"op": "sddvv", "ms": ms, "edges_per_s": E / ms * 1e3, "alg_GBps": (4 * (N + 1) + 8 * E + 8 * N) / ms / 1e6}), flush=True)
    if "softmax" in todo:
        s = torch.rand(E, device="cuda")
        ms = timeit(lambda: ops.edge_softmax(dg, s))
        print(json.dumps({"op": "softmax_fwd", "ms": ms, "edges_per_s": E / ms * 1e3, "alg_GBps": (4 * (N + 1) + 8 * E) / ms / 1e6}), flush=True)
        d = torch.rand(E, device="cuda")
        ms = timeit(lambda: ops.edge_softmax_bwd(dg, s, d))
        print(json.dumps({"op": "softmax_bwd", "ms": ms, "edges_per_s": E / ms * 1e3, "alg_GBps": (4 * (N + 1) + 12 * E) / ms / 1e6}), flush=True)


if __name__ == "__main__":
    main()
