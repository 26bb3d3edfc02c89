#!/usr/bin/env python3
"""Probe (measurement, not a test): the SpMM on config 5's short rows (11.1 M vertices,
2.45 stored edges per row) and on the Products shape (51 per row) at F = 32 / 128 / 256, and
the FFN weight gradient (gala_dense_grad_f32) on config 5's and config 2's layer shapes.
Run it once with GALA_SPMM_SPARSE_ROWS=0 (the wide row groups) and once without (the short-row
dispatch); one JSON line per case, with GALA_SPMM_SPARSE_ROWS in each."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
from gala import layout, ops  # noqa: E402


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    mode = os.environ.get("GALA_SPMM_SPARSE_ROWS", "1")
    graphs = {"config5": (11_105_995, (27_262_853 - 11_105_995) // 2),
              "products": (2_449_029, (126_167_309 - 2_449_029) // 2)}
    for name, (n, und) in graphs.items():
        hg = layout.gen_graph("uniform", n, und, seed=42)
        dg = ops.DeviceGraph.from_host(hg)
        for F in (32, 128, 256):
            X = torch.rand((n, F), device="cuda")
            ms = timed(lambda: ops.spmm(dg, X))
            gather = hg.nnz * F * 4
            print(json.dumps({"op": "spmm", "graph": name, "rows": n, "edges": hg.nnz, "F": F, "ms": round(ms, 4),
                              "gather_GBps": round(gather / ms / 1e6, 1), "GALA_SPMM_SPARSE_ROWS": mode}), flush=True)
            del X
        del dg
    if mode == "0":
        return
    for N, K, M in ((11_105_995, 128, 128), (11_105_995, 128, 172), (169_343, 128, 128), (2_449_029, 100, 32)):
        X = torch.rand((N, K), device="cuda")
        dY = torch.rand((N, M), device="cuda")
        ms = timed(lambda: ops.dense_grad(X, dY))
        tf = 2.0 * N * K * M / ms / 1e9
        print(json.dumps({"op": "dense_grad", "N": N, "K": K, "M": M, "ms": round(ms, 4), "TFLOPs": round(tf, 1),
                          "GBps": round(4 * N * (K + M) / ms / 1e6, 1)}), flush=True)
        del X, dY


if __name__ == "__main__":
    main()
