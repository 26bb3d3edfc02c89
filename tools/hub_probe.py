#!/usr/bin/env python3
"""Probe of the REF-order hub-row SpMM (k_spmm_hub_exact) on synthetic shapes:
  one   -- one hub row of D edges (default 388 138, the R-MAT Products maximum), every other
           row a self-loop: the serial chain of the longest row alone
  many  -- R rows of K edges each (default 27 000 x 2 800, the R-MAT Products hub mass)
Each prints the REF-order time, the chunked fast mode's time, and the same-process gather
probe of the hub edges (no order, no output rows)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, ROOT)
from gala import layout, ops  # noqa: E402
import bench  # noqa: E402


def graph(N, hub_rows, K, seed=3, span=None):
    rng = np.random.default_rng(seed)
    deg = np.ones(N, np.int64)
    deg[hub_rows] = K
    rp = np.zeros(N + 1, np.int64)
    np.cumsum(deg, out=rp[1:])
    col = np.arange(N, dtype=np.int32).repeat(deg)
    for r in hub_rows:
        col[rp[r]:rp[r + 1]] = np.sort(rng.integers(0, span or N, K).astype(np.int32))
    return layout.HostGraph(N, N, rp.astype(np.int32), col)


def run(tag, hg, F, timer):
    X = torch.rand((hg.n_rows, F), device="cuda") * 2 - 1
    Y = torch.empty_like(X)
    dg = ops.DeviceGraph.from_host(hg)
    te = timer(lambda: ops.spmm(dg, X, out=Y), 5)
    Ye = Y.clone()
    tc = timer(lambda: ops.spmm(dg, X, out=Y, hub="chunked"), 5)
    tg = bench.gather_ceiling(dg.col, X, timer)
    print(json.dumps({"case": tag, "F": F, "hub_rows": dg.split_rows, "edges": hg.nnz,
                      "exact_ms": te * 1e3, "chunked_ms": tc * 1e3,
                      "gather_ms": None if tg is None else tg * 1e3,
                      "max_abs_diff": float((Y - Ye).abs().max())}), flush=True)


def main():
    N = 2449029
    F = int(os.environ.get("GALA_F", "32"))
    timer = bench.Timer(True)
    which = sys.argv[1:] or ["one", "l2", "many"]
    if "one" in which:
        D = int(os.environ.get("GALA_HUB_D", "388138"))
        run(f"one x {D}", graph(N, [7], D), F, timer)
    if "l2" in which:   # the same row over 2048 columns: the gathers hit L2, the chain is the cost
        D = int(os.environ.get("GALA_HUB_D", "388138"))
        run(f"one x {D} over 2048 columns", graph(N, [7], D, span=2048), F, timer)
    if "many" in which:
        R, K = 27000, 2800
        rows = np.random.default_rng(5).choice(N, R, replace=False)
        run(f"many {R} x {K}", graph(N, rows, K), F, timer)


if __name__ == "__main__":
    main()
