#!/usr/bin/env python3
"""Experiment driver: time the 8-head (F=256) and 1-head (F=32) GAT forward kernels of an
alternative libgala_hip.so build (argv[1]: its directory) on the Products-shaped uniform
graph; prints one JSON line per op.  Y rows of the first variant are kept in
gpurun_out/gatv_ref_*.pt and later variants report their max deviation from them.

A/B driver for kernel experiments: each variant is libgala_hip.so relinked with gat.hip
built from a temporary patch (exp/<name>/).  The round-2 variants (batch size, occupancy
hints, DPP reductions, column prefetch, no padding masks, no Ym / accm / aR_out, non-temporal
stores; profiles/r02_gat_fwd_variants_stores.jsonl) changed nothing beyond
1 %, so none of those patches is in the tree."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
from gala import _abi  # noqa: E402

_abi.LIB_PATH = os.path.join(os.path.abspath(sys.argv[1]), "libgala_hip.so")
from gala import layout, ops  # noqa: E402


def timeit(fn, reps=10):
    fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ts]))


def main():
    name = os.path.basename(os.path.abspath(sys.argv[1]))
    kind = os.environ.get("GALA_GRAPH", "uniform")   # "rmat": skewed, with the hub-row plan
    hg = layout.gen_graph(kind, 2_449_029, 61_859_140, seed=42)
    dg = ops.DeviceGraph.from_host(hg)
    N = hg.n_rows
    g = torch.Generator(device="cuda").manual_seed(0)
    for H, F in ((8, 256), (1, 32)):
        X = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
        aL = torch.rand((N, H), device="cuda", generator=g) - 0.5
        wR = (torch.rand(F, device="cuda", generator=g) - 0.5) * 0.2
        bR = torch.zeros(H, device="cuda")
        Y = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)[0]
        ref = os.path.join(ROOT, "gpurun_out", f"gatv_ref_{H}.pt")
        dev = None
        if os.path.exists(ref):
            R = torch.load(ref, weights_only=True).cuda()
            dev = float((Y[:20000] - R).abs().max())
        else:
            torch.save(Y[:20000].cpu(), ref)
        dY = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
        _, q, Ym, sma, aRo = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
        rec = {"variant": name, "graph": kind, "heads": H, "F": F,
               "fwd_stats_rc_ms": timeit(lambda: ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)),
               "bwd_stats_ms": timeit(lambda: ops.gat_bwd_stats(dg, aL, aRo, dY, q, Y, Ym, sma, heads=H)),
               "fwd_q_rc_ms": timeit(lambda: ops.gat_fwd_ex(dg, aL, X, wR=wR, bR=bR, heads=H, factored="q")),
               "max_dev_vs_first": dev}
        print(json.dumps(rec), flush=True)
        del X, Y, dY, q, Ym, sma, aRo
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
