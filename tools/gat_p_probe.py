#!/usr/bin/env python3
"""Probe: the 8-head GAT layer step of bench.py (config 3's shape) with the backward's alpha
recomputed from the gathered source logit aR[c] (bench.py's step) against alpha from the
forward's parked per-edge p (gala_gat_fwd_stats_f32 want_p: E*H floats written once, read
once in CSR order instead of one random aR[c] line per edge).  Both backward outputs are
checked bit-identical.  Measurement only."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, ROOT)
from gala import ops  # noqa: E402
import bench  # noqa: E402


def main():
    dev = torch.device("cuda")
    hg = bench.products_graph("uniform", 1.0)
    dg = ops.DeviceGraph.from_host(hg)
    H, F = bench.GAT_HEADS, bench.GAT_HEADS * bench.GAT_HEAD_F
    N = hg.n_rows
    gen = torch.Generator(device=dev).manual_seed(4321)
    X = torch.rand((N, F), device=dev, generator=gen) * 2 - 1
    dY = torch.rand((N, F), device=dev, generator=gen) * 2 - 1
    aL = torch.rand((N, H), device=dev, generator=gen) - 0.5
    wR = (torch.rand(F, device=dev, generator=gen) - 0.5) * 0.2
    bR = torch.zeros(H, device=dev)
    st = {}

    def step_aR():
        Y, q, Ym, sma, aRo = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
        st["a"] = ops.gat_bwd_stats(dg, aL, aRo, dY, q, Y, Ym, sma, heads=H)

    def step_p():
        Y, q, Ym, sma, aRo, p = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True, want_p=True)
        st["p"] = ops.gat_bwd_stats(dg, aL, None, dY, q, Y, Ym, sma, heads=H, p=p)

    for name, fn in (("aR_gather", step_aR), ("parked_p", step_p)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"variant": name, "ms_per_step": e0.elapsed_time(e1) / 5, "E": hg.nnz, "heads": H, "F": F}),
              flush=True)
    same = all(torch.equal(a, b) for a, b in zip(st["a"], st["p"]))
    print(json.dumps({"backward_outputs_bit_identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
