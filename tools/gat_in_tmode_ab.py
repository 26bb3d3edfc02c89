#!/usr/bin/env python3
"""In-process A/B of the input-space GAT layer's two backward formulations at config 3's
Products shape (8 heads x 32 from 100 inputs): the walk (gala_gat_in_fwd_f32, then
gala_gat_in_bwd_f32 gathering the extended rows over the transposed pattern) against T mode
(gala_gat_in_fwd_t_f32: a q pass, then the forward forming the backward's per-column
aggregates T; gala_gat_in_bwd_t_f32 reading T).  Medians of 5 calls per round, alternated,
and the largest difference of Y / q / d_aL / M between the modes (relative to each
tensor's largest entry).  Measurement only.
    python tools/gat_in_tmode_ab.py [rounds] [scale]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gala import ops  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    dev = torch.device("cuda")
    hg = bench.products_graph("uniform", scale)
    dg = ops.DeviceGraph.from_host(hg, split=False)
    H, D, FIN = bench.GAT_HEADS, bench.GAT_HEAD_F, bench.GAT_IN_F
    F, N = H * D, hg.n_rows
    gen = torch.Generator(device=dev).manual_seed(4321)
    Xin = torch.rand((N, FIN), device=dev, generator=gen) * 2 - 1
    dY = torch.rand((N, F), device=dev, generator=gen) * 2 - 1
    W = (torch.rand((F, FIN), device=dev, generator=gen) * 2 - 1) / 10
    b = (torch.rand(F, device=dev, generator=gen) - 0.5) * 0.2
    wL, wR = ((torch.rand(F, device=dev, generator=gen) - 0.5) * 0.6 for _ in range(2))
    bL, bR = ((torch.rand(H, device=dev, generator=gen) - 0.5) * 0.2 for _ in range(2))
    order = torch.from_numpy(ops.degree_order(hg.rowptr)).to(dev)
    u, c = ops.gat_in_compose(W, b, wL, bL, wR, bR, H)
    xext = ops.gat_in_prep(Xin, u, c, H)
    T = torch.empty(N, 896, device=dev)
    res = {}

    def fwd(tm):
        res[tm, "f"] = ops.gat_in_fwd(dg, xext, W, b, H, FIN, order=order, relu=True, T=T if tm else None)

    def bwd(tm):
        Y, Ym, q, sma = res[tm, "f"]
        res[tm, "b"] = ops.gat_in_bwd(dg, xext, dY, Y, Ym, sma, H, FIN, order=order, relu=True,
                                      T=T if tm else None)
    timer = bench.Timer(True)
    samples = {m: {"fwd": [], "bwd": []} for m in ("walk", "tmode")}
    for r in range(rounds + 1):
        for tm, name in ((False, "walk"), (True, "tmode")):
            fwd(tm)
            bwd(tm)
            torch.cuda.synchronize()
            tf = timer(lambda: fwd(tm), 5)
            tb = timer(lambda: bwd(tm), 5)
            if r:
                samples[name]["fwd"].append(round(tf * 1e3, 4))
                samples[name]["bwd"].append(round(tb * 1e3, 4))
    med = {k: {p: sorted(v)[len(v) // 2] for p, v in d.items()} for k, d in samples.items()}
    # the two modes' outputs (the walk's q is the MFMA-ordered sum, T mode's the sequential one)
    fwd(False), bwd(False), fwd(True), bwd(True)
    torch.cuda.synchronize()
    a = list(res[False, "f"]) + list(res[False, "b"])
    t = list(res[True, "f"]) + list(res[True, "b"])
    names = ("Y", "Ym", "q", "sma", "daL", "M")
    rel = {n: float((x - y).abs().max() / max(float(x.abs().max()), 1e-30)) for n, x, y in zip(names, a, t)}
    print(json.dumps({"n": N, "nnz": int(hg.nnz), "medians_ms": med, "samples": samples, "max_rel_diff": rel}),
          flush=True)


if __name__ == "__main__":
    main()
