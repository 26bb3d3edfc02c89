#!/usr/bin/env python3
"""Profiling target: the 8-head (F=256) GAT forward on the Products-shaped uniform graph,
row-statistics (RC, aR_out) vs q-only (RC), then the row-statistics backward; 5 launches
each, nothing else on the GPU between them."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
from gala import layout, ops  # noqa: E402

H, F = 8, 256
hg = layout.gen_graph("uniform", 2_449_029, 61_859_140, seed=42)
dg = ops.DeviceGraph.from_host(hg)
N = hg.n_rows
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
dY = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
aL = torch.rand((N, H), device="cuda", generator=g) - 0.5
wR = (torch.rand(F, device="cuda", generator=g) - 0.5) * 0.2
bR = torch.zeros(H, device="cuda")
for _ in range(5):
    st = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
torch.cuda.synchronize()
for _ in range(5):
    yq = ops.gat_fwd_ex(dg, aL, X, wR=wR, bR=bR, heads=H, factored="q")
torch.cuda.synchronize()
Y, q, Ym, sma, aRo = st
for _ in range(5):
    ops.gat_bwd_stats(dg, aL, aRo, dY, q, Y, Ym, sma, heads=H)
torch.cuda.synchronize()
print("done")
