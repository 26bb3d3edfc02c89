#!/usr/bin/env python3
"""Profiling aid: the 8-head GAT layer kernels (F = 256) on the ogbn-products shape, three
launches each, for rocprofv3 kernel-trace and PMC passes (tools/gpu_pmc_gat.sh):
    1. gala_gat_fwd_ex_f32, REF, q only (the layer's forward; alpha recomputed later)
    2. gala_spmm_f32 weighted, 8 value heads (the same gathers with a stored weight)
    3. gala_gat_bwd_fused_f32 (recomputed alpha, dX fused)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gala-gnn-acceleration-language_amd"))
from gala import layout, ops  # noqa: E402

hg = layout.gen_graph("uniform", 2_449_029, 61_859_140, seed=42)
dg = ops.DeviceGraph.from_host(hg)
N, H, F = hg.n_rows, 8, 256
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.rand((N, F), device="cuda", generator=g)
dY = torch.rand((N, F), device="cuda", generator=g)
aL = torch.rand((N, H), device="cuda", generator=g)
aR = torch.rand((N, H), device="cuda", generator=g)
val = torch.rand(hg.nnz * H, device="cuda", generator=g)
for _ in range(3):
    _, q = ops.gat_fwd_ex(dg, aL, X, aR=aR, heads=H, factored="q")
for _ in range(3):
    ops.spmm(dg.with_values(val, val_heads=H), X)
for _ in range(3):
    ops.gat_bwd_fused(dg, aL, X, dY, q, aR=aR, heads=H)
torch.cuda.synchronize()
print("done")
