#!/usr/bin/env python3
"""Profiling aid: the 8-head GAT forward (F = 256, alpha out) on the Products shape, a few
launches, for rocprofv3 PMC passes (tools/gpu_pmc_gat.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gala-gnn-acceleration-language_amd"))
from gala import layout, ops  # noqa: E402

hg = layout.gen_graph("uniform", 2_449_029, 61_859_140, seed=42)
dg = ops.DeviceGraph.from_host(hg)
N, H, F = hg.n_rows, 8, 256
X = torch.rand((N, F), device="cuda")
aL = torch.rand((N, H), device="cuda")
aR = torch.rand((N, H), device="cuda")
for _ in range(3):
    ops.gat_fwd(dg, aL, aR, X, heads=H, want_alpha=True)
    ops.spmm(dg.with_values(torch.rand(hg.nnz * H, device="cuda"), val_heads=H), X)
torch.cuda.synchronize()
print("done")
