#!/usr/bin/env python3
"""Profiling target: the F=32 SpMM on the R-MAT Products-shaped graph with its hub-row plan
(k_spmm_rows_chunks + k_spmm_fixup), 5 launches, for rocprofv3 --pmc passes."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
from gala import layout, ops  # noqa: E402

hg = layout.gen_graph("rmat", 2_449_029, 61_859_140, seed=42)
dg = ops.DeviceGraph.from_host(hg)
X = torch.rand((hg.n_rows, 32), device="cuda") * 2 - 1
Y = torch.empty_like(X)
for _ in range(5):
    ops.spmm(dg, X, out=Y)
torch.cuda.synchronize()
print("done", dg.split_rows)
