#!/usr/bin/env python3
"""Time K7 (gala_row_sum_f32) in the reference's order against the chunked hub mode on the
Products-shaped uniform and R-MAT graphs, 1 and 8 heads (JSON lines)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, ROOT)
from gala import layout, ops  # noqa: E402
import bench  # noqa: E402


def main():
    timer = bench.Timer(True)
    for kind in ("uniform", "rmat"):
        g = layout.gen_graph(kind, 2_449_029, 61_859_140, seed=42)
        dg = ops.DeviceGraph.from_host(g)
        for heads in (1, 8):
            v = torch.rand(g.nnz * heads, device="cuda") * 2 - 1
            out = torch.empty(g.n_rows * heads, device="cuda")
            rec = {"graph": kind, "heads": heads, "edges": g.nnz, "hub_rows": dg.split_rows}
            for hub in ("exact", "chunked"):
                ms = timer(lambda: ops.row_sum(dg, v, heads=heads, out=out, hub=hub), 10) * 1e3
                rec[f"{hub}_ms"] = ms
                rec[f"{hub}_GBps"] = (4 * g.nnz * heads + 4 * (g.n_rows + 1) + 4 * g.n_rows * heads) / ms / 1e6
            print(json.dumps(rec), flush=True)
            del v, out


if __name__ == "__main__":
    main()
