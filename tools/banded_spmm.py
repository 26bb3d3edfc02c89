#!/usr/bin/env python3
"""The headline SpMM (F = 32, dst norm) on the banded Products-shaped graph alone, for PMC
passes (tools/gpu_job.sh pmccmd=banded,python3,tools/banded_spmm.py): the kernel name is the
uniform graph's, so bench.py's own PMC run cannot tell the two apart.  Runs 1 warm-up + 5
SpMMs and prints their HIP-event time."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gala-gnn-acceleration-language_amd"), ROOT]
from gala import ops  # noqa: E402
import bench  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "banded"
    hg = bench.products_graph(kind, float(os.environ.get("GALA_SCALE", "1.0")))
    dg = ops.DeviceGraph.from_host(hg)
    norm = ops.degree(dg, power=-0.5)
    X = torch.rand((hg.n_rows, 32), device="cuda") * 2 - 1
    Xs = ops.row_broadcast(norm, X)
    Y = torch.empty_like(X)
    t = bench.Timer(True)(lambda: ops.spmm(dg, Xs, out=Y, dst_scale=norm), 5)
    print(json.dumps({"graph": kind, "N": hg.n_rows, "E": hg.nnz, "spmm_ms": t * 1e3}), flush=True)


if __name__ == "__main__":
    main()
