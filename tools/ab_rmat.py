#!/usr/bin/env python3
"""In-process A/B of builds of libgala_hip.so on a Products-shape SpMM, F = 32: the R-MAT graph
in the reference's hub order (bench.py's "rmat" family) or the uniform graph (the headline's):
tools/ab/libgala_hip_<label>.so and "tree" (this tree's build), alternated on the same inputs;
medians and bit-identity to the tree.  Measurement only.
    python tools/ab_rmat.py [rounds] [rmat|uniform] [spmm|wspmm|sddvv|sddmm]
wspmm: the SpMM with one value per edge; sddvv: K5 (ADD, one head: a[row] + b[col] per edge); sddmm: K9 at F = 32.
"""
import glob
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from ab_gat import load  # noqa: E402
from gala import _abi, ops  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    libs = {os.path.basename(f)[len("libgala_hip_"):-3]: load(f)
            for f in sorted(glob.glob(os.path.join(ROOT, "tools", "ab", "libgala_hip_*.so")))}
    libs["tree"] = _abi.lib()
    kind = sys.argv[2] if len(sys.argv) > 2 else "rmat"
    hg = bench.products_graph(kind, 1.0)
    dg = ops.DeviceGraph.from_host(hg)
    op = sys.argv[3] if len(sys.argv) > 3 else "spmm"
    X = torch.rand((hg.n_rows, 32), device="cuda") * 2 - 1
    a = torch.rand(hg.n_rows, device="cuda") - 0.5
    b = torch.rand(hg.n_rows, device="cuda") - 0.5
    Y = torch.empty_like(X)
    gw = dg.with_values(torch.rand(hg.nnz, device="cuda")) if op == "wspmm" else None
    res = {}

    def run():
        if op == "spmm":
            ops.spmm(dg, X, out=Y)
            res["y"] = Y
        elif op == "wspmm":
            ops.spmm(gw, X, out=Y)
            res["y"] = Y
        elif op == "sddvv":
            res["y"] = ops.sddvv(dg, a, b)
        else:
            res["y"] = ops.sddmm(dg, X, X)
    timer = bench.Timer(True)
    outs, samples = {}, {k: [] for k in libs}
    for r in range(rounds + 1):
        for k in libs:
            _abi._lib = libs[k]
            run()
            torch.cuda.synchronize()
            outs.setdefault(k, res["y"].clone())
            t = timer(run, 10)
            if r:
                samples[k].append(round(t * 1e3, 4))
    _abi._lib = libs["tree"]
    print(json.dumps({"graph": kind, "op": op, "medians_ms": {k: sorted(v)[len(v) // 2] for k, v in samples.items()}, "samples": samples,
                      "bit_identical_to_tree": {k: bool(torch.equal(outs[k], outs["tree"])) for k in libs}}), flush=True)


if __name__ == "__main__":
    main()
