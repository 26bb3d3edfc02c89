"""R-MAT Products-shape REF-order SpMM (F = 32): the longest hub chains in a launch of their
own, a whole CU each (gala_split_plan_t.n_long, the default), against one hub launch
(GALA_HUB_LONG=0), alternated in one process; outputs compared bit for bit.  One JSON line
per variant: median ms over rounds of 10 calls.

    python tools/hub_long_ab.py [--rounds 7]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, ROOT)
from gala import ops  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    hg = bench.products_graph("rmat", 1.0)
    graphs = {}
    for name, env in (("long_own_cu", "131072"), ("one_hub_launch", "0")):
        os.environ["GALA_HUB_LONG"] = env
        graphs[name] = ops.DeviceGraph.from_host(hg)
    os.environ.pop("GALA_HUB_LONG")
    timer = bench.Timer(True)
    X = torch.rand((hg.n_rows, 32), device="cuda") * 2 - 1
    outs = {k: ops.spmm(g, X) for k, g in graphs.items()}
    torch.cuda.synchronize()
    same = torch.equal(outs["long_own_cu"], outs["one_hub_launch"])
    t = {k: [] for k in graphs}
    for _ in range(a.rounds):
        for k, g in graphs.items():
            Y = outs[k]
            t[k].append(timer(lambda: ops.spmm(g, X, out=Y), 10) * 1e3)
    for k in graphs:
        print(json.dumps({"variant": k, "n_long": int(graphs[k]._split["plan"].n_long),
                          "ms_median": float(np.median(t[k])), "ms_all": [round(v, 4) for v in t[k]],
                          "bit_identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
