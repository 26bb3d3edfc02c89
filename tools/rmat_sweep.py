#!/usr/bin/env python3
"""R-MAT Products-shape SpMM schedule sweep (bench.py's second family): hub-row threshold,
chunk length and the degree-ordered row schedule, against the unordered gather probe of the
same column array.  One JSON line per setting (HIP events, mean of 10)."""
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
    F = int(os.environ.get("GALA_F", "32"))
    hg = bench.products_graph("rmat", float(os.environ.get("GALA_SCALE", "1.0")))
    timer = bench.Timer(True)
    X = torch.rand((hg.n_rows, F), device="cuda") * 2 - 1
    Y = torch.empty_like(X)
    base = ops.DeviceGraph.from_host(hg, split=False)
    t = timer(lambda: ops.spmm(base, X, out=Y), 10)
    print(json.dumps({"setting": "no plan", "ms": t * 1e3}), flush=True)
    ref = Y.clone()
    for thr, chunk, order in [(1024, 512, True), (1024, 512, False), (0, 512, True), (512, 256, True),
                              (2048, 512, True), (4096, 1024, True), (1024, 1024, True), (1024, 256, True),
                              (8192, 2048, True), (16384, 4096, True)]:
        dg = ops.DeviceGraph.from_host(hg, split=False)
        dg.set_split_plan(hg.rowptr, thr, chunk=chunk, row_order=order)
        t = timer(lambda: ops.spmm(dg, X, out=Y), 10)
        same = bool(torch.equal(Y, ref)) if thr == 0 else None
        print(json.dumps({"setting": f"thr={thr} chunk={chunk} order={order}", "ms": t * 1e3,
                          "split_rows": dg.split_rows, "bitexact_vs_unsplit": same}), flush=True)
        del dg
    tc = bench.gather_ceiling(base.col, X, timer)
    print(json.dumps({"setting": "gather probe (CSR order)", "ms": None if tc is None else tc * 1e3}), flush=True)
    # the same gather in the degree-ordered row schedule's edge order
    import numpy as np
    from gala import _abi
    rp = np.ascontiguousarray(hg.rowptr, np.int32)
    order = np.empty(hg.n_rows, np.int32)
    _abi.call("gala_host_row_order", hg.n_rows, rp.ctypes.data, order.ctypes.data)
    deg = np.diff(rp.astype(np.int64))
    starts = rp[:-1].astype(np.int64)[order]
    lens = deg[order]
    idx = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(int(lens.sum()))
    col_o = torch.from_numpy(np.ascontiguousarray(hg.col[idx])).cuda()
    to = bench.gather_ceiling(col_o, X, timer)
    print(json.dumps({"setting": "gather probe (degree order)", "ms": None if to is None else to * 1e3}), flush=True)


if __name__ == "__main__":
    main()
