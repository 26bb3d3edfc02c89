#!/usr/bin/env python3
# Needs commit f2516f9's tree (the GALA_HUB_TRACE build of spmm.hip and the ABI 6 plan fields, since reverted).
"""Timeline of one REF-order R-MAT SpMM (F = 32, Products shape) from a trace build of
libgala_hip.so (-DGALA_HUB_TRACE: wall-clock stamps written by the kernels themselves):
the row kernel's first start / last end, the hub kernel's, the 8 longest hub rows' workgroups
(start, end) and the longest chain's progress per eighth of its tiles, in microseconds from the
first start.  Measurement only.
    python tools/hub_trace.py LIB [calls]
Each call runs twice: with the plan's side stream as built (a normal-priority stream), and with
a high-priority side stream in its place ("prio").
"""
import ctypes
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
    lib = load(sys.argv[1])
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    _abi._lib = lib
    hg = bench.products_graph("rmat", 1.0)
    dg = ops.DeviceGraph.from_host(hg)
    deg = (hg.rowptr[1:] - hg.rowptr[:-1])
    top = sorted(deg.tolist(), reverse=True)[:8]
    X = torch.rand((hg.n_rows, 32), device="cuda") * 2 - 1
    Y = torch.empty_like(X)
    buf = (ctypes.c_ulonglong * 64)()
    fn = lib.gala_dbg_hub_trace
    plan = dg._split["plan"]
    normal = plan.aux_stream
    hi = torch.cuda.Stream(priority=-1)
    for c, variant in ((c, v) for c in range(calls + 1) for v in ("normal", "prio")):
        plan.aux_stream = normal if variant == "normal" else hi.cuda_stream
        fn(buf, 1)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        ops.spmm(dg, X, out=Y)
        ev1.record()
        torch.cuda.synchronize()
        fn(buf, 0)
        v = list(buf)
        t0 = min(v[16], v[18])
        us = lambda t: round((t - t0) / 100.0, 1) if t else None  # 100 MHz
        rec = {"call": c, "variant": variant, "event_ms": round(ev0.elapsed_time(ev1), 4),
               "row_kernel_us": [us(v[18]), us(v[19])], "hub_kernel_us": [us(v[16]), us(v[17])],
               "longest_rows_deg": top,
               "longest_rows_wg_us": [[us(v[2 * i]), us(v[2 * i + 1])] for i in range(8)],
               "chain0_tiles": v[24], "chain0_eighths_us": [us(v[24 + k]) for k in range(1, 9)]}
        if c:
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
