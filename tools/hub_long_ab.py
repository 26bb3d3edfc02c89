#!/usr/bin/env python3
# Needs commit f2516f9's tree (the GALA_HUB_TRACE build of spmm.hip and the ABI 6 plan fields, since reverted).
"""In-process A/B of the REF-order R-MAT SpMM (Products shape, F = 32) with and without the
ABI 6 long-chain launch: "long" -- the plan as gala.ops builds it (the longest chains on CU 0 of
every XCD, the other hub rows and the row kernel on the other CUs) -- against "one" -- one hub
launch on an unmasked side stream beside the row kernel on the caller's stream (ABI 5's
schedule).  Alternated rounds of 10 calls, medians, bit-identity.  With a trace build
(-DGALA_HUB_TRACE, tools/hub_trace.py) given as LIB, also each variant's timeline.
Measurement only.
    python tools/hub_long_ab.py [rounds] [LIB]
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
from gala import _abi, ops  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    from ab_gat import load
    libs = {"tree": _abi.lib()}
    for f in sys.argv[2:]:
        libs[os.path.basename(f)[len("libgala_hip_"):-3]] = load(f)
    hg = bench.products_graph("rmat", 1.0)
    dg = ops.DeviceGraph.from_host(hg)
    plan = dg._split["plan"]
    long_cfg = (plan.n_long, plan.aux_stream, plan.long_stream, plan.row_stream)
    pool = torch.cuda.Stream()
    hi = torch.cuda.Stream(priority=-1)
    cfgs = {"long": long_cfg, "one": (0, pool.cuda_stream, None, None), "one_prio": (0, hi.cuda_stream, None, None)}

    def use(cfg):
        plan.n_long, plan.aux_stream, plan.long_stream, plan.row_stream = cfg
    X = torch.rand((hg.n_rows, 32), device="cuda") * 2 - 1
    Y = torch.empty_like(X)
    timer = bench.Timer(True)
    variants = [(lib, c) for lib in libs for c in cfgs]
    outs, samples = {}, {f"{lib}/{c}": [] for lib, c in variants}
    for r in range(rounds + 1):
        for lib, c in variants:
            _abi._lib = libs[lib]
            trace = getattr(libs[lib], "gala_dbg_hub_trace", None)
            name, cfg = f"{lib}/{c}", cfgs[c]
            use(cfg)
            ops.spmm(dg, X, out=Y)
            torch.cuda.synchronize()
            outs.setdefault(name, Y.clone())
            if trace is not None and r:
                buf = (ctypes.c_ulonglong * 64)()
                trace(buf, 1)
                torch.cuda.synchronize()
                ops.spmm(dg, X, out=Y)
                torch.cuda.synchronize()
                trace(buf, 0)
                v = list(buf)
                t0 = min(v[16], v[18])
                us = lambda t: round((t - t0) / 100.0, 1) if t else None  # noqa: E731
                print(json.dumps({"round": r, "variant": name, "row_kernel_us": [us(v[18]), us(v[19])],
                                  "hub_wg0_us": [us(v[0]), us(v[1])], "hub_last_end_us": us(v[17]),
                                  "chain0_eighths_us": [us(v[24 + k]) for k in range(1, 9)],
                                  # the chain wave's shader clock per eighth (s_memtime cycles over
                                  # the 100 MHz wall clock), MHz
                                  "chain0_clock_mhz": [round((v[40 + k] - v[39 + k]) /
                                                             max((v[24 + k] - (v[23 + k] if k > 1 else v[56])) / 100.0, 1e-9), 1)
                                                       for k in range(1, 9)]}), flush=True)
            t = timer(lambda: ops.spmm(dg, X, out=Y), 10)
            if r:
                samples[name].append(round(t * 1e3, 4))
    # the longest row alone (every other row a self loop): its chain's clock without load
    for lib in libs:
        trace = getattr(libs[lib], "gala_dbg_hub_trace", None)
        if trace is None:
            continue
        import numpy as np
        from gala import layout
        n = hg.n_rows
        deg = np.diff(hg.rowptr)
        r0 = int(np.argmax(deg))
        cnt = np.ones(n, np.int64)
        cnt[r0] = deg[r0]
        rp = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
        col = np.arange(n, dtype=np.int32).repeat(cnt)
        col[rp[r0]:rp[r0 + 1]] = hg.col[hg.rowptr[r0]:hg.rowptr[r0 + 1]]
        ag = ops.DeviceGraph.from_host(layout.HostGraph(n, n, rp, col))
        _abi._lib = libs[lib]
        buf = (ctypes.c_ulonglong * 64)()
        for _ in range(3):
            trace(buf, 1)
            torch.cuda.synchronize()
            ops.spmm(ag, X, out=Y)
            torch.cuda.synchronize()
            trace(buf, 0)
        v = list(buf)
        print(json.dumps({"variant": f"{lib}/alone", "hub_wg0_us": [0.0, round((v[1] - v[0]) / 100.0, 1)],
                          "chain0_clock_mhz": [round((v[40 + k] - v[39 + k]) /
                                                     max((v[24 + k] - (v[23 + k] if k > 1 else v[56])) / 100.0, 1e-9), 1)
                                               for k in range(1, 9)]}), flush=True)
    use(long_cfg)
    _abi._lib = libs["tree"]
    ref = outs["tree/one"]
    print(json.dumps({"graph": "rmat", "n_long": long_cfg[0],
                      "medians_ms": {k: sorted(v)[len(v) // 2] for k, v in samples.items()}, "samples": samples,
                      "bit_identical": {k: bool(torch.equal(v, ref)) for k, v in outs.items()}}), flush=True)


if __name__ == "__main__":
    main()
