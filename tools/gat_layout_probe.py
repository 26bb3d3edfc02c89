#!/usr/bin/env python3
"""Experiment: does the 8-head row-statistics pair (config 3's GAT layer on the Products
shape) run faster when the forward writes Y and Ym into ONE [N, 2F] buffer (each row's
2 KB of outputs contiguous; the C ABI's ldy / ldym strides) instead of two [N, F] arrays?
The backward then reads both rows of a destination contiguously too.  HIP events, median of
reps, the two layouts alternated; results bit-identical.  One JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gala-gnn-acceleration-language_amd"))
from gala import _abi, layout, ops  # noqa: E402
from gala.ops import _dp, _stream  # noqa: E402


def ev_time(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    return a, b


def main():
    scale = float(os.environ.get("GALA_SCALE", "1.0"))
    reps = int(os.environ.get("GALA_REPS", "10"))
    hg = layout.gen_graph("uniform", int(2_449_029 * scale), int(61_859_140 * scale), seed=42)
    dg = ops.DeviceGraph.from_host(hg)
    N, H, F = hg.n_rows, 8, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
    dY = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
    aL = torch.rand((N, H), device="cuda", generator=g) - 0.5
    wR = (torch.rand(F, device="cuda", generator=g) - 0.5) * 0.2
    bR = torch.zeros(H, device="cuda")
    q = torch.empty(N * H, device="cuda")
    sma = torch.empty(N * H, device="cuda")
    aR = torch.empty(N * H, device="cuda")
    sep = (torch.empty((N, F), device="cuda"), torch.empty((N, F), device="cuda"))
    buf = torch.empty((N, 2 * F), device="cuda")
    inter = (buf[:, :F], buf[:, F:])
    dX = torch.empty((N, F), device="cuda")
    d_aL = torch.empty(N * H, device="cuda")

    def fwd(YYm):
        Y, Ym = YYm
        _abi.call("gala_gat_fwd_stats_f32", dg.csr(2 * F + 3 * H), _dp(aL), None, _dp(wR), _dp(bR), _dp(X),
                  X.stride(0), F, H, 0.2, _dp(Y), Y.stride(0), _dp(q), _dp(Ym), Ym.stride(0), _dp(sma), _dp(aR),
                  None, _stream())

    def bwd(YYm):
        Y, Ym = YYm
        _abi.call("gala_gat_bwd_stats_f32", dg.csr(F), _dp(aL), _dp(aR), None, _dp(dY), dY.stride(0), F, H, 0.2,
                  _dp(q), _dp(Y), Y.stride(0), _dp(Ym), Ym.stride(0), _dp(sma), _dp(dX), dX.stride(0), _dp(d_aL),
                  _stream())

    res = {}
    for name, lay in (("separate", sep), ("interleaved", inter)):
        fwd(lay)
        bwd(lay)
    torch.cuda.synchronize()
    outs = {}
    for name, lay in (("separate", sep), ("interleaved", inter)):
        fwd(lay)
        bwd(lay)
        torch.cuda.synchronize()
        outs[name] = (lay[0].clone(), lay[1].clone(), dX.clone(), d_aL.clone())
    same = all(torch.equal(a, b) for a, b in zip(outs["separate"], outs["interleaved"]))
    del outs
    ts = {k: {"fwd": [], "bwd": []} for k in ("separate", "interleaved")}
    for r in range(reps):
        order = (("separate", sep), ("interleaved", inter)) if r % 2 == 0 else (("interleaved", inter), ("separate", sep))
        for name, lay in order:
            ts[name]["fwd"].append(ev_time(lambda: fwd(lay)))
            ts[name]["bwd"].append(ev_time(lambda: bwd(lay)))
    torch.cuda.synchronize()
    for k, v in ts.items():
        res[k] = {p: float(np.median([a.elapsed_time(b) for a, b in v[p]])) for p in v}
    print(json.dumps({"probe": "gat_layout", "N": N, "E": hg.nnz, "heads": H, "F": F, "bit_identical": same,
                      **res}), flush=True)


if __name__ == "__main__":
    main()
