#!/usr/bin/env python3
"""In-process A/B of builds of libgala_hip.so on config 3's input-space GAT kernels
(gala_gat_in_fwd_f32 / gala_gat_in_bwd_f32, Products shape, 8 heads x 32 from 100 inputs, the
bench's inputs): tools/ab/libgala_hip_<label>.so and "tree", alternated on the same extended
rows; medians of 5 calls per round and bit-identity of Y / Ym / q / sma and d_aL / M to the
tree.  Measurement only.
    python tools/ab_gat_in.py [rounds]
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
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    ref_lib = sys.argv[3] if len(sys.argv) > 3 else "tree"   # the build the others are compared with
    libs = {os.path.basename(f)[len("libgala_hip_"):-3]: load(f)
            for f in sorted(glob.glob(os.path.join(ROOT, "tools", "ab", "libgala_hip_*.so")))}
    libs["tree"] = _abi.lib()
    dev = torch.device("cuda")
    hg = bench.products_graph("uniform", scale)
    dg = ops.DeviceGraph.from_host(hg)
    H, D, FIN = bench.GAT_HEADS, bench.GAT_HEAD_F, bench.GAT_IN_F
    F, N = H * D, hg.n_rows
    gen = torch.Generator(device=dev).manual_seed(4321)
    Xin = torch.rand((N, FIN), device=dev, generator=gen) * 2 - 1
    dY = torch.rand((N, F), device=dev, generator=gen) * 2 - 1
    W = (torch.rand((F, FIN), device=dev, generator=gen) * 2 - 1) / 10
    b = (torch.rand(F, device=dev, generator=gen) - 0.5) * 0.2
    wL, wR = ((torch.rand(F, device=dev, generator=gen) - 0.5) * 0.6 for _ in range(2))
    bL, bR = ((torch.rand(H, device=dev, generator=gen) - 0.5) * 0.2 for _ in range(2))
    order = torch.from_numpy(ops.degree_order(hg.rowptr)).to(dev)
    f0 = ops.gat_input_layer(dg, Xin, W, b, wL, bL, wR, bR, H, order=order, relu=True)
    xext = f0["xext"]
    res = {}

    def k_fwd():
        res["f"] = ops.gat_in_fwd(dg, xext, W, b, H, FIN, order=order, relu=True)

    def k_bwd():
        res["b"] = ops.gat_in_bwd(dg, xext, dY, f0["Y"], f0["Ym"], f0["sma"], H, FIN, order=order, relu=True)
    timer = bench.Timer(True)
    samples = {k: {"fwd": [], "bwd": []} for k in libs}
    outs = {}
    for r in range(rounds + 1):
        for k in libs:
            _abi._lib = libs[k]
            k_fwd()
            k_bwd()
            torch.cuda.synchronize()
            if k not in outs:
                f, bw = res["f"], res["b"]
                outs[k] = [t.clone() for t in (f if isinstance(f, (tuple, list)) else [f])] + \
                          [t.clone() for t in bw]
            tf, tb = timer(k_fwd, 5), timer(k_bwd, 5)
            if r:
                samples[k]["fwd"].append(round(tf * 1e3, 4))
                samples[k]["bwd"].append(round(tb * 1e3, 4))
    _abi._lib = libs["tree"]
    med = {k: {p: sorted(v)[len(v) // 2] for p, v in d.items()} for k, d in samples.items()}
    same = {k: all(torch.equal(a, b) for a, b in zip(outs[k], outs[ref_lib])) for k in libs}
    diff = {k: max(float((a - b).abs().max()) for a, b in zip(outs[k], outs[ref_lib])) for k in libs}
    print(json.dumps({"medians_ms": med, "samples": samples, "reference_build": ref_lib, "bit_identical": same, "max_abs_diff": diff}), flush=True)


if __name__ == "__main__":
    main()
