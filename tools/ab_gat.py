#!/usr/bin/env python3
"""In-process A/B of builds of libgala_hip.so on the 8-head GAT statistics pair (bench.py's
"gat" leg: F = 256, the Products-shaped uniform graph).  Between processes and boxes the pair
and the gather probe both move by up to 10 % (the tables' physical placement), more than most
kernel changes, so the builds run alternately in one process on the same inputs:
tools/ab/libgala_hip_<label>.so (builds of other commits: git worktree + make) and "tree", this
tree's gala/libgala_hip.so.  Prints per round fwd / bwd ms of each, the medians, and whether
each build's outputs are bit-identical to the tree's.  Measurement only.
    python tools/ab_gat.py [rounds] [h8|h1f32]
h1f32: one head at F = 32 with the source logits given (aR, not recomputed: the
reference-emitted GAT's first layer), the same statistics pair.
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gala import _abi, ops  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    for name, (res, args) in _abi.SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    assert L.gala_abi_version() == _abi.ABI_VERSION, path
    return L


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    kind = sys.argv[2] if len(sys.argv) > 2 else "h8"
    import glob
    libs = {os.path.basename(f)[len("libgala_hip_"):-3]: load(f)
            for f in sorted(glob.glob(os.path.join(ROOT, "tools", "ab", "libgala_hip_*.so")))}
    libs["tree"] = _abi.lib()
    fns = {k: ctypes.cast(L.gala_gat_fwd_stats_f32, ctypes.c_void_p).value for k, L in libs.items()}
    assert len(set(fns.values())) == len(fns), fns   # every build loaded as its own copy
    print(json.dumps({"builds": list(libs), "kind": kind}), flush=True)
    H, F = (8, 256) if kind == "h8" else (1, 32)
    hg = bench.products_graph("uniform", 1.0)
    dg = ops.DeviceGraph.from_host(hg)
    N = hg.n_rows
    gen = torch.Generator(device="cuda").manual_seed(4321)
    X = torch.rand((N, F), device="cuda", generator=gen) * 2 - 1
    dY = torch.rand((N, F), device="cuda", generator=gen) * 2 - 1
    aL = torch.rand((N, H), device="cuda", generator=gen) - 0.5
    wR = (torch.rand(F, device="cuda", generator=gen) - 0.5) * 0.2
    bR = torch.zeros(H, device="cuda")
    aR = torch.rand((N, H), device="cuda", generator=gen) - 0.5
    timer = bench.Timer(True)
    outs, samples = {}, {k: [] for k in libs}
    for r in range(rounds + 1):          # round 0: warm-up, not recorded
        for k in libs:
            _abi._lib = libs[k]
            st = {}

            def fwd():
                if kind == "h8":
                    st["f"] = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
                else:
                    st["f"] = ops.gat_fwd_stats(dg, aL, X, aR=aR, heads=H) + (aR,)

            def bwd():
                Y, q, Ym, sma, aRo = st["f"]
                st["b"] = ops.gat_bwd_stats(dg, aL, aRo, dY, q, Y, Ym, sma, heads=H)
            fwd()
            bwd()
            torch.cuda.synchronize()
            if k not in outs:
                outs[k] = [t.clone() for t in st["f"]] + [t.clone() for t in st["b"]]
            tf, tb = timer(fwd, 10), timer(bwd, 10)
            if r > 0:
                samples[k].append((tf * 1e3, tb * 1e3))
                print(json.dumps({"round": r, "lib": k, "fwd_ms": round(tf * 1e3, 3), "bwd_ms": round(tb * 1e3, 3)}),
                      flush=True)
            del st
    _abi._lib = libs["tree"]
    same = {k: all(torch.equal(a, b) for a, b in zip(outs[k], outs["tree"])) for k in libs}
    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
    res = {k: {"fwd_ms_median": round(med([a for a, _ in v]), 3), "bwd_ms_median": round(med([b for _, b in v]), 3)}
           for k, v in samples.items()}
    t_ceil = bench.gather_ceiling(dg.col, X, timer)
    print(json.dumps({"summary": res, "bit_identical_to_tree": same,
                      "gather_ceiling_ms": round(t_ceil * 1e3, 3) if t_ceil else None}), flush=True)


if __name__ == "__main__":
    main()
