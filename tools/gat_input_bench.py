"""Config 3's layer 1 at the Products shape, timed from the 100-d input (Linear included):
the mirror's gat_input_layer_apply (input space, gala_gat_in_*) against the three ops it
replaces (ffn_apply -> head_attn_apply -> gat_aggregate_ffn_apply: the Linear output
gathered, the row-statistics GAT pair), forward and backward with autograd, alternated in one
process.  Prints one JSON line per variant.

    python tools/gat_input_bench.py [--scale 1.0] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import bench
    import gala
    E = gala.torch_ext()
    g = bench.products_graph("uniform", a.scale)
    E.slots_clear()
    off, cols = torch.from_numpy(g.rowptr).cuda(), torch.from_numpy(g.col).cuda()
    vals = torch.ones(g.nnz, device="cuda")
    E.slots_push(off, cols, vals, None, 1, False)
    E.slots_push(off, cols, vals, None, 1, False)
    fin, H, D = 100, 8, 32
    F = H * D
    gen = torch.Generator(device="cuda").manual_seed(5)
    x = torch.rand(g.n_rows, fin, device="cuda", generator=gen) * 2 - 1
    dY = torch.rand(g.n_rows, F, device="cuda", generator=gen) * 2 - 1
    W = ((torch.rand(F, fin, device="cuda", generator=gen) * 2 - 1) / 10).requires_grad_()
    b = ((torch.rand(F, device="cuda", generator=gen) - 0.5) * 0.2).requires_grad_()
    wL, wR = (((torch.rand(1, F, device="cuda", generator=gen) - 0.5) * 0.6).requires_grad_() for _ in range(2))
    bL, bR = (((torch.rand(H, device="cuda", generator=gen) - 0.5) * 0.2).requires_grad_() for _ in range(2))
    params = (W, b, wL, bL, wR, bR)

    def chain():
        v1 = E.ffn_apply(x, W, b)
        return E.gat_aggregate_ffn_apply(E.head_attn_apply(v1, wL, bL), v1, wR, bR, 0, 0.2, 0)

    def inspace():
        return E.gat_input_layer_apply(x, W, b, wL, bL, wR, bR, 0, 0.2, 0)

    assert E.gat_input_layer_eligible(x, W, 0, H, 0)
    variants = {"input_space": inspace, "chain": chain}
    res = {k: {"fwd": [], "bwd": []} for k in variants}
    outs = {}
    for rep in range(a.reps + 1):
        for name, fn in variants.items():
            for p in params:
                p.grad = None
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            torch.cuda.synchronize()
            e[0].record()
            Y = fn()
            e[1].record()
            Y.backward(dY)
            e[2].record()
            torch.cuda.synchronize()
            if rep > 0:
                res[name]["fwd"].append(e[0].elapsed_time(e[1]))
                res[name]["bwd"].append(e[1].elapsed_time(e[2]))
            else:
                outs[name] = [Y.detach()] + [p.grad.clone() for p in params]
            del Y
    # agreement of the two spellings (the tests' tolerance)
    err = {}
    for i, nm in enumerate(("Y", "W", "b", "wL", "bL", "wR", "bR")):
        u, v = outs["input_space"][i], outs["chain"][i]
        err[nm] = float((u - v).abs().max() / max(v.abs().max().item(), 1e-30))
    E_ = g.nnz
    for name in variants:
        f, bw = float(np.median(res[name]["fwd"])), float(np.median(res[name]["bwd"]))
        print(json.dumps({"variant": name, "n": g.n_rows, "nnz": E_, "fin": fin, "heads": H, "D": D,
                          "fwd_ms": round(f, 3), "bwd_ms": round(bw, 3), "layer_ms": round(f + bw, 3),
                          "edges_per_s": E_ / ((f + bw) / 1e3), "fwd_all": res[name]["fwd"],
                          "bwd_all": res[name]["bwd"]}), flush=True)
    print(json.dumps({"max_rel_diff_vs_chain": err}), flush=True)


if __name__ == "__main__":
    main()
