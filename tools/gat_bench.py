#!/usr/bin/env python3
"""GAT op timings on the ogbn-products shape (uniform graph, HIP events, median of reps):
the fused forward with materialised alpha vs the factored (p, q) output, the weighted SpMM
of the same shape (the forward's floor: same gathers, a stored weight instead of a
softmax), the dX SpMM on (p, q) and the fused backward -- at 8 heads (F = 256) and one
head (F = 32, with and without the attention recompute), and the row-statistics forward /
backward pair.  One JSON line per op."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gala-gnn-acceleration-language_amd"))
from gala import layout, ops  # noqa: E402


def timeit(fn, reps=10):
    fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ts]))


def main():
    scale = float(os.environ.get("GALA_SCALE", "1.0"))
    n = int(2_449_029 * scale)
    m = int(61_859_140 * scale)
    hg = layout.gen_graph("uniform", n, m, seed=42)
    dg = ops.DeviceGraph.from_host(hg)
    N, E = hg.n_rows, hg.nnz
    g = torch.Generator(device="cuda").manual_seed(0)
    out = []
    for H, F in ((8, 256), (1, 32)):
        X = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
        dY = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
        aL = torch.rand((N, H), device="cuda", generator=g) - 0.5
        aR = torch.rand((N, H), device="cuda", generator=g) - 0.5
        wR = (torch.rand(F, device="cuda", generator=g) - 0.5) * 0.2
        bR = torch.zeros(H, device="cuda")
        Y, al = ops.gat_fwd(dg, aL, aR, X, heads=H, want_alpha=True)
        _, p, q = ops.gat_fwd_ex(dg, aL, X, aR=aR, heads=H, factored=True)
        rec = {
            "gat_fwd_alpha": timeit(lambda: ops.gat_fwd(dg, aL, aR, X, heads=H, want_alpha=True)),
            "gat_fwd_factored": timeit(lambda: ops.gat_fwd_ex(dg, aL, X, aR=aR, heads=H, factored=True)),
            "gat_fwd_no_alpha": timeit(lambda: ops.gat_fwd(dg, aL, aR, X, heads=H)),
            "gat_fwd_recompute_factored": timeit(lambda: ops.gat_fwd_ex(dg, aL, X, wR=wR, bR=bR, heads=H,
                                                                        factored=True)),
            "spmm_weighted": timeit(lambda: ops.spmm(dg.with_values(al, val_heads=H), X)),
            "spmm_factored": timeit(lambda: ops.spmm(dg.with_values(p, val_heads=H, row_scale=q), X)),
            "gat_bwd_alpha": timeit(lambda: ops.gat_bwd(dg, aL, aR, X, dY, al, heads=H)),
            "gat_bwd_factored": timeit(lambda: ops.gat_bwd_ex(dg, aL, X, dY, p, q=q, aR=aR, heads=H)),
            "gat_fwd_q_only": timeit(lambda: ops.gat_fwd_ex(dg, aL, X, aR=aR, heads=H, factored="q")),
            "gat_fwd_recompute_q_only": timeit(lambda: ops.gat_fwd_ex(dg, aL, X, wR=wR, bR=bR, heads=H,
                                                                      factored="q")),
            "gat_bwd_fused": timeit(lambda: ops.gat_bwd_fused(dg, aL, X, dY, q, aR=aR, heads=H)),
            "gat_bwd_fused_recompute": timeit(lambda: ops.gat_bwd_fused(dg, aL, X, dY, q, wR=wR, bR=bR, heads=H)),
        }
        # the row-statistics pair (gala_gat_{fwd,bwd}_stats_f32)
        Ys, qs, Ym, sma = ops.gat_fwd_stats(dg, aL, X, aR=aR, heads=H)
        _, _, _, _, aRo = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
        rec["gat_fwd_stats"] = timeit(lambda: ops.gat_fwd_stats(dg, aL, X, aR=aR, heads=H))
        rec["gat_fwd_stats_recompute"] = timeit(lambda: ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H,
                                                                         want_aR=True))
        rec["gat_bwd_stats"] = timeit(lambda: ops.gat_bwd_stats(dg, aL, aR, dY, qs, Ys, Ym, sma, heads=H))
        pe = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_p=True)[-1]
        rec["gat_fwd_stats_recompute_p"] = timeit(lambda: ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H,
                                                                           want_aR=True, want_p=True))
        rec["gat_bwd_stats_p"] = timeit(lambda: ops.gat_bwd_stats(dg, aL, None, dY, qs, Ys, Ym, sma, heads=H, p=pe))
        del Ys, qs, Ym, sma, aRo, pe
        for k, v in rec.items():
            line = {"op": k, "heads": H, "F": F, "ms": v, "N": N, "E": E}
            out.append(line)
            print(json.dumps(line), flush=True)
        del X, dY, al, p, q
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
