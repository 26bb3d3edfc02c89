#!/usr/bin/env python3
"""The compute one rank of a P-rank row partition spends in the GAT training pair, without
the exchange (comm None; config 3's 8-head layer on the Products shape): HaloGat (the one-GPU
statistics kernels over the gathered table) against HaloGatOverlap (own-column partial
statistics, then the halo columns continued from them, gala_gat_fwd_continue_f32) -- the
price of making the exchange overlappable.  Also the own-column share of each pass, the
part that can hide the exchange.  HIP events, median of reps.  One JSON line per P."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gala-gnn-acceleration-language_amd"))
from gala import dist as gdist, layout  # noqa: E402
from gala.backend import HipBackend  # noqa: E402


def med(fn, reps):
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
    reps = int(os.environ.get("GALA_REPS", "5"))
    worlds = [int(w) for w in os.environ.get("GALA_WORLDS", "2,8").split(",")]
    hg = layout.gen_graph("uniform", int(2_449_029 * scale), int(61_859_140 * scale), seed=42)
    H, F = 8, 256
    be = HipBackend("cuda")
    for P in worlds:
        pt = gdist.partition_graph(hg, 0, P)
        n = pt.n
        g = torch.Generator(device="cuda").manual_seed(0)
        aL = torch.rand((n, H), device="cuda", generator=g) - 0.5
        wR = (torch.rand(F, device="cuda", generator=g) - 0.5) * 0.2
        bR = torch.zeros(H, device="cuda")
        res = {}
        for name, cls in (("halo", gdist.HaloGat), ("halo_overlap", gdist.HaloGatOverlap)):
            lay = cls(pt, F, H, be, None)
            lay.Xs.uniform_(-1, 1, generator=g)
            lay.dYs.uniform_(-1, 1, generator=g)
            X, dY = lay.own_rows("X"), lay.own_rows("dY")

            def pair():
                lay.forward_train(aL, None, X, wR, bR)
                lay.backward(dY, linear=False)
            res[name + "_pair_ms"] = med(pair, reps)
            if name == "halo_overlap":
                U, Um, S, M = be.empty(n, F), be.empty(n, F), be.empty(n, H), be.empty(n, H)
                res["own_fwd_partial_ms"] = med(lambda: be.gat_partial_stats(
                    lay.groups[0], aL, None, lay.Xs, H, 0.2, U, S, Um, M, wR=wR, bR=bR, self_col=lay.self_col,
                    aR_out=lay.As), reps)
                res["halo_fwd_continue_ms"] = med(lambda: be.gat_continue(
                    lay.groups[1], aL, None, lay.Xs, H, 0.2, U, S, Um, M, wR=wR, bR=bR), reps)
                Pb = be.empty(n, F)
                res["own_bwd_partial_ms"] = med(lambda: be.gat_partial(
                    lay.groups[0], aL, lay.As, lay.dYs, H, 0.2, Pb, lay.Ssc), reps)
            del lay
            torch.cuda.empty_cache()
        print(json.dumps({"probe": "halo_gat_overlap", "world": P, "rank": 0, "n_rows": n, "n_cols": pt.n_cols,
                          "edges": pt.graph.nnz, "own_edges": pt.groups[0].nnz, "halo_mode": pt.halo_mode,
                          "heads": H, "F": F, **res}), flush=True)


if __name__ == "__main__":
    main()
