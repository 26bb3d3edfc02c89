#!/usr/bin/env python3
"""Where the vertex-cut GAT training pair spends its time beyond the one-GPU pair, at one
rank without collectives (config 3's 8-head layer, Products shape): the pair itself, the
one-GPU statistics pair, and the owner-side torch passes alone (q, Y = q U, Ym = q Um,
sma, dX = q P on the received [n, 2F] / [n, F] rows).  HIP events, median of reps.  One
JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gala-gnn-acceleration-language_amd"))
from gala import layout, ops, vertex_cut as vc  # noqa: E402
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
    reps = int(os.environ.get("GALA_REPS", "6"))
    hg = layout.gen_graph("uniform", int(2_449_029 * scale), int(61_859_140 * scale), seed=42)
    N, H, F = hg.n_rows, 8, 256
    be = HipBackend("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
    dY = torch.rand((N, F), device="cuda", generator=g) * 2 - 1
    aL = torch.rand((N, H), device="cuda", generator=g) - 0.5
    wR = (torch.rand(F, device="cuda", generator=g) - 0.5) * 0.2
    bR = torch.zeros(H, device="cuda")
    res = {}
    part = vc.vertex_cut_partition(hg, 0, 1, 4)
    lay = vc.VertexCutGat(part, F, H, be, None)

    def vpair():
        lay.forward_train(aL, None, X, wR, bR)
        lay.backward(dY, linear=False)
    res["vcut_pair_ms"] = med(vpair, reps)
    dg = ops.DeviceGraph.from_host(hg)

    def one():
        Y, q, Ym, sma, aR = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
        ops.gat_bwd_stats(dg, aL, aR, dY, q, Y, Ym, sma, heads=H)
    res["one_gpu_pair_ms"] = med(one, reps)
    UU = torch.rand((N, 2 * F), device="cuda", generator=g)
    So = torch.rand((N, H), device="cuda", generator=g) + 1
    Mo = torch.rand((N, H), device="cuda", generator=g)
    q = 1.0 / (So + 1e-12)
    res["owner_q_ms"] = med(lambda: 1.0 / (So + 1e-12), reps)
    res["owner_Y_ms"] = med(lambda: lay._owner_scale(q, UU[:, :F]), reps)
    res["owner_Ym_ms"] = med(lambda: lay._owner_scale(q, UU[:, F:]), reps)
    res["owner_sma_ms"] = med(lambda: Mo * q, reps)
    P = torch.rand((N, F), device="cuda", generator=g)
    res["owner_dX_ms"] = med(lambda: lay._owner_scale(q, P), reps)
    res["copy_UU_ms"] = med(lambda: UU.clone(), reps)
    print(json.dumps({"probe": "vcut_gat_owner", "N": N, "E": hg.nnz, "heads": H, "F": F, **res}), flush=True)


if __name__ == "__main__":
    main()
