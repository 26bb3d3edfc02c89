#!/usr/bin/env python3
"""Where does the error on long hub rows come from?  On the Products-shaped R-MAT graph's
longest rows, compare three values of each output against the float64 evaluation of the
reference's formulas (the same fp32 inputs):

  gpu -- libgala_hip.so (the 8-head REF statistics pair; gala_row_sum_f32)
  ref -- the oracle's restatement of the reference's pass sequence in fp32 (sequential
         row sums in CSR order, cuda.h:505-524), i.e. what the reference computes
and prints per output the worst |gpu - exact|, |ref - exact| and |gpu - ref| over the rows
(JSON lines).  python tools/gat_hub_err_probe.py [n_rows]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc  # noqa: E402
from gala import layout, ops  # noqa: E402


def rows_graph(g, rows):
    rp = g.rowptr.astype(np.int64)
    deg = rp[rows + 1] - rp[rows]
    sp = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(deg, out=sp[1:])
    col = np.concatenate([g.col[rp[r]:rp[r + 1]] for r in rows])
    return sp.astype(np.int32), np.ascontiguousarray(col, np.int32)


def exact_layer(r, cols, X, dY, aL, aR, H, D, slope=0.2):
    """float64 daL / Y of row r (the reference's formulas, no rounding)."""
    Xc = X[cols].astype(np.float64).reshape(len(cols), H, D)
    s = aL[r].astype(np.float64)[None, :] + aR[cols].astype(np.float64)
    t = np.where(s > 0, s, s * slope)
    p = np.minimum(np.exp(t), 1e12)
    q = 1.0 / (1e-12 + p.sum(0))
    al = p * q
    Y = np.einsum("eh,ehd->hd", al, Xc).reshape(-1)
    da = np.einsum("hd,ehd->eh", dY[r].astype(np.float64).reshape(H, D), Xc)
    sds = al * da
    acc = 1e-12 + sds.sum(0)
    ds = sds - al * acc
    dt = np.where(s > 0, ds, ds * slope)
    return Y, 1e-12 + dt.sum(0)


def main():
    n_long = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    orc.set_threads(min(16, len(os.sched_getaffinity(0))))
    H, D = 8, 32
    F = H * D
    g = layout.gen_graph("rmat", 2_449_029, 61_859_140, seed=42)
    deg = np.diff(g.rowptr.astype(np.int64))
    gen = torch.Generator(device="cuda").manual_seed(4321)
    X = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    dY = torch.rand((g.n_rows, F), device="cuda", generator=gen) * 2 - 1
    aL = torch.rand((g.n_rows, H), device="cuda", generator=gen) - 0.5
    wR = (torch.rand(F, device="cuda", generator=gen) - 0.5) * 0.2
    bR = (torch.rand(H, device="cuda", generator=gen) - 0.5) * 0.2
    dg = ops.DeviceGraph.from_host(g)
    Y, q, Ym, sma, aR = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
    dX, daL = ops.gat_bwd_stats(dg, aL, aR, dY, q, Y, Ym, sma, heads=H)
    torch.cuda.synchronize()
    if n_long > 0:
        rows = np.sort(np.argsort(deg, kind="stable")[-n_long:]).astype(np.int64)
    else:   # the test's sample: 2 000 leading rows + the 64 longest
        rows = np.unique(np.concatenate([np.arange(2000), np.argsort(deg, kind="stable")[-64:]])).astype(np.int64)
    rp, col = rows_graph(g, rows)
    Xh, dYh, aLh = X.cpu().numpy(), dY.cpu().numpy(), aL.cpu().numpy()
    ref = orc.GatRefLayer(rp, col, len(rows), Xh, dYh, aLh, wR.cpu().numpy(), bR.cpu().numpy(), H,
                          row_ids=rows).run()
    aRh = ref.aR   # fp32 source logits, as the reference computes them
    rt = torch.from_numpy(rows).cuda()
    gY, gdaL = Y[rt].cpu().numpy(), daL.view(-1, H)[rt].cpu().numpy()
    worst = {"Y": [0, 0, 0], "daL": [0, 0, 0]}
    # exact evaluation for the rows where the GPU and the reference differ most
    diff = np.abs(gdaL.astype(np.float64) - ref.daL).max(1) / (1e-4 + 1e-4 * np.abs(ref.daL).max(1))
    for i in np.argsort(diff)[-16:]:
        r = rows[i]
        cols = col[rp[i]:rp[i + 1]]
        eY, edaL = exact_layer(r, cols, Xh, dYh, aLh, aRh, H, D)
        for k, (gv, rv, ev) in {"Y": (gY[i], ref.Y[i], eY), "daL": (gdaL[i], ref.daL[i], edaL)}.items():
            w = worst[k]
            w[0] = max(w[0], float(np.max(np.abs(gv - ev))))
            w[1] = max(w[1], float(np.max(np.abs(rv - ev))))
            w[2] = max(w[2], float(np.max(np.abs(gv.astype(np.float64) - rv))))
        print(json.dumps({"row": int(r), "deg": int(deg[r]), "ratio_gpu_vs_ref": float(diff[i]),
                          "daL_gpu_err": float(np.max(np.abs(gdaL[i] - edaL))),
                          "daL_ref_err": float(np.max(np.abs(ref.daL[i] - edaL))),
                          "daL_max": float(np.max(np.abs(edaL)))}), flush=True)
    for k, w in worst.items():
        print(json.dumps({"output": k, "rows": len(rows), "gpu_vs_exact": w[0], "ref_vs_exact": w[1],
                          "gpu_vs_ref": w[2]}), flush=True)
    # K7 on signed unit terms: the same three-way comparison
    v = torch.rand(g.nnz * H, device="cuda", generator=gen) * 2 - 1
    got = ops.row_sum(dg, v, heads=H, eps=1e-12).view(-1, H)[rt].cpu().numpy()
    vh = v.view(-1, H).cpu().numpy()
    sub = orc.Graph(len(rows), g.n_cols, rp, col)
    rp64 = g.rowptr.astype(np.int64)
    sel = np.concatenate([np.arange(rp64[r], rp64[r + 1]) for r in rows])
    want = orc.row_sum(sub, vh[sel].ravel(), heads=H, eps=1e-12).reshape(-1, H)
    ex = np.stack([vh[rp64[r]:rp64[r + 1]].astype(np.float64).sum(0) + 1e-12 for r in rows])
    print(json.dumps({"output": "row_sum_signed", "gpu_vs_exact": float(np.max(np.abs(got - ex))),
                      "ref_vs_exact": float(np.max(np.abs(want - ex))),
                      "gpu_vs_ref": float(np.max(np.abs(got.astype(np.float64) - want)))}), flush=True)


if __name__ == "__main__":
    main()
