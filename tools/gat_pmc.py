#!/usr/bin/env python3
"""Where the 8-head GAT statistics pair's HBM bytes go.

Run under two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; tools/gpu_job.sh
pmccmd=gat,python3,<repo>/tools/gat_pmc.py), this program launches, once each and in this
order, on the Products-shaped uniform graph at F = 256 (bench.py's "gat" leg):

  1. the gather probe over X        (k_gather: X[col[e]] for every edge, nothing else)
  2. the forward                    (k_gat_fwd, gala_gat_fwd_stats_f32: Y, Ym, q, sma, aR_out)
  3. the backward                   (k_gat_bwd_fused, ST: dY[col] + aR[col] per edge)
  4. the forward writing p as well  (the same kernel, alpha_out = p)
  5. the backward from p            (the same kernel, alpha from p * q: no aR[col])

`python3 tools/gat_pmc.py --split FETCH_DIR WRITE_DIR OUT.json` then attributes the bytes
(FETCH_SIZE x 2 per MI355X_MICROARCH.md's gfx950 correction, as tools/pmc_traffic.py):
forward reads beyond the probe's gather, forward writes (Y, Ym and the row statistics), the
backward's aR[col] lines (3 - 5 fetch, plus the p bytes 5 reads) and its other reads.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORDER = ["probe_gather", "fwd", "bwd", "fwd_p", "bwd_p"]


def run():
    import torch
    sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
    sys.path.insert(0, ROOT)
    import bench
    from gala import ops
    H, F = 8, 256
    hg = bench.products_graph("uniform", 1.0)
    dg = ops.DeviceGraph.from_host(hg)
    N = hg.n_rows
    gen = torch.Generator(device="cuda").manual_seed(4321)
    X = torch.rand((N, F), device="cuda", generator=gen) * 2 - 1
    dY = torch.rand((N, F), device="cuda", generator=gen) * 2 - 1
    aL = torch.rand((N, H), device="cuda", generator=gen) - 0.5
    wR = (torch.rand(F, device="cuda", generator=gen) - 0.5) * 0.2
    bR = torch.zeros(H, device="cuda")
    torch.cuda.synchronize()
    assert bench.gather_ceiling(dg.col, X, lambda fn, reps: (fn(), torch.cuda.synchronize(), 1.0)[2]) is not None
    f = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)
    ops.gat_bwd_stats(dg, aL, f[4], dY, f[1], f[0], f[2], f[3], heads=H)
    torch.cuda.synchronize()
    del f
    f = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True, want_p=True)
    ops.gat_bwd_stats(dg, aL, f[4], dY, f[1], f[0], f[2], f[3], heads=H, p=f[5])
    torch.cuda.synchronize()
    print(json.dumps({"rows": N, "edges": int(hg.nnz), "F": F, "heads": H}), flush=True)


def read(d, name):
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if r.get("Counter_Name") != name:
                continue
            k = r["Kernel_Name"]
            if "k_gather" in k or "k_gat_fwd<" in k or "k_gat_bwd_fused<" in k:
                rows.append((int(r.get("Dispatch_Id", 0)), k, float(r["Counter_Value"])))
    rows.sort()
    probe = [r for r in rows if "k_gather" in r[1]]
    return probe[-1:] + [r for r in rows if "k_gather" not in r[1]]   # the timed probe launch


def split(fdir, wdir, out):
    fetch, write = read(fdir, "FETCH_SIZE"), read(wdir, "WRITE_SIZE")
    assert len(fetch) == len(ORDER) and len(write) == len(ORDER), (fetch, write)
    GB = 1e9
    fb = {n: 2 * v * 1024 / GB for n, (_, _, v) in zip(ORDER, fetch)}
    wb = {n: v * 1024 / GB for n, (_, _, v) in zip(ORDER, write)}
    N, E, F, H = 2_449_029, 126_167_309, 256, 8
    p_gb = 4 * E * H / GB
    res = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; fetch x2 (gfx950), GB per launch",
        "kernels": {n: k for n, (_, k, _) in zip(ORDER, fetch)},
        "fetch_GB": {n: round(v, 3) for n, v in fb.items()},
        "write_GB": {n: round(v, 3) for n, v in wb.items()},
        "model_GB": {"X_or_dY_rows_once": round(4 * N * F / GB, 3), "one_row_per_edge": round(4 * E * F / GB, 3),
                     "p": round(p_gb, 3), "Y_plus_Ym": round(8 * N * F / GB, 3)},
        "split": {
            "fwd_gather_as_probe": round(fb["probe_gather"], 3),
            "fwd_reads_beyond_gather": round(fb["fwd"] - fb["probe_gather"], 3),
            "fwd_writes_Y_Ym_stats": round(wb["fwd"], 3),
            "bwd_aR_lines": round(fb["bwd"] - (fb["bwd_p"] - p_gb), 3),
            "bwd_aR_bytes_per_edge": round((fb["bwd"] - (fb["bwd_p"] - p_gb)) * GB / E, 1),
            "bwd_reads_beyond_gather_and_aR": round(fb["bwd_p"] - p_gb - fb["probe_gather"], 3),
            "bwd_writes_dX_daL": round(wb["bwd"], 3),
            "fwd_p_extra_writes": round(wb["fwd_p"] - wb["fwd"], 3),
        },
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res["split"]))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--split":
        split(*sys.argv[2:5])
    else:
        run()
