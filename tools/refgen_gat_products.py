#!/usr/bin/env python3
"""Config 3's drop-in path at its own shape: the GAT program the reference compiler emits
(tests/GALA-DSL/gat/Products/h100.txt: F 100 -> 32 -> 47, one head, col_tile(10000000), i.e.
one column segment) through HIPGenerator (refgen/bin/gala_gat_products), run on the MI355X on
a synthetic dataset of the ogbn-products shape (2 449 029 vertices, 126 167 309 stored edges)
in the reference's npy format.  Its edge operators are the base generator's own autograd
classes (common.h:622-894) over the operator mirror's unfused K5 / K7 / K8 / K9 and the
weighted SpMM.  Stages (one JSON line each):

  dataset  -- the npy files
  program  -- the program's own timing line (epochs 1-4 dropped, common.h:1494-1585)
  check    -- its first-epoch prediction on sampled rows against the float64 IR executor of
              galac's program of the same DSL (bench/dsl/gat_products_ref_codegen.txt), on the
              rows' 2-hop induced subgraph with the weights the program dumped
  op       -- each mirror op the program calls, timed alone at the same shape (HIP events on
              the current stream, 10 calls): ms, SURVEY §8(d) algorithmic bytes, frac of 8 TB/s

REFGEN_PROF=<dir> runs the program under rocprofv3 --kernel-trace --stats.
"""
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gala-gnn-acceleration-language_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _ir_ref as ref  # noqa: E402
import _refgen_check as rc  # noqa: E402
import bench  # noqa: E402
from gala import _abi, layout, ops  # noqa: E402

N, E_UND, F_IN, HID, LABELS = 2_449_029, 61_859_140, 100, 32, 47
PEAK = 8.0e12


def say(**kw):
    print(json.dumps(kw), flush=True)


def khop_induced(rowptr, col, seeds, hops):
    """Rows within `hops` of the seeds and the induced CSR on them (local ids); rows at distance
    < hops keep every edge (all an `hops`-layer forward of the seeds reads)."""
    cur = np.unique(np.asarray(seeds, np.int64))
    allr = cur
    for _ in range(hops):
        nb = np.concatenate([col[rowptr[r]:rowptr[r + 1]] for r in cur]).astype(np.int64)
        cur = np.setdiff1d(np.unique(nb), allr)
        allr = np.union1d(allr, cur)
    loc = np.full(len(rowptr) - 1, -1, np.int64)
    loc[allr] = np.arange(len(allr))
    rp, cl = [0], []
    for r in allr:
        cs = loc[col[rowptr[r]:rowptr[r + 1]]]
        cs = cs[cs >= 0]
        cl.append(cs)
        rp.append(rp[-1] + len(cs))
    return allr, np.asarray(rp, np.int64), np.concatenate(cl)


def main():
    n, e_und = N, E_UND
    if len(sys.argv) > 1:      # a smaller run: refgen_gat_products.py ROWS
        n = int(sys.argv[1])
        e_und = n * (E_UND // N)
    exe = os.path.join(PKG, "refgen", "bin", "gala_gat_products")
    root = tempfile.mkdtemp(prefix="refgen_gat_")
    t0 = time.time()
    g = layout.gen_graph("uniform", n, e_und, seed=42)
    d = os.path.join(root, "Data", "Cora")
    os.makedirs(d)
    rows = np.repeat(np.arange(n, dtype=np.uint32), np.diff(g.rowptr))
    np.save(os.path.join(d, "Adj_src.npy"), np.concatenate([np.array([n, n], np.uint32), rows]))
    np.save(os.path.join(d, "Adj_dst.npy"), g.col.astype(np.uint32))
    del rows
    rng = np.random.default_rng(5)
    X = rng.uniform(-1, 1, (n, F_IN)).astype(np.float32)
    np.save(os.path.join(d, "Feat.npy"), X)
    np.save(os.path.join(d, "Lab.npy"), rng.integers(0, LABELS, (n, 1)).astype(np.int64))
    for name, frac in (("TnMsk", 0.08), ("VlMsk", 0.02), ("TsMsk", 0.9)):
        np.save(os.path.join(d, name + ".npy"), (rng.random((n, 1)) < frac).astype(np.int32))
    say(stage="dataset", vertices=n, edges=int(g.nnz), F=F_IN, s=round(time.time() - t0, 1))

    # the program (10 epochs; the dump holds epoch 1)
    cwd = os.path.join(root, "run", "b")
    os.makedirs(cwd)
    dump_path = os.path.join(root, "dump.bin")
    env = dict(os.environ, GALA_DEVICE="cuda", GALA_DUMP=dump_path, GALA_SEED="3")
    cmd = [exe]
    if os.environ.get("REFGEN_PROF"):
        cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.abspath(os.environ["REFGEN_PROF"]),
               "-o", "run", "--"] + cmd
    t0 = time.time()
    p = subprocess.Popen(cmd, cwd=cwd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    while True:
        try:
            out, err = p.communicate(timeout=60)
            break
        except subprocess.TimeoutExpired:
            say(stage="program", running_s=round(time.time() - t0, 1))
    if p.returncode != 0:
        say(stage="program", rc=p.returncode, stderr=err[-2000:])
        return 1
    last = [ln for ln in out.splitlines() if re.fullmatch(r"[0-9.e+-]+,[0-9.e+-]+", ln.strip())][-1].strip()
    fwd_s, total_s = (float(v) for v in last.split(","))
    dump = rc.read_dump(dump_path)
    say(stage="program", epochs=10, wall_s=round(time.time() - t0, 1), fwd_mean_s=fwd_s, epoch_mean_s=total_s,
        timing_line=last, loss_first=float(dump["loss"][0]))

    # galac's programs on the same dataset: the same DSL and passes, and galac's defaults
    for prog in ("gat_products_ref_codegen", "gat_products"):
        pexe = os.path.join(PKG, "progs", prog, "gala_prog")
        if not os.path.exists(pexe):
            continue
        r = subprocess.run([pexe, "--data", d + "/", "--iters", "10"], capture_output=True, text=True, timeout=600)
        line = (r.stdout.strip().splitlines() or [""])[-1].strip()
        rec = {"stage": "galac", "program": prog, "rc": r.returncode, "timing_line": line}
        if r.returncode == 0 and re.fullmatch(r"[0-9.e+-]+,[0-9.e+-]+", line):
            rec["fwd_mean_s"], rec["epoch_mean_s"] = (float(v) for v in line.split(","))
        else:
            rec["stderr"] = r.stderr[-1500:]
        say(**rec)

    # check: galac's IR of the same DSL in float64 on the sampled rows' 2-hop induced subgraph
    t0 = time.time()
    ir_path = os.path.join(root, "ir.json")
    subprocess.run([rc.GALAC, os.path.join(ROOT, "bench", "dsl", "gat_products_ref_codegen.txt"), "--quiet",
                    "--ir-json", ir_path], check=True)
    ir = ref.load_ir(ir_path)["post"]
    rowptr = g.rowptr.astype(np.int64)
    seeds = np.array([0, n // 3, (2 * n) // 3, n - 1])
    allr, rp, cl = khop_induced(rowptr, g.col, seeds, 2)
    graphs = ref.Graphs(ir, rp, cl, np.ones(len(allr), np.int32))
    params = {k: torch.as_tensor(v, dtype=torch.float64) for k, v in dump.items()
              if k not in ("prediction", "loss") and not k.endswith(".grad")}
    with torch.no_grad():
        want = ref.run(ir, graphs, torch.as_tensor(X[allr], dtype=torch.float64), params).numpy()
    at = np.searchsorted(allr, seeds)
    got = dump["prediction"][seeds].astype(np.float64)
    err = np.abs(got - want[at])
    ok = bool(np.all(err <= 1e-4 + 1e-4 * np.abs(want[at])))
    say(stage="check", seeds=seeds.tolist(), induced_rows=int(len(allr)), induced_edges=int(len(cl)),
        max_abs_err=float(err.max()), within_1e4=ok, s=round(time.time() - t0, 1))

    # the mirror ops the program's GAT classes call, each alone at the same shape
    timer = bench.Timer(True)
    dg = ops.DeviceGraph.from_host(g)
    E = g.nnz
    gen = torch.Generator(device="cuda").manual_seed(9)
    aL = torch.rand(n, device="cuda", generator=gen) - 0.5
    aR = torch.rand(n, device="cuda", generator=gen) - 0.5
    s = torch.rand(E, device="cuda", generator=gen)
    q = torch.rand(n, device="cuda", generator=gen)
    rp_b = 4 * (n + 1)
    table = []

    def op(name, fn, alg_bytes, kernel, in_program=True):
        ms = timer(fn, 10) * 1e3
        table.append(dict(stage="op", op=name, kernel=kernel, ms=round(ms, 4), alg_bytes=int(alg_bytes),
                          achieved_GBps=round(alg_bytes / ms / 1e6, 1), frac=round(alg_bytes / (ms * 1e-3) / PEAK, 4),
                          in_program=in_program))

    op("K5 edge_sddvv (ADD)", lambda: ops.sddvv(dg, aL, aR, op=_abi.GALA_SDDVV_ADD),
       rp_b + 4 * E + 8 * n + 4 * E, "k_sddvv")
    op("K7 node_spmv_backward_of_sddmm (row sum)", lambda: ops.row_sum(dg, s, eps=1e-12),
       rp_b + 4 * E + 4 * n, "k_row_sum")
    sc = s.clone()
    op("K8 inplace_softmax_sddvv (row scale)", lambda: ops.row_scale_(dg, q, sc), rp_b + 8 * E + 4 * n,
       "k_row_scale")
    gw = dg.with_values(s)
    # F = 47 is the width the DSL's second layer would aggregate at; the reference's operator
    # reordering moves that layer's FFN after its aggregation, so the program aggregates at 32
    # in both layers (the F = 47 rows are for reference)
    for F in (HID, LABELS):
        Xf = torch.rand(n, F, device="cuda", generator=gen)
        Af = torch.rand(n, F, device="cuda", generator=gen)
        op(f"weighted SpMM F={F} (aggregate_node_mul_sum, attention values)", lambda: ops.spmm(gw, Xf),
           rp_b + 8 * E + 8 * n * F, "k_spmm_rowgroup<W>", F == HID)
        op(f"K9 edge_sddmm F={F}", lambda: ops.sddmm(dg, Af, Xf), rp_b + 4 * E + 8 * n * F + 4 * E, "k_sddmm",
           F == HID)
        del Xf, Af
    for t in table:
        say(**t)
    worst = min((t for t in table if t["in_program"]), key=lambda t: t["frac"])
    say(stage="worst_op", op=worst["op"], frac=worst["frac"])
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
