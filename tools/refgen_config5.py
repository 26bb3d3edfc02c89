#!/usr/bin/env python3
"""Config 5's GCN-3 as the reference compiler emits it, at config 5's shape, on the MI355X.

refgen/bin/gala_gcn3_papers (refgen/build.py: the reference driver's steps with HIPGenerator on
the three-layer GCN IR, F = 128, hidden 128, 172 labels, col_tile(1000000) as
bench/dsl/gcn3_papers10.txt) runs on a synthetic dataset of the 10 % ogbn-papers100M node
subgraph's shape (11 105 995 vertices, 27.3 M stored edges incl. self loops) written in the
reference's npy format; the program's own timing line (forward, forward + backward + step; the
reference's protocol, epochs 1-4 dropped, common.h:1494-1585) and its first-epoch prediction are
reported, the prediction checked against galac's program of the same DSL in the float64 IR
executor on the weights the program dumped.  Measurement; prints one JSON line per stage.
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
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _ir_ref as ref  # noqa: E402
import _refgen_check as rc  # noqa: E402
from gala import layout  # noqa: E402

N, E_UND, F, LABELS = 11_105_995, (27_262_853 - 11_105_995) // 2, 128, 172


def say(**kw):
    print(json.dumps(kw), flush=True)


def main():
    global N, E_UND
    device = "cuda"
    if len(sys.argv) > 1:                      # dry run: refgen_config5.py ROWS cpu
        N, device = int(sys.argv[1]), sys.argv[2]
        E_UND = N
    exe = os.path.join(PKG, "refgen", "bin", "gala_gcn3_papers")   # 10 epochs (refgen/build.py)
    root = tempfile.mkdtemp(prefix="refgen_c5_")
    t0 = time.time()
    g = layout.gen_graph("uniform", N, E_UND, seed=42)
    d = os.path.join(root, "Data", "Cora")
    os.makedirs(d)
    rows = np.repeat(np.arange(N, dtype=np.uint32), np.diff(g.rowptr))
    np.save(os.path.join(d, "Adj_src.npy"), np.concatenate([np.array([N, N], np.uint32), rows]))
    np.save(os.path.join(d, "Adj_dst.npy"), g.col.astype(np.uint32))
    del rows
    rng = np.random.default_rng(5)
    X = rng.uniform(-1, 1, (N, F)).astype(np.float32)
    np.save(os.path.join(d, "Feat.npy"), X)
    np.save(os.path.join(d, "Lab.npy"), rng.integers(0, LABELS, (N, 1)).astype(np.int64))
    for name, frac in (("TnMsk", 0.3), ("VlMsk", 0.2), ("TsMsk", 0.5)):
        np.save(os.path.join(d, name + ".npy"), (rng.random((N, 1)) < frac).astype(np.int32))
    say(stage="dataset", vertices=N, edges=int(g.nnz), F=F, s=round(time.time() - t0, 1))

    # the program, iters epochs on the GPU (the dump holds epoch 1)
    cwd = os.path.join(root, "run", "b")
    os.makedirs(cwd)
    dump_path = os.path.join(root, "dump.bin")
    env = dict(os.environ, GALA_DEVICE=device, GALA_DUMP=dump_path)
    t0 = time.time()
    cmd = [exe]
    if os.environ.get("REFGEN_PROF"):          # kernel trace of the program: REFGEN_PROF=out_dir
        cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.abspath(os.environ["REFGEN_PROF"]),
               "-o", "run", "--"] + cmd
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
    say(stage="program", epochs=10, wall_s=round(time.time() - t0, 1), fwd_mean_s=fwd_s,
        epoch_mean_s=total_s, timing_line=last, loss_first=float(dump["loss"][0]))

    # galac's programs on the same dataset: the same DSL and passes (tests/dsl/
    # gcn3_papers_ref_codegen.txt: gala_inference's operator reordering, no code motion, no
    # training subgraph) and galac's defaults (bench/dsl/gcn3_papers10.txt: code motion hoists
    # the first aggregation out of the loop)
    for prog in ("gcn3_papers_ref_codegen", "gcn3_papers10"):
        pexe = os.path.join(PKG, "progs", prog, "gala_prog")
        if not os.path.exists(pexe) or device != "cuda":
            continue
        r = subprocess.run([pexe, "--data", d + "/", "--iters", "10"], capture_output=True, text=True, timeout=600)
        line = (r.stdout.strip().splitlines() or [""])[-1].strip()
        rec = {"stage": "galac", "program": prog, "rc": r.returncode, "timing_line": line}
        if r.returncode == 0 and re.fullmatch(r"[0-9.e+-]+,[0-9.e+-]+", line):
            rec["fwd_mean_s"], rec["epoch_mean_s"] = (float(v) for v in line.split(","))
        else:
            rec["stderr"] = r.stderr[-1500:]
        say(**rec)

    # galac's program of the same DSL, forward in float64 on the dumped weights
    t0 = time.time()
    ir_path = os.path.join(root, "ir.json")
    subprocess.run([rc.GALAC, os.path.join(ROOT, "tests", "dsl", "gcn3_papers_ref_codegen.txt"), "--quiet",
                    "--ir-json", ir_path], check=True)
    ir = ref.load_ir(ir_path)["post"]
    graphs = ref.Graphs(ir, g.rowptr, g.col, np.ones(N, np.int32))
    params = {k: torch.as_tensor(v, dtype=torch.float64) for k, v in dump.items()
              if k not in ("prediction", "loss") and not k.endswith(".grad")}
    with torch.no_grad():
        want = ref.run(ir, graphs, torch.as_tensor(X, dtype=torch.float64), params).numpy()
    err = np.abs(dump["prediction"].astype(np.float64) - want)
    ok = bool(np.all(err <= 1e-4 + 1e-4 * np.abs(want)))
    say(stage="check", rows=N, max_abs_err=float(err.max()), within_1e4=ok, s=round(time.time() - t0, 1))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
