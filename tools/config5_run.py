#!/usr/bin/env python3
"""Config 5 (and config 3) programs at size through the multi-rank runtime on one GPU.

Runs, one after another (each a child process with its own time limit), and prints one JSON
line per run:
  gcn3_papers10  the galac-generated single-device binary (progs/gcn3_papers10/gala_prog)
  gcn3_papers10  gala.dist_run, halo layout (world 1: exact SpMM, no collectives)
  gcn3_papers10  gala.dist_run --layout vcut --dist: the vertex cut with its collectives
                 over RCCL at world 1 (dense reduce-scatter, and the sparse all-to-all)
  gat_products_h8  the generated binary, then gala.dist_run --layout vcut --dist (config 3's
                 8-head GAT program as VertexCutGat layers) and the halo layout over RCCL
                 (HaloGat layers)
  sage_reddit_sampled  config 4 (kernel-sampled SAGE on the Reddit shape): the generated
                 binary, then gala.dist_run on the row partition, alone and over RCCL
Epoch times are the programs' own means (first epochs dropped, as gala.cu:613-637).
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gala-gnn-acceleration-language_amd")
GALAC = os.path.join(PKG, "gala", "galac")


def run(tag, cmd, env, limit=600):
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=limit, env=env, cwd=ROOT)
    rec = {"run": tag, "rc": r.returncode, "wall_s": time.time() - t0}
    js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if js:
        rec["summary"] = json.loads(js[-1])
    rec["result_line"] = (r.stdout.strip().splitlines() or [""])[-1]
    if r.returncode != 0:
        rec["stderr"] = r.stderr[-2000:]
    print(json.dumps(rec), flush=True)
    return r.returncode


def main():
    iters = sys.argv[1] if len(sys.argv) > 1 else "20"
    env = dict(os.environ)
    env["PYTHONPATH"] = PKG + os.pathsep + env.get("PYTHONPATH", "")
    env.pop("GALA_DIST_BACKEND", None)
    irs = {}
    for prog in ("gcn3_papers10", "gat_products_h8", "sage_reddit_sampled"):
        irs[prog] = f"/tmp/{prog}.json"
        subprocess.run([GALAC, os.path.join(ROOT, "bench", "dsl", f"{prog}.txt"), "--quiet", "--ir-json",
                        irs[prog]], check=True)
    dr = [sys.executable, "-m", "gala.dist_run"]
    steps = [
        ("gcn3_papers10 generated binary", [os.path.join(PKG, "progs", "gcn3_papers10", "gala_prog"), "--synthetic",
                                            "--iters", iters]),
        ("gcn3_papers10 dist_run halo world1", dr + [irs["gcn3_papers10"], "--synthetic", "--iters", iters]),
        ("gcn3_papers10 dist_run vcut dense RCCL world1",
         dr + [irs["gcn3_papers10"], "--synthetic", "--iters", iters, "--layout", "vcut", "--dist",
               "--exchange", "dense"]),
        ("gcn3_papers10 dist_run vcut sparse RCCL world1",
         dr + [irs["gcn3_papers10"], "--synthetic", "--iters", iters, "--layout", "vcut", "--dist",
               "--exchange", "sparse"]),
        ("gat_products_h8 generated binary", [os.path.join(PKG, "progs", "gat_products_h8", "gala_prog"),
                                              "--synthetic", "--iters", iters]),
        ("gat_products_h8 dist_run vcut dense RCCL world1",
         dr + [irs["gat_products_h8"], "--synthetic", "--iters", iters, "--layout", "vcut", "--dist",
               "--exchange", "dense"]),
        ("gat_products_h8 dist_run halo RCCL world1",
         dr + [irs["gat_products_h8"], "--synthetic", "--iters", iters, "--dist"]),
        ("sage_reddit_sampled generated binary", [os.path.join(PKG, "progs", "sage_reddit_sampled", "gala_prog"),
                                                  "--synthetic", "--iters", iters]),
        ("sage_reddit_sampled dist_run halo world1", dr + [irs["sage_reddit_sampled"], "--synthetic", "--iters", iters]),
        ("sage_reddit_sampled dist_run halo RCCL world1",
         dr + [irs["sage_reddit_sampled"], "--synthetic", "--iters", iters, "--dist"]),
    ]
    only = sys.argv[2:]
    steps = [s for s in steps if not only or any(s[0].startswith(o) for o in only)]
    for tag, cmd in steps:
        if run(tag, cmd, env) != 0:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
