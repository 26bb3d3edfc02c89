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
  gcn3_papers10  gala.dist_run on 4 ranks of this one GPU over gloo (halo, vertex cut sparse):
                 the 4-way partitions and exchanges at the full shape
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
    """One run as a child process; a heartbeat line every 60 s while it runs (a long
    host-staged multi-rank run would otherwise print nothing for minutes)."""
    import tempfile
    t0 = time.time()
    with tempfile.TemporaryFile("w+") as out, tempfile.TemporaryFile("w+") as err:
        p = subprocess.Popen(cmd, stdout=out, stderr=err, text=True, env=env, cwd=ROOT)
        while True:
            try:
                p.wait(timeout=60)
                break
            except subprocess.TimeoutExpired:
                if time.time() - t0 > limit:
                    p.kill()
                    p.wait()
                    break
                print(f"[config5_run] {tag}: running, {time.time() - t0:.0f} s", flush=True)
        out.seek(0)
        err.seek(0)
        stdout, stderr = out.read(), err.read()
    rec = {"run": tag, "rc": p.returncode, "wall_s": time.time() - t0}
    js = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    if js:
        rec["summary"] = json.loads(js[-1])
    rec["result_line"] = (stdout.strip().splitlines() or [""])[-1]
    if p.returncode != 0:
        rec["stderr"] = stderr[-2000:]
    print(json.dumps(rec), flush=True)
    return p.returncode


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
    # config 5's program split over 4 ranks on this one GPU (gloo: host-staged collectives, the
    # layouts' partitions and exchanges at the full 11.1 M-row shape)
    tr = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4", "--master-addr",
          "127.0.0.1", "--master-port=29533", "-m", "gala.dist_run"]
    steps += [
        ("gcn3_papers10 dist_run halo gloo world4", tr + [irs["gcn3_papers10"], "--synthetic", "--iters", iters,
                                                          "--dist"]),
        ("gcn3_papers10 dist_run vcut sparse gloo world4",
         tr + [irs["gcn3_papers10"], "--synthetic", "--iters", iters, "--layout", "vcut", "--dist",
               "--exchange", "sparse"]),
    ]
    only = sys.argv[2:]
    steps = [s for s in steps if not only or any(o in s[0] for o in only)]
    for tag, cmd in steps:
        e = dict(env, GALA_DIST_BACKEND="gloo") if "gloo" in tag else env
        if run(tag, cmd, e, limit=900 if "gloo" in tag else 600) != 0:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
