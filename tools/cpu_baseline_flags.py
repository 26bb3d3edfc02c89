#!/usr/bin/env python3
"""Container table for DESIGN §5: the reference gSpMM (oracle/_ref) under different -march
flags and timing harnesses, on the ogbn-products-shaped uniform graph, F = 32.

  build  REF_MARCH=x86-64-v3 | x86-64-v4 | native  (oracle/build_ref.sh, into /tmp)
  timing "alloc":  ref_gspmm(og, X) with val = ones(E) and Y = zeros(N, F) made per call
         "kernel": val / Y preallocated, Y re-zeroed outside the timed region (bench.py)

Prints one JSON line per (march, timing) cell: median of `--reps` calls after a warm-up.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc  # noqa: E402
from gala import layout  # noqa: E402


def load(march):
    out = f"/tmp/gala_ref_{march}.so"
    env = dict(os.environ, REF_MARCH=march, REF_OUT=out)
    subprocess.run([os.path.join(ROOT, "oracle", "build_ref.sh")], check=True, env=env,
                   stdout=subprocess.DEVNULL)
    return ctypes.CDLL(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--F", type=int, default=32)
    a = ap.parse_args()
    n = int(2_449_029 * a.scale)
    E = n + 2 * ((int(126_167_309 * a.scale) - n) // 2)
    g = layout.gen_graph("uniform", n, (E - n) // 2, seed=42)
    X = np.random.default_rng(1234).uniform(-1, 1, (g.n_cols, a.F)).astype(np.float32)
    val = np.ones(g.nnz, np.float32)
    Y = np.zeros((g.n_rows, a.F), np.float32)
    ip = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    for march in ("x86-64-v3", "x86-64-v4", "native"):
        L = load(march)
        L.ref_set_threads(a.threads)
        for timing in ("alloc", "kernel"):
            def call():
                if timing == "alloc":
                    v = np.ones(g.nnz, np.float32)
                    y = np.zeros((g.n_rows, a.F), np.float32)
                else:
                    v, y = val, Y
                L.ref_gspmm(g.n_rows, g.n_cols, g.nnz, ip(g.rowptr), ip(g.col), ip(v), ip(X), a.F, ip(y))
            call()
            ts = []
            for _ in range(a.reps):
                Y.fill(0.0)
                t0 = time.perf_counter()
                call()
                ts.append(time.perf_counter() - t0)
            t = float(np.median(ts))
            print(json.dumps({"march": march, "timing": timing, "threads": a.threads, "s_per_call": t,
                              "edges_per_s": g.nnz / t, "N": g.n_rows, "E": g.nnz, "F": a.F}), flush=True)


if __name__ == "__main__":
    main()
