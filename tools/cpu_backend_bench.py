#!/usr/bin/env python3
"""Host cores: libgala_cpu.so's SpMM (the CPU backend, include/gala_cpu.h) against the
reference's own gSpMM + wsumAgg compiled from /root/reference (oracle/_ref) on the same
Products-shaped graph and features; checks the two outputs are bit-identical and prints one
JSON line per F (median of timed calls, all host threads for both)."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from gala import _abi, layout  # noqa: E402
import oracle as orc  # noqa: E402


def median_time(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_449_029)
    ap.add_argument("--u", type=int, default=61_859_140)
    ap.add_argument("--F", default="32")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    g = layout.gen_graph("uniform", a.n, a.u, seed=42)
    og = orc.Graph(g.n_rows, g.n_cols, g.rowptr, g.col, None)
    c = _abi.gala_csr_t()
    c.n_rows, c.n_cols, c.nnz = g.n_rows, g.n_cols, g.nnz
    c.rowptr, c.col, c.val, c.val_heads, c.n_seg = g.rowptr.ctypes.data, g.col.ctypes.data, None, 1, 1
    c.seg_bounds, c.split = None, None
    for F in [int(f) for f in a.F.split(",")]:
        X = np.random.default_rng(1234).uniform(-1, 1, (g.n_cols, F)).astype(np.float32)
        Y = np.empty((g.n_rows, F), np.float32)

        def ours():
            _abi.call_cpu("gala_spmm_f32", ctypes.byref(c), X.ctypes.data, F, Y.ctypes.data, F, F,
                          None, None, 0, 0, 5, 7, None)
        t_ours = median_time(ours, a.reps)
        line = {"F": F, "E": g.nnz, "gala_cpu_edges_per_s": g.nnz / t_ours, "gala_cpu_s": t_ours,
                "threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count()))}
        if orc.ref_available():
            ref = {}

            def theirs():
                ref["Y"] = orc.ref_gspmm(og, X)
            t_ref = median_time(theirs, a.reps)
            line.update(reference_edges_per_s=g.nnz / t_ref, reference_s=t_ref,
                        reference_threads=orc.ref_threads(), bit_identical=bool(np.array_equal(Y, ref["Y"])))
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
