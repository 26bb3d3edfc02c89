#!/usr/bin/env python3
"""Headline benchmark: aggregated edges/sec of the GCN-2 hot path on an
ogbn-products-shaped graph (BASELINE.json: "aggregated edges/sec, GCN-2 ogbn-products at
1/2/4/8 MI355X; % HBM roofline").

One step = the hot-path work of one GCN-2 training epoch of the generated program
(codegen/gala.cu:423-459 + the autograd backward, gala.cu:391-414):
    norm = degree(A)^-1/2                       (gala_degree_f32, fused pow)
    layer-1 forward  H1 = norm * A (norm * X)   (gala_row_broadcast_f32 + gala_spmm_f32
                                                 with the dst norm fused, F=32)
    layer-2 forward  H2 = norm * A (norm * H1)
    layer-2 backward dH1 = norm * A (norm * dH2)   (undirected: same CSR, gala.cu:403-413)
    layer-1 backward dX  = norm * A (norm * dH1)
Edges counted per step = 4 * E (the four F=32 aggregations; the degree pass is timed
but not counted).  Synthetic data: uniform random symmetric graph with the Products
shape (N=2,449,029, E=126,167,309 incl. self loops), X ~ U[-1,1) fp32.

N>1 (torch.distributed, one rank per GPU): see DESIGN.md §Multi-GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))

from gala import layout, ops  # noqa: E402

PRODUCTS_N = 2_449_029
PRODUCTS_UNDIRECTED = 61_859_140  # 2*U + N = 126,167,309 stored edges
HBM_PEAK = 8.0e12                 # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spmm_alg_bytes(n_rows, n_cols, nnz, F, weighted=False, scaled=True):
    """4(N+1) + 4E [+4E] + 4*N*F (X once) + 4*N*F (Y write) [+ 4N dst norm]."""
    b = 4 * (n_rows + 1) + 4 * nnz + 4 * n_cols * F + 4 * n_rows * F
    if weighted:
        b += 4 * nnz
    if scaled:
        b += 4 * n_rows
    return b


def cpu_baseline(g: layout.HostGraph, F: int, budget_s: float = 20.0):
    """Reference CPU aggregation timed on the host cores (rank 0, N=1 only)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    og = orc.Graph(g.n_rows, g.n_cols, g.rowptr, g.col, None)
    X = np.random.default_rng(1234).uniform(-1, 1, (g.n_cols, F)).astype(np.float32)
    kind = "reference" if orc.ref_available() else "port"
    fn = (lambda: orc.ref_gspmm(og, X)) if kind == "reference" else (lambda: orc.gspmm(og, X))
    cores = orc.ref_threads() if kind == "reference" else int(os.environ.get("OMP_NUM_THREADS", os.cpu_count()))
    fn()  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 5 and (time.perf_counter() - t_start) < budget_s:
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": g.nnz / t, "unit": "edges/s", "cores": cores, "kind": kind,
            "sample": f"{len(times)} full-graph SpMM calls (F={F}, E={g.nnz}) after 1 warm-up, "
                      f"median {t:.3f} s; {'reference gSpMM+wsumAgg compiled from /root/reference' if kind == 'reference' else 'oracle restatement of gSpMM'}"}


def load_traffic(kernel_substr: str):
    """Per-launch HBM bytes of the dominant kernel from a committed PMC summary (or None)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        for k, v in d.get("kernels", {}).items():
            if kernel_substr in k:
                return float(v["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--F", type=int, default=32)
    ap.add_argument("--graph", default="uniform", choices=["uniform", "rmat"])
    ap.add_argument("--scale", type=float, default=1.0, help="graph size multiplier (debug)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    N = int(PRODUCTS_N * args.scale)
    U = int(PRODUCTS_UNDIRECTED * args.scale)
    F = args.F
    t0 = time.time()
    hg = layout.gen_graph(args.graph, N, U, seed=42)
    log(f"[rank {rank}] graph N={hg.n_rows} E={hg.nnz} built in {time.time() - t0:.1f}s")
    dg = ops.DeviceGraph.from_host(hg)
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    X = torch.rand((N, F), device="cuda", generator=gen) * 2 - 1
    dY = torch.rand((N, F), device="cuda", generator=gen) * 2 - 1
    Xs = torch.empty_like(X)   # norm-prescaled input of the current aggregation
    H1 = torch.empty_like(X)
    H2 = torch.empty_like(X)
    G1 = torch.empty_like(X)
    G0 = torch.empty_like(X)

    stream = torch.cuda.current_stream()
    spmm_ev = []

    def step(record=False):
        norm = ops.degree(dg, power=-0.5)
        for src, dst in ((X, H1), (H1, H2), (dY, G1), (G1, G0)):
            ops.row_broadcast(norm, src, out=Xs)           # `norm * res` (ROW_BROADCAST)
            if record:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            ops.spmm(dg, Xs, dst_scale=norm, out=dst)        # norm * A (.)
            if record:
                e1.record(stream)
                spmm_ev.append((e0, e1))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t_start = torch.cuda.Event(enable_timing=True)
    t_end = torch.cuda.Event(enable_timing=True)
    w0 = time.perf_counter()
    t_start.record(stream)
    for _ in range(args.steps):
        step(record=True)
    t_end.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - w0
    elapsed = t_start.elapsed_time(t_end) / 1e3
    elapsed = max(elapsed, 0.0)
    if world > 1:
        t = torch.tensor([wall], device="cuda", dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        wall = float(t.item())
    t_step = wall / args.steps
    spmm_ms = [a.elapsed_time(b) for a, b in spmm_ev]
    t_spmm = float(np.mean(spmm_ms)) / 1e3
    edges_per_step = 4 * hg.nnz
    value = world * edges_per_step / t_step

    alg = spmm_alg_bytes(hg.n_rows, hg.n_cols, hg.nnz, F)
    achieved = alg / t_spmm
    traffic = load_traffic("k_spmm_rowgroup")
    out = {
        "metric": "aggregated edges/sec, GCN-2 ogbn-products (4 F=32 aggregations per step)",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_step * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic {args.graph} symmetric graph + self loops (seed 42), X~U[-1,1)",
        "config": {"workload": "GCN-2 ogbn-products-shaped hot path (degree + 2 fwd + 2 bwd SpMM, F=32)",
                   "n_rows": hg.n_rows, "nnz": hg.nnz, "F": F, "parallelism": f"replica{world}" if world > 1 else "1gpu"},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic,
                     "kernel": "k_spmm_rowgroup<4,8,1,8,unweighted,dst-scaled> (gala_spmm_f32 F=32)",
                     "kernel_ms": t_spmm * 1e3, "alg_bytes_per_launch": alg,
                     "gather_GBps": (4 * (hg.n_rows + 1) + hg.nnz * (4 + 4 * F + 4) + 4 * hg.n_rows * F) / t_spmm / 1e9},
        "event_ms_per_step": elapsed * 1e3 / args.steps,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(hg, F)
        except Exception as e:  # the baseline is reported, never the target
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
