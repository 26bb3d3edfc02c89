#!/usr/bin/env python3
"""Headline benchmark: aggregated edges/sec of the GCN-2 hot path, ogbn-products shape
(BASELINE.json: "aggregated edges/sec, GCN-2 ogbn-products at 1/2/4/8 MI355X; % HBM roofline").

One step = the hot-path work of one GCN-2 training epoch of the generated program
(codegen/gala.cu:423-459 forward + the autograd backward, gala.cu:391-414):
    norm = degree(A)^-1/2                               gala_degree_f32 (fused pow)
    layer-1 forward   H1 = norm * A (norm * X)          gala_row_broadcast_f32 +
    layer-2 forward   H2 = norm * A (norm * H1)         gala_spmm_f32 (dst norm fused),
    layer-2 backward dH1 = norm * A (norm * dH2)        F = 32, fp32
    layer-1 backward  dX = norm * A (norm * dH1)        (undirected: same CSR, gala.cu:403-413)
Edges counted per step = 4 * E per GPU (the four aggregations; the degree pass is timed
but not counted).  The dense layers and activations of the epoch are torch, not the
hot path, and are not part of the step.

N = 1: the ogbn-products-shaped graph (N=2,449,029 vertices, E=126,167,309 stored edges
incl. self loops), uniform random symmetric edges, X ~ U[-1,1).
N > 1 (one process per GPU, RCCL): weak scaling over vertex partitions (gala/dist.py):
every GPU owns an ogbn-products-sized partition (same N and E per GPU); 10% of each
partition's edges are cut edges to the other partitions' boundary vertices (10% of each
partition), whose feature rows arrive by one RCCL all-gather per aggregation, overlapped
with the local-edge SpMM.
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

from gala import dist as gdist  # noqa: E402
from gala import layout, ops  # noqa: E402

PRODUCTS_N = 2_449_029
PRODUCTS_E = 126_167_309          # 2 * 61,859,140 undirected + N self loops
HBM_PEAK = 8.0e12                 # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spmm_alg_bytes(n_rows, n_cols_read, nnz, F):
    """SURVEY §8(d) unweighted SpMM: 4(N+1) + 4E + 4*N*F (X read once) + 4*N*F (Y write),
    + 4N for the fused dst norm."""
    return 4 * (n_rows + 1) + 4 * nnz + 4 * n_cols_read * F + 4 * n_rows * F + 4 * n_rows


def cpu_baseline(g: layout.HostGraph, F: int, budget_s: float = 20.0):
    """Reference CPU aggregation on the host cores (rank 0, N=1 only)."""
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
            "sample": f"{len(times)} full-graph F={F} SpMM calls (E={g.nnz}) after 1 warm-up, median "
                      f"{t:.3f} s; " + ("reference gSpMM+wsumAgg (src/ops/aggregators.h) compiled from "
                                        "/root/reference, OpenMP" if kind == "reference"
                                        else "oracle restatement of gSpMM, OpenMP")}


def load_traffic(kernel_substr: str):
    """Per-launch HBM bytes of the dominant kernel from the committed PMC summary."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(path))
        for k, v in d.get("kernels", {}).items():
            if kernel_substr in k:
                return float(v["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def gather_ceiling(col, X, stream, reps=10):
    """Time (HIP events, same stream) an unordered gather of the very rows the SpMM fetches:
    X[col[e]] for every edge e, any order, no row bookkeeping, no output rows
    (tools/gather_ceiling.hip -> tools/libgala_probe.so).  The floor for any kernel that
    fetches one X row per edge.  None when the probe library was not built."""
    import ctypes
    path = os.path.join(ROOT, "tools", "libgala_probe.so")
    if not os.path.exists(path) or X.shape[1] not in (32, 128, 256):
        return None
    L = ctypes.CDLL(path)
    fn = L.gala_probe_gather_f32
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                   ctypes.c_void_p]
    E, F = col.numel(), X.shape[1]
    out = torch.empty(((E + 63) // 64, F), device=X.device, dtype=torch.float32)
    args = (col.data_ptr(), X.data_ptr(), E, F, out.data_ptr(), stream.cuda_stream)
    if fn(*args) != 0:
        return None
    return event_time(lambda: fn(*args), reps, stream)


def event_time(fn, reps, stream):
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        ts.append((a, b))
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ts])) / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--F", type=int, default=32)
    ap.add_argument("--scale", type=float, default=1.0, help="per-GPU graph size multiplier (debug)")
    ap.add_argument("--cut-frac", type=float, default=0.1)
    ap.add_argument("--boundary-frac", type=float, default=0.1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("GALA_DIST_BACKEND", "nccl")  # gloo: 1-GPU rehearsal only
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    n = int(PRODUCTS_N * args.scale)
    E = n + 2 * ((int(PRODUCTS_E * args.scale) - n) // 2)
    F = args.F
    t0 = time.time()
    part = gdist.make_partition(rank, world, n, E, cut_frac=args.cut_frac,
                                boundary_frac=args.boundary_frac, seed=42)
    hg = part.graph
    log(f"[rank {rank}/{world}] partition n={hg.n_rows} cols={hg.n_cols} E={hg.nnz} "
        f"(cut {part.n_cut_edges}) built in {time.time() - t0:.1f}s")
    agg = gdist.DistGCNAggregator(part, F, dev)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    X = torch.rand((n, F), device=dev, generator=gen) * 2 - 1
    dY = torch.rand((n, F), device=dev, generator=gen) * 2 - 1
    H1, H2, G1, G0 = (torch.empty_like(X) for _ in range(4))
    stream = torch.cuda.current_stream()

    def step():
        agg.norm = ops.degree(agg.full, power=-0.5)   # recomputed every forward (gala.cu:433-440)
        agg(X, H1)
        agg(H1, H2)
        agg(dY, G1)
        agg(G1, G0)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - w0
    if world > 1:
        t = torch.tensor([wall], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        wall = float(t.item())
    t_step = wall / args.steps
    value = world * 4 * hg.nnz / t_step

    # dominant kernel, measured live with HIP events on the launch stream: the local
    # (segment-0) SpMM of one aggregation = the whole-graph SpMM at N = 1
    seg0 = agg.segs[0]
    Y = torch.empty_like(X)
    t_kernel = event_time(lambda: ops.spmm(seg0, agg.Xs, dst_scale=agg.norm, out=Y), 10, stream)
    alg = spmm_alg_bytes(hg.n_rows, hg.n_rows, seg0.nnz, F)
    achieved = alg / t_kernel
    gather_bytes = 4 * (hg.n_rows + 1) + seg0.nnz * (4 + 4 * F) + 4 * hg.n_rows * F
    traffic = load_traffic("k_spmm_rowgroup<4, 8, 1, 4, false, false, false>") if world == 1 else None
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
        "data": "synthetic: uniform random symmetric graph + self loops per GPU partition (seed 42), "
                "X~U[-1,1) fp32; N>1 adds 10% cut edges between partitions' boundary vertices",
        "config": {"workload": "GCN-2 ogbn-products-shaped hot path per GPU: degree + 2 fwd + 2 bwd "
                               "norm-scaled SpMM aggregations, F=32",
                   "n_vertices_per_gpu": hg.n_rows, "edges_per_gpu": hg.nnz, "F": F,
                   "cut_edges_per_gpu": part.n_cut_edges,
                   "parallelism": "1 GPU" if world == 1 else f"vertex partitions x{world}, RCCL all-gather halo"},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic,
                     "kernel": "gala::k_spmm_rowgroup<VEC=4,G=8,CH=1,U=4,unweighted> (gala_spmm_f32, F=32, dst norm)",
                     "kernel_ms": t_kernel * 1e3, "alg_bytes_per_launch": alg,
                     "gather_model_GBps": gather_bytes / t_kernel / 1e9,
                     "traffic_note": "PMC FETCH_SIZE*2+WRITE_SIZE per launch (profiles/traffic.json); "
                                     "uniform random columns: each edge's 128-B X row misses L2"},
        "event_ms_per_step": ev0.elapsed_time(ev1) / args.steps,
    }
    t_ceil = gather_ceiling(seg0.col, agg.Xs, stream)
    if t_ceil:
        out["roofline"]["gather_ceiling_ms"] = t_ceil * 1e3
        out["roofline"]["frac_of_gather_ceiling"] = t_ceil / t_kernel
        out["roofline"]["gather_ceiling_note"] = (
            "same process and graph: X[col[e]] for every edge, unordered, no output rows "
            "(tools/gather_ceiling.hip); the SpMM's floor on a graph without reuse")
    if world > 1:
        send = agg.Xs[:part.b]
        recv = agg.Xs[part.n:]
        t_ag = event_time(lambda: torch.distributed.all_gather_into_tensor(recv, send), 5, stream)
        out["comm"] = {"all_gather_ms": t_ag * 1e3, "bytes_per_rank_recv": int(recv.numel() * 4),
                       "algbw_GBps": recv.numel() * 4 / t_ag / 1e9}
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
