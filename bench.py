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
Edges counted per step = 4 * E of the graph (the four aggregations; the degree pass is
timed but not counted).  The dense layers and activations of the epoch are torch, not the
hot path, and are not part of the step.

The graph: ogbn-products shape (N=2,449,029 vertices, E=126,167,309 stored edges incl.
self loops), uniform random symmetric edges (seed 42), X ~ U[-1,1).  At N = 1 an R-MAT
graph of the same shape is timed as a second family (field "rmat"), and the SDDMM +
edge-softmax half of the path as one 8-head GAT layer of config 3 on the same graph,
forward + backward (field "gat", its own roofline and gather ceiling; at N > 1 the same
layer strong-scaled over the vertex cut).

N > 1 GPUs: STRONG scaling of that one graph (one process per GPU, RCCL over xGMI).
Every rank partitions the same graph (gala/dist.py, gala/vertex_cut.py) and the bench
times each candidate layout for a few steps, then runs the timed steps with the fastest:
    halo-exact     row partition, the halo gathered first, one SpMM (bit-exact vs 1 GPU)
    halo-overlap   row partition, own-column edges overlap the halo, halo edges after
    halo-pipe      row partition, the halo all-gathered in 4 row chunks, each chunk's
                   edges accumulated as it lands
    vcut / vcut-pipe  column ownership, partial rows reduce-scattered (1 / 4 chunks,
                   chunk k's reduce-scatter overlapping chunk k+1's SpMM)
The JSON line carries every candidate's step time and the per-aggregation halo bytes and
exchange time ("comm"), and the weak-scaling number of the earlier design (one
Products-sized synthetic partition per GPU) as the secondary field "weak".

Launch: `python bench.py --gpus N` starts N ranks itself (torch.distributed.run on
127.0.0.1) unless it already runs under a launcher (WORLD_SIZE set, which must equal N).
`--device cpu` runs the same code on the host-CPU backend with gloo (plumbing checks only).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

# the wall clock the N > 1 budget counts from: the launching process's start (a self-launch
# hands it to its ranks)
START = float(os.environ.get("GALA_BENCH_T0", "0")) or time.time()

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))

PRODUCTS_N = 2_449_029
PRODUCTS_E = 126_167_309          # 2 * 61,859,140 undirected + N self loops
HBM_PEAK = 8.0e12                 # MI355X HBM3E spec (MI355X_MICROARCH.md)
PIPE_CHUNKS = 4


def log(*a):
    print(f"[+{time.time() - START:.1f}s]", *a, file=sys.stderr, flush=True)


def start_heartbeat(rank: int, period_s: float = 60.0):
    """N > 1: rank 0 logs that it is alive every period_s (a phase of host-staged gloo
    collectives, or a slow rank, can run for minutes without a log line)."""
    import threading
    if rank != 0:
        return
    stop = threading.Event()

    def beat():
        while not stop.wait(period_s):
            log("[bench] alive")
    threading.Thread(target=beat, daemon=True).start()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n: int) -> int:
    """Start n ranks of this script under torch.distributed.run (before any GPU call in
    this process) and return their exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", str(max(1, min(16, (os.cpu_count() or 8) // n))))
    env["GALA_BENCH_T0"] = repr(START)
    log(f"[bench] launching {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def spmm_alg_bytes(n_rows, n_cols_read, nnz, F, out_rows=None):
    """SURVEY §8(d) unweighted SpMM: 4(N+1) + 4E + 4*N*F (X read once) + 4*N*F (Y write),
    + 4N for the fused dst norm."""
    out_rows = n_rows if out_rows is None else out_rows
    return 4 * (n_rows + 1) + 4 * nnz + 4 * n_cols_read * F + 4 * out_rows * F + 4 * n_rows


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """Threads for the CPU baselines: every core of the affinity mask, capped by a cgroup CPU
    quota and by OMP_NUM_THREADS when the pool sets one (the GPU box sets 16: its CPU share
    per GPU, while the affinity mask shows the whole machine)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    c = orc.usable_cores()
    omp = os.environ.get("OMP_NUM_THREADS")
    c["omp_num_threads_env"] = int(omp) if omp and omp.isdigit() else None
    if c["omp_num_threads_env"]:
        c["threads"] = min(c["threads"], c["omp_num_threads_env"])
    return c


def cpu_baseline(g, F: int, budget_s: float = 20.0):
    """Reference CPU aggregation on the host cores (rank 0, N=1 only): the reference's own
    gSpMM + wsumAgg (src/ops/aggregators.h:55-127) built -O3 -march=x86-64-v4 -fopenmp from
    /root/reference (oracle/build_ref.sh), or the oracle restatement when that library is
    absent.  Only the gSpMM call is timed: the value array (all ones, as readSM_npy32's
    set_all(1) leaves it) and Y are allocated and prefaulted before, and Y is re-zeroed
    outside the timed region (the generated code hands gSpMM a zero-filled output)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    cores = host_threads()
    n = cores["threads"]
    kind = "reference" if orc.ref_available() else "port"
    val = np.ones(g.nnz, np.float32)
    og = orc.Graph(g.n_rows, g.n_cols, g.rowptr, g.col, val)
    X = np.random.default_rng(1234).uniform(-1, 1, (g.n_cols, F)).astype(np.float32)
    Y = np.zeros((g.n_rows, F), np.float32)
    if kind == "reference":
        orc.ref_set_threads(n)
        fn = lambda: orc.ref_gspmm(og, X, Y)  # noqa: E731
    else:
        orc.set_threads(n)
        fn = lambda: orc.lib().orc_gspmm(orc._i64(og.n_rows), orc._ptr(og.rowptr), orc._ptr(og.col),  # noqa: E731
                                         orc._ptr(val), orc._ptr(X), orc._i32(F), orc._ptr(Y))
    fn()  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 5 and (time.perf_counter() - t_start) < budget_s:
        Y.fill(0.0)
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": g.nnz / t, "unit": "edges/s", "cores": n, "kind": kind, "cpu_model": cpu_model(),
            "host_cores": cores,
            "sample": f"{len(times)} full-graph F={F} SpMM calls (E={g.nnz}) after 1 warm-up, median "
                      f"{t:.3f} s, gSpMM call only (val and Y preallocated); " +
                      ("reference gSpMM+wsumAgg (src/ops/aggregators.h) compiled -O3 -march=x86-64-v4 -fopenmp "
                       "from /root/reference (oracle/_ref, shipped on purpose: north_star asks for the "
                       "reference CPU path timed in the same run)"
                       if kind == "reference" else "oracle restatement of gSpMM, OpenMP")}


def gat_cpu_baseline(hg, X, dY, aL, wR, bR, heads, budget_s: float = 12.0):
    """Host-CPU baseline of the SDDMM + edge-softmax half (rank 0, N = 1): the REF GAT layer,
    forward + backward, as the reference composes it pass by pass (K5 sddvv, LeakyReLU,
    exp/clamp, K7 row sum, reciprocal, K8 row scale, weighted K1 SpMM; backward SpMM on the
    forward alpha, K9 sddmm, softmax backward, LeakyReLU backward, K7), restated in C with
    OpenMP (oracle/gala_oracle.c orc_gat_ref_layer; the reference has no CPU code for these
    kernels, so kind "port").  Same graph and inputs as the GPU "gat" step, on a bounded
    sample: the first rows of the graph (all their edges, sources anywhere in X), sized so
    one call takes about budget_s / 3; value = 2 * sampled edges / median call time."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    cores = host_threads()
    orc.set_threads(cores["threads"])
    rp = hg.rowptr

    def rows_for(edges):
        return max(1, min(hg.n_rows, int(np.searchsorted(rp, edges))))
    k0 = rows_for(min(hg.nnz, 1 << 19))
    cal = orc.GatRefLayer(rp, hg.col, k0, X, dY, aL, wR, bR, heads)
    t0 = time.perf_counter()
    cal.run()                                    # warm-up + rate estimate
    rate = cal.nnz / max(time.perf_counter() - t0, 1e-6)
    del cal
    k = rows_for(int(rate * budget_s / 3))
    layer = orc.GatRefLayer(rp, hg.col, k, X, dY, aL, wR, bR, heads)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        layer.run()
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": 2 * layer.nnz / t, "unit": "edges/s", "cores": cores["threads"], "kind": "port",
            "cpu_model": cpu_model(), "host_cores": cores,
            "sample": f"rows [0, {k}) of the graph ({layer.nnz} edges, {layer.nnz / hg.nnz:.1%} of E), "
                      f"3 calls after a {k0}-row warm-up, median {t:.3f} s per forward + backward; "
                      "oracle orc_gat_ref_layer: the reference's GAT pass sequence restated, OpenMP"}


# the sources a kernel's machine code comes from (its .hip file, the shared headers, the ABI)
_KERNEL_SOURCES = (("k_gat_in_", "gat_input.hip"), ("k_gat_bwd_fused", "gat_fused.hip"), ("k_gat_", "gat.hip"),
                   ("k_spmm_", "spmm.hip"), ("k_rows", "spmm.hip"), ("k_degree", "spmm.hip"))
_COMMON_SOURCES = ("gala_internal.h", "edge_common.h", "gat_common.h")


def _sources_fresh(kernel: str, recorded: dict) -> bool:
    """Do the kernel's sources in this tree still have the digests its PMC pass recorded?"""
    import hashlib
    files = [f for key, f in _KERNEL_SOURCES if key in kernel][:1] + list(_COMMON_SOURCES)
    if not recorded or len(files) == len(_COMMON_SOURCES):
        return False
    for f in files:
        rel = os.path.join("gala-gnn-acceleration-language_amd", "csrc", f)
        try:
            now = hashlib.sha256(open(os.path.join(ROOT, rel), "rb").read()).hexdigest()
        except OSError:
            return False
        if recorded.get(rel) != now:
            return False
    return True


TRAFFIC_STALE = []   # kernels whose committed PMC bytes predate their current sources


def load_traffic(kernel_substr: str):
    """Per-launch HBM bytes of the dominant kernel from the committed PMC summary
    (profiles/traffic.json), or None when the kernel's sources changed since that PMC pass
    (the summary records their sha256): a stale byte count is never reported."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(path))
        for k, v in d.get("kernels", {}).items():
            # "banded|" / "rmat|" entries are another graph's launches of the same kernel
            if kernel_substr in k and ("|" in kernel_substr or "|" not in k):
                if not _sources_fresh(k, v.get("sources_sha256")):
                    TRAFFIC_STALE.append(kernel_substr)
                    return None
                return float(v["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def with_traffic_rate(roof: dict) -> dict:
    """north_star's "rocprof achieved HBM GB/s against the chip's peak": the PMC bytes per
    launch (roof["traffic"]) over this run's kernel time, and its fraction of the peak."""
    if roof.get("traffic"):
        rate = roof["traffic"] / (roof["kernel_ms"] / 1e3)
        roof["traffic_GBps"] = rate / 1e9
        roof["traffic_frac_of_peak"] = rate / HBM_PEAK
    return roof


class Timer:
    """HIP events on the current stream (device runs) or wall time (host runs)."""

    def __init__(self, cuda: bool):
        self.cuda = cuda

    def __call__(self, fn, reps):
        import numpy as np
        import torch
        if not self.cuda:
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            return (time.perf_counter() - t0) / reps
        # the kernels run on torch's current stream (gala.ops passes it to the C ABI).  One
        # untimed call is queued first, so the stream is busy when the first event is
        # recorded and the host's launch latency never shows as idle time between events
        stream = torch.cuda.current_stream()
        fn()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / 1e3 / reps


def gather_ceiling(col, X, timer, reps=10):
    """Time (HIP events, same stream) an unordered gather of the very rows the SpMM fetches:
    X[col[e]] for every edge e, any order, no row bookkeeping, no output rows
    (tools/gather_ceiling.hip -> tools/libgala_probe.so).  The floor for any kernel that
    fetches one X row per edge.  None when the probe library was not built."""
    import ctypes
    import torch
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
    args = (col.data_ptr(), X.data_ptr(), E, F, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    if fn(*args) != 0:
        return None
    return timer(lambda: fn(*args), reps)


def products_graph(kind: str, scale: float):
    from gala import layout
    n = max(int(PRODUCTS_N * scale), 2)
    E = n + 2 * ((int(PRODUCTS_E * scale) - n) // 2)
    return layout.gen_graph(kind, n, (E - n) // 2, seed=42)


def data_dir(args):
    """The real dataset to run on: --data DIR, else Data/Products/ next to this script (the
    reference's layout, scripts/Data/gala_export_npy.py:100-112) when it holds the graph."""
    if args.data:
        return args.data
    d = os.path.join(ROOT, "Data", "Products")
    return d if os.path.exists(os.path.join(d, "Adj_src.npy")) else None


def headline_graph(args):
    """(graph, data description): the npy dataset when one is given / present, else the
    synthetic uniform Products-shaped graph."""
    d = data_dir(args)
    if d is None:
        return products_graph("uniform", args.scale), None
    from gala import layout
    if d.endswith(".mtx"):    # a Matrix Market graph, as the reference's readSM reads it
        g = layout.load_mtx(d)
        g.val = None           # the GCN step aggregates the pattern (values 1, like readSM_npy32)
        desc = (f"real: {os.path.abspath(d)} (Matrix Market, readSM / MtxIO semantics: 1-based, "
                f"symmetric files mirrored; the pattern aggregated); X~U[-1,1) fp32")
    else:
        g = layout.load_npy_dataset(d)
        desc = (f"real: {os.path.abspath(d)} (Adj_src/Adj_dst.npy, gala_export_npy.py format: CSR rows = src, "
                f"values 1); X~U[-1,1) fp32")
    if g.n_rows != g.n_cols:
        raise SystemExit(f"bench.py: {d} holds a {g.n_rows} x {g.n_cols} graph; the aggregation needs it square")
    return g, desc


class OneGpuGCN:
    """The single-device step: norm * A (norm * H) with the dst norm fused into the SpMM."""

    def __init__(self, hg, F, be):
        self.be, self.F = be, F
        self.g = be.graph(hg)
        self.norm = be.degree(self.g)
        self.Xs = be.empty(hg.n_cols, F)
        self.Xs2 = None
        self.n = hg.n_rows
        self.nnz = hg.nnz

    def refresh_norm(self):
        self.norm = self.be.degree(self.g)          # recomputed every forward (gala.cu:433-440)

    def __call__(self, H, out):
        self.be.row_broadcast(self.norm, H, self.Xs)
        return self.be.spmm(self.g, self.Xs, out, self.norm, False)


def make_step(agg, X, dY, bufs):
    H1, H2, G1, G0 = bufs

    def step():
        agg.refresh_norm()
        agg(X, H1)
        agg(H1, H2)
        agg(dY, G1)
        agg(G1, G0)
    return step


def make_fused_step(agg, X, dY, bufs):
    """The same step with the degree pass and the ROW_BROADCASTs folded (gala_spmm_ex_f32,
    gala_row_broadcast_deg_f32): the input's `norm * X` pass forms the norm from the rowptr,
    each SpMM forms its dst norm the same way, and the first aggregation of each direction
    also writes the second one's pre-scaled input, norm * H (codegen/gala.cu:433-456: the
    degree, two forward and two backward aggregations).  Outputs bit-identical to make_step."""
    H1, H2, G1, G0 = bufs
    be, g, Xs = agg.be, agg.g, agg.Xs
    if agg.Xs2 is None:
        agg.Xs2 = be.empty(agg.n, agg.F)
    Xs2 = agg.Xs2

    def step():
        be.row_broadcast_deg(g, X, Xs)
        be.spmm_deg(g, Xs, H1, out2=Xs2)
        be.spmm_deg(g, Xs2, H2)
        be.row_broadcast_deg(g, dY, Xs)
        be.spmm_deg(g, Xs, G1, out2=Xs2)
        be.spmm_deg(g, Xs2, G0)
    return step


def timed_steps(step, steps, warmup, sync, barrier, reduce_max):
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    w0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    sync()
    return reduce_max(time.perf_counter() - w0) / steps


# ---- strong-scaling candidates ---------------------------------------------------------------
class HaloMode:
    def __init__(self, name, part, F, be, comm, exact):
        from gala import dist as gdist
        self.name, self.part = name, part
        self.agg = gdist.DistAggregator(part, F, be, comm, exact=exact)
        self.be, self.comm, self.F = be, comm, F

    def kernel(self, timer):
        """(seconds, algorithmic bytes) of the rank's SpMM over all its edges."""
        a, p = self.agg, self.part
        Y = self.be.empty(p.n, self.F)
        t = timer(lambda: self.be.spmm(a.graph, a.Xs, Y, a.norm, False), 10)
        return t, spmm_alg_bytes(p.n, p.n + p.n_halo_rows, p.graph.nnz, self.F)

    def exchange(self, timer):
        a = self.agg
        if a.exchange is None:
            return 0.0
        return timer(lambda: [self.comm.wait(w) for w in a.exchange.start(a.Xs)], 5)


class VcutMode:
    def __init__(self, name, part, F, be, comm):
        from gala import vertex_cut as vc
        self.name, self.part = name, part
        self.agg = vc.VertexCutAggregator(part, F, be, comm)
        self.be, self.comm, self.F = be, comm, F

    def kernel(self, timer):
        """(seconds, algorithmic bytes) of the rank's partial-row SpMMs (every chunk)."""
        p = self.part
        t = timer(lambda: self.agg.local_spmm(), 10)
        rows = p.partial_rows()
        alg = 4 * (rows + p.chunks) + 4 * p.chunk_nnz() + 4 * p.n * self.F + 4 * rows * self.F
        return t, alg

    def exchange(self, timer):
        return timer(lambda: self.agg.exchange_only(), 5)


def _recoverable(e: Exception) -> bool:
    """Whether bench.py may go on after `e`: a Python-level failure of one layout yes; a GPU
    runtime error (a fault leaves the device unusable) or an RCCL error never."""
    text = repr(e)
    return not any(k in text for k in ("HIP", "hip", "CUDA", "cuda", "NCCL", "nccl", "RCCL"))


class Budget:
    """The N > 1 run's wall-clock budget (--budget-s from the process start), so the driver's
    run always gets its headline line.  Every decision is agreed over the ranks (one MAX
    all-reduce of "out of time"): a rank that skips a phase its peers run would leave them
    waiting in a collective.  `phases` holds each phase's wall seconds, `skipped` what was left
    out and why."""

    def __init__(self, limit_s: float, reduce_max=None):
        self.t0 = START
        self.limit = float(limit_s)
        self.reduce_max = reduce_max
        self.phases, self.skipped = {}, []

    def elapsed(self) -> float:
        return time.time() - self.t0

    def ok(self, need_s: float, what: str) -> bool:
        """Whether `what`, estimated at need_s seconds, still fits (the same answer on every rank)."""
        over = 1.0 if self.elapsed() + need_s > self.limit else 0.0
        if self.reduce_max is not None:
            over = self.reduce_max(over)
        if over > 0:
            self.skipped.append(f"{what} (needs ~{need_s:.0f} s, {self.elapsed():.0f} of {self.limit:.0f} s used)")
            log(f"[bench] budget: skipping {what}")
        return over == 0

    def note(self):
        return {"budget_s": self.limit, "elapsed_s": round(self.elapsed(), 1),
                "phase_s": {k: round(v, 1) for k, v in self.phases.items()}, "skipped_for_time": self.skipped}


def strong_family(args, kind, rank, world, dev, be, comm, timer, sync, barrier, reduce_max, budget=None):
    """Strong scaling of one Products-shaped graph of family `kind` over the ranks: every
    candidate layout timed for a few steps, the timed steps on the fastest.  Returns
    (result fields, graph, bounds)."""
    import torch
    from gala import dist as gdist, vertex_cut as vc
    F = args.F
    t0 = time.time()
    g, real = headline_graph(args) if kind == "uniform" else (products_graph(kind, args.scale), None)
    log(f"[rank {rank}/{world}] {kind} graph N={g.n_rows} E={g.nnz} built in {time.time() - t0:.1f}s")
    bounds = gdist.row_bounds(g.rowptr, world)
    t0 = time.time()
    # candidates are built when they are timed (a candidate the budget skips costs nothing)
    pt1 = gdist.partition_graph(g, rank, world, bounds=bounds)
    modes = [("halo-exact", lambda: HaloMode("halo-exact", pt1, F, be, comm, exact=True)),
             ("halo-overlap", lambda: HaloMode("halo-overlap", pt1, F, be, comm, exact=False))]
    if pt1.halo_mode == "dense":
        # finer chunks leave less of the first chunk's transfer and the last chunk's SpMM
        # outside the overlap, at more (smaller) collectives: both are timed
        for ck, nm in ((PIPE_CHUNKS, "halo-pipe"), (2 * PIPE_CHUNKS, f"halo-pipe{2 * PIPE_CHUNKS}")):
            modes.append((nm, lambda ck=ck, nm=nm: HaloMode(nm, gdist.partition_graph(
                g, rank, world, bounds=bounds, halo_mode="dense", chunks=ck), F, be, comm, exact=False)))
    modes.append(("vcut", lambda: VcutMode("vcut", vc.vertex_cut_partition(g, rank, world, 1, bounds), F, be, comm)))
    modes.append(("vcut-pipe", lambda: VcutMode("vcut-pipe", vc.vertex_cut_partition(g, rank, world, PIPE_CHUNKS,
                                                                                    bounds), F, be, comm)))
    frac = vc.touched_fraction(g, bounds) if world > 1 else 0.0
    if frac < 0.9:      # the DCSR exchange can only win when some partial rows are empty
        modes.append(("vcut-sparse", lambda: VcutMode("vcut-sparse", vc.vertex_cut_partition(
            g, rank, world, 1, bounds, "sparse"), F, be, comm)))
        modes.append(("vcut-sparse-pipe", lambda: VcutMode("vcut-sparse-pipe", vc.vertex_cut_partition(
            g, rank, world, PIPE_CHUNKS, bounds, "sparse"), F, be, comm)))
    log(f"[rank {rank}] {kind} candidates {[m[0] for m in modes]}, halo {pt1.halo_mode}, "
        f"{pt1.n_halo_rows} halo rows, touched fraction {frac:.3f}; row partition in {time.time() - t0:.1f}s")
    n, r0 = pt1.n, pt1.r0
    gen = torch.Generator(device=dev).manual_seed(1234)
    # every rank draws the whole X so row r is the same on any number of ranks
    Xall = torch.rand((g.n_rows, F), device=dev, generator=gen) * 2 - 1
    X = Xall[r0:r0 + n].clone()
    dY = (torch.rand((g.n_rows, F), device=dev, generator=gen) * 2 - 1)[r0:r0 + n].clone()
    del Xall
    bufs = [be.empty(n, F) for _ in range(4)]
    cand, failed, best, longest = {}, {}, None, 0.0
    forced = os.environ.get("GALA_DIST_MODE")
    for name, make in modes:
        # after the first candidate, one more is timed only while the budget holds (the
        # estimate: the slowest candidate so far, build included)
        if cand and budget is not None and not budget.ok(longest, f"{kind} candidate {name}"):
            continue
        # a layout that raises (on every rank alike: the same code on the same graph) is
        # skipped and reported; the others are still timed
        tc = time.time()
        try:
            m = make()
            st = make_step(m.agg, X, dY, bufs)
            cand[name] = timed_steps(st, args.calib_steps, 2, sync, barrier, reduce_max)
            log(f"[rank {rank}] {kind} candidate {name}: {cand[name] * 1e3:.3f} ms/step")
            keep = name == forced or (forced not in dict(modes) and (best is None or cand[name] < cand[best.name]))
            if keep:
                best = m
            del m, st
        except Exception as e:  # noqa: BLE001
            if not _recoverable(e):
                raise
            failed[name] = repr(e)[:300]
            log(f"[rank {rank}] {kind} candidate {name} failed: {failed[name]}")
        longest = max(longest, time.time() - tc)
    if best is None:
        raise RuntimeError(f"bench.py: every {kind} layout failed: {failed}")
    name = best.name
    t_step = timed_steps(make_step(best.agg, X, dY, bufs), args.steps if kind == "uniform" else max(args.steps // 2, 2),
                         args.warmup if kind == "uniform" else 2, sync, barrier, reduce_max)
    t_kernel, alg = best.kernel(timer)
    t_ex = best.exchange(timer) if world > 1 else 0.0
    out = {"value": 4 * g.nnz / t_step, "ms_per_step": t_step * 1e3, "real_data": real,
           "roofline": {"bound": "hbm", "achieved": alg / t_kernel / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                        "frac": alg / t_kernel / HBM_PEAK, "traffic": None,
                        "kernel": f"gala::k_spmm_rowgroup (rank 0's SpMM launches of mode {best.name})",
                        "kernel_ms": t_kernel * 1e3, "alg_bytes_per_launch": alg},
           "comm": {"mode": best.name, "backend": dist_backend(),
                    "candidates_ms_per_step": {k: v * 1e3 for k, v in cand.items()},
                    "halo_bytes_per_aggregation_per_rank": best.agg.halo_bytes(),
                    "exchange_ms_per_aggregation": t_ex * 1e3,
                    # the link rate the exchange achieved: this rank's exchanged bytes over the
                    # time of one aggregation's collectives alone (xGMI under RCCL)
                    "exchange_GBps_per_rank": (best.agg.halo_bytes() / t_ex / 1e9) if t_ex > 0 else None,
                    "spmm_ms_per_aggregation": t_kernel * 1e3,
                    "halo_layout": pt1.halo_mode, "halo_rows_rank0": pt1.n_halo_rows,
                    "vcut_touched_fraction": frac,
                    "failed_candidates": failed,
                    "note": "halo-exact is bit-identical to one GPU; the other modes agree to fp32 rounding. "
                            "Exchange time is the collective(s) of one aggregation alone; it overlaps the SpMM "
                            "in the -overlap/-pipe modes. vcut-sparse: DCSR partial rows (only rows with a held "
                            "edge) sent by all-to-all, timed when the touched fraction is below 0.9."}}
    if comm.rccl:
        out["comm"]["rccl_note"] = "RCCL collectives over the node's GPUs"
    else:
        out["comm"]["rccl_note"] = f"{dist_backend()} rehearsal: host-staged collectives, not RCCL over xGMI"
    del modes, best, bufs, X, dY
    return out, g, bounds


def dist_backend():
    import torch.distributed as dist
    return dist.get_backend()


def run_multi(args, rank, world, dev, be, timer, sync):
    import torch
    import torch.distributed as dist
    from gala.comm import Comm

    comm = Comm()
    F = args.F

    def barrier():
        dist.barrier()

    def reduce_max(x):
        t = torch.tensor([x], dtype=torch.float64, device=dev if be.name == "hip" and comm.rccl else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    budget = Budget(args.budget_s, reduce_max)
    start_heartbeat(rank)
    t0 = time.time()
    fam, g, bounds = strong_family(args, "uniform", rank, world, dev, be, comm, timer, sync, barrier, reduce_max,
                                   budget)
    budget.phases["uniform"] = t_uniform = time.time() - t0
    out = {
        "metric": "aggregated edges/sec, GCN-2 ogbn-products (4 F=32 aggregations per step)",
        "value": fam["value"],
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": fam["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": fam.pop("real_data") or ("synthetic: one uniform random symmetric ogbn-products-shaped graph + self "
                                         "loops (seed 42), partitioned across the ranks; X~U[-1,1) fp32"),
        "config": {"workload": "GCN-2 ogbn-products-shaped hot path: degree + 2 fwd + 2 bwd norm-scaled "
                               "SpMM aggregations, F=32, one graph split over the GPUs",
                   "n_vertices": g.n_rows, "edges": g.nnz, "F": F,
                   "parallelism": f"{fam['comm']['mode']} x{world} (RCCL)" if comm.rccl
                   else f"{fam['comm']['mode']} x{world} ({dist.get_backend()})"},
        "roofline": fam["roofline"],
        "comm": fam["comm"],
    }
    # secondary fields, each only while the budget holds; estimates from the uniform family's
    # own wall time (a family of the same shape: graph, partitions, candidates)
    if not args.no_gat and budget.ok(t_uniform, "gat field"):
        t0 = time.time()
        try:
            out["gat"] = gat_multi(args, g, rank, world, dev, be, comm, bounds, sync, barrier, reduce_max, budget)
        except Exception as e:  # noqa: BLE001  (reported; the headline line stays)
            if not _recoverable(e):
                raise
            out["gat"] = {"error": repr(e)[:500]}
        budget.phases["gat"] = time.time() - t0
    del g
    for kind in ("rmat", "banded"):   # the skewed family, and one that shards naturally
        if getattr(args, f"no_{kind}") or not budget.ok(1.2 * t_uniform, f"{kind} family"):
            continue
        t0 = time.time()
        try:    # a secondary family that fails on every rank is reported; the headline line stays
            rm, gr, _ = strong_family(args, kind, rank, world, dev, be, comm, timer, sync, barrier, reduce_max,
                                      budget)
        except Exception as e:  # noqa: BLE001
            if not _recoverable(e):
                raise
            out[kind] = {"error": repr(e)[:500]}
            continue
        finally:
            budget.phases[kind] = time.time() - t0
        rm.pop("real_data")
        rm["graph"] = (f"{FAMILY_GRAPH[kind]}, N={gr.n_rows}, E={gr.nnz}, "
                       f"max degree {int((gr.rowptr[1:] - gr.rowptr[:-1]).max())}")
        rm["unit"] = "edges/s"
        out[kind] = rm
        del gr
    if not args.no_weak and budget.ok(0.5 * t_uniform, "weak field"):
        t0 = time.time()
        try:
            out["weak"] = weak_scaling(args, rank, world, dev, be, comm, sync, barrier, reduce_max)
        except Exception as e:  # noqa: BLE001
            if not _recoverable(e):
                raise
            out["weak"] = {"error": repr(e)[:500]}
        budget.phases["weak"] = time.time() - t0
    out["budget"] = budget.note()
    # the largest message each collective kind sent (max over ranks) and its rounds: whether
    # the all-to-all / p2p cut at MAX_MSG_BYTES held (RCCL corrupts payloads past 1 GiB, gala/comm.py)
    from gala.comm import message_stats
    out["comm"]["messages"] = message_stats(reduce_max)
    return out


def gat_multi(args, g, rank, world, dev, be, comm, bounds, sync, barrier, reduce_max, budget=None):
    """The "gat" field at N > 1: the same 8-head GAT layer as at N = 1 (forward + backward,
    REF, the source logit formed from X), strong-scaled over the one graph.  The layouts are
    timed for a few steps and the faster runs the timed steps:
      halo   the row partition gathers the X rows its edges read (then the source logits,
             and dY in the backward) and runs the one-GPU statistics kernels over its rows
             (gala/dist.py HaloGat): bit-identical to one GPU, F + H (forward) and F
             (backward) floats per halo row;
      halo-overlap  the same exchange, the own-column edges' partial statistics run while
             it is in flight and the halo columns continue them after it (gala/dist.py
             HaloGatOverlap; fp32 rounding of one GPU, each row's sums grouped per range);
      halo-overlap-pipe  (dense halo, N > 1) the table all-gathered in PIPE_CHUNKS row
             chunks, each chunk's edges continued as it lands;
      vcut   north_star's vertex cut (gala/vertex_cut.py VertexCutGat): the row-statistics
             forward and the backward's partial aggregation over the edges whose source a
             rank owns, 2F + 2H (forward) and F (backward) partial floats per row
             reduce-scattered to the owners, in 4 overlapped row blocks."""
    import torch
    from gala import dist as gdist, vertex_cut as vc
    H, F = GAT_HEADS, GAT_HEADS * GAT_HEAD_F
    gen = torch.Generator(device=dev).manual_seed(4321 + rank)
    r0, n = int(bounds[rank]), int(bounds[rank + 1] - bounds[rank])
    aL = torch.rand((n, H), device=dev, generator=gen) - 0.5
    wR = (torch.rand(F, device=dev, generator=gen) - 0.5) * 0.2
    bR = torch.zeros(H, device=dev)
    hpart = gdist.partition_graph(g, rank, world, bounds=bounds)
    halo = gdist.HaloGat(hpart, F, H, be, comm)
    X = halo.own_rows("X")              # the layer input, written into the table
    X.copy_(torch.rand((n, F), device=dev, generator=gen) * 2 - 1)
    dY = halo.own_rows("dY")
    dY.copy_(torch.rand((n, F), device=dev, generator=gen) * 2 - 1)
    comm_bytes = {"halo": hpart.halo_bytes(2 * F + H) if world > 1 else 0}
    comm_bytes["halo-overlap"] = comm_bytes["halo"]

    def pipe_layer():       # the all-gather in row chunks, pipelined
        ppart = gdist.partition_graph(g, rank, world, bounds=bounds, halo_mode="dense", chunks=PIPE_CHUNKS)
        comm_bytes["halo-overlap-pipe"] = ppart.halo_bytes(2 * F + H)
        return gdist.HaloGatOverlap(ppart, F, H, be, comm)

    def vcut_layer():
        vpart = vc.vertex_cut_partition(g, rank, world, PIPE_CHUNKS, bounds)
        comm_bytes["vcut"] = vpart.comm_bytes(2 * F + 2 * H) + vpart.comm_bytes(F)
        return vc.VertexCutGat(vpart, F, H, be, comm)

    # candidates are built when they are timed; after the first, one more is timed only while
    # the budget holds (the estimate: the slowest candidate so far, build included)
    makers = [("halo", lambda: halo), ("halo-overlap", lambda: gdist.HaloGatOverlap(hpart, F, H, be, comm))]
    if world > 1 and hpart.halo_mode == "dense":
        makers.append(("halo-overlap-pipe", pipe_layer))
    makers.append(("vcut", vcut_layer))

    def step_of(layer):
        def step():
            layer.forward_train(aL, None, X, wR, bR)   # source logits recomputed from X, as at N = 1
            layer.backward(dY, linear=False)           # the aggregation's backward, as gala_gat_bwd_stats_f32
        return step
    cand, kept, longest = {}, {}, 0.0
    for name, make in makers:
        if cand and budget is not None and not budget.ok(longest, f"gat candidate {name}"):
            continue
        tc = time.time()
        layer = make()
        cand[name] = timed_steps(step_of(layer), args.calib_steps, 2, sync, barrier, reduce_max)
        log(f"[rank {rank}] gat candidate {name}: {cand[name] * 1e3:.3f} ms/step")
        if cand[name] == min(cand.values()):
            kept = {name: layer}
        del layer
        longest = max(longest, time.time() - tc)
    best = min(cand, key=cand.get)
    steps = max(args.steps // 2, 2)
    t_step = timed_steps(step_of(kept[best]), steps, 2, sync, barrier, reduce_max)
    desc = {"halo": "row partition, gathered X / logits / dY rows, the one-GPU kernels (bit-identical)",
            "halo-overlap": "row partition, gathered X / logits / dY rows; own-column partial statistics "
                            "overlap the exchange (fp32 rounding of one GPU)",
            "halo-overlap-pipe": f"row partition, the X / dY table all-gathered in {PIPE_CHUNKS} row chunks, each "
                                 f"chunk's edges continued as it lands (fp32 rounding of one GPU)",
            "vcut": f"vertex cut, row-statistics partials reduce-scattered to the row owners in {PIPE_CHUNKS} "
                    f"overlapped row blocks"}
    out = {"value": 2 * g.nnz / t_step, "unit": "edges/s", "ms_per_step": t_step * 1e3, "steps": steps,
           "layer": f"GAT {H} heads x {GAT_HEAD_F} (F={F}), REF softmax; forward + backward",
           "layout": f"{best} x{world}: " + desc[best],
           "candidates_ms_per_step": {k: v * 1e3 for k, v in cand.items()},
           "comm_bytes_per_step_per_rank": comm_bytes[best],
           "comm_bytes_per_step_per_rank_candidates": comm_bytes}
    del kept, halo, X, dY
    return out


def weak_scaling(args, rank, world, dev, be, comm, sync, barrier, reduce_max):
    """The secondary number: one ogbn-products-sized synthetic partition per GPU, 10% of its
    edges cut edges to other partitions' boundary rows (all-gathered, overlapped)."""
    import torch
    from gala import dist as gdist
    F = args.F
    n = max(int(PRODUCTS_N * args.scale), 2)
    E = n + 2 * ((int(PRODUCTS_E * args.scale) - n) // 2)
    part = gdist.make_partition(rank, world, n, E, cut_frac=0.1, boundary_frac=0.1, seed=42)
    agg = gdist.DistGCNAggregator(part, F, be, comm)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    X = torch.rand((n, F), device=dev, generator=gen) * 2 - 1
    dY = torch.rand((n, F), device=dev, generator=gen) * 2 - 1
    bufs = [be.empty(n, F) for _ in range(4)]
    t = timed_steps(make_step(agg, X, dY, bufs), max(args.steps // 2, 2), 2, sync, barrier, reduce_max)
    return {"value": world * 4 * part.graph.nnz / t, "ms_per_step": t * 1e3, "edges_per_gpu": part.graph.nnz,
            "cut_edges_per_gpu": part.n_cut_edges, "halo_bytes_per_aggregation_per_rank": agg.halo_bytes(),
            "note": "weak scaling: every GPU owns its own Products-sized synthetic partition"}


def run_single(args, dev, be, timer, sync):
    import torch
    F = args.F
    t0 = time.time()
    hg, real = headline_graph(args)
    log(f"[bench] uniform graph N={hg.n_rows} E={hg.nnz} in {time.time() - t0:.1f}s")
    agg = OneGpuGCN(hg, F, be)
    gen = torch.Generator(device=dev).manual_seed(1234)
    X = torch.rand((hg.n_rows, F), device=dev, generator=gen) * 2 - 1
    dY = torch.rand((hg.n_rows, F), device=dev, generator=gen) * 2 - 1
    bufs = [be.empty(hg.n_rows, F) for _ in range(4)]
    ident = lambda x: x  # noqa: E731
    # the fused step's outputs against the unfused chain's, once, outside the timed region
    make_step(agg, X, dY, bufs)()
    want = [b.clone() for b in bufs]
    make_fused_step(agg, X, dY, bufs)()
    fused_same = all(bool(torch.equal(a, b)) for a, b in zip(want, bufs))
    del want
    if not fused_same:
        raise RuntimeError("bench.py: the fused step's outputs differ from the degree + ROW_BROADCAST + SpMM chain")
    t_step = timed_steps(make_fused_step(agg, X, dY, bufs), args.steps, args.warmup, sync, lambda: None, ident)
    value = 4 * hg.nnz / t_step
    Y = bufs[0]
    # the kernel and (HIP) the same-process gather probe, interleaved over three rounds
    # (medians; both move with the GPU's load state)
    k_rounds, c_rounds = [], []
    for _ in range(3):
        k_rounds.append(timer(lambda: be.spmm(agg.g, agg.Xs, Y, agg.norm, False), 10))
        t_c = gather_ceiling(agg.g.col, agg.Xs, timer) if be.name == "hip" else None
        if t_c:
            c_rounds.append(t_c)
    t_kernel = sorted(k_rounds)[1]
    alg = spmm_alg_bytes(hg.n_rows, hg.n_rows, hg.nnz, F)
    achieved = alg / t_kernel
    gather_bytes = 4 * (hg.n_rows + 1) + hg.nnz * (4 + 4 * F) + 4 * hg.n_rows * F
    out = {
        "metric": "aggregated edges/sec, GCN-2 ogbn-products (4 F=32 aggregations per step)",
        "value": value,
        "unit": "edges/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_step * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": real or "synthetic: uniform random symmetric ogbn-products-shaped graph + self loops (seed 42), "
                        "X~U[-1,1) fp32",
        "config": {"workload": "GCN-2 ogbn-products-shaped hot path: degree + 2 fwd + 2 bwd norm-scaled "
                               "SpMM aggregations, F=32",
                   "step": "degree norm and the next aggregation's ROW_BROADCAST folded into the SpMM "
                           "epilogues (gala_spmm_ex_f32 / gala_row_broadcast_deg_f32); outputs checked "
                           "bit-identical to the unfused chain in this run",
                   "fused_step_bit_identical": fused_same,
                   "n_vertices": hg.n_rows, "edges": hg.nnz, "F": F, "parallelism": "1 GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK,
                     "traffic": load_traffic("k_spmm_rowgroup<4, 8, 1, 4, false, false, false, false>") if be.name == "hip" else None,
                     "kernel": "gala::k_spmm_rowgroup<VEC=4,G=8,CH=1,U=4,unweighted> (gala_spmm_f32, F=32, dst norm)",
                     "kernel_ms": t_kernel * 1e3, "alg_bytes_per_launch": alg,
                     "gather_model_GBps": gather_bytes / t_kernel / 1e9,
                     "traffic_note": "PMC FETCH_SIZE*2+WRITE_SIZE per launch (profiles/traffic.json, null when the kernel's "
                                     "sources changed since that pass); "
                                     "uniform random columns: each edge's 128-B X row misses L2"},
    }
    with_traffic_rate(out["roofline"])
    if c_rounds:
        t_ceil = sorted(c_rounds)[len(c_rounds) // 2]
        if t_ceil:
            out["roofline"]["gather_ceiling_ms"] = t_ceil * 1e3
            out["roofline"]["frac_of_gather_ceiling"] = sorted(c / k for c, k in zip(c_rounds, k_rounds))[len(c_rounds) // 2]
            out["roofline"]["gather_ceiling_note"] = (
                "same process and graph: X[col[e]] for every edge, unordered, no output rows "
                "(tools/gather_ceiling.hip); the SpMM's floor on a graph without reuse")
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(hg, F)
        except Exception as e:  # the baseline is reported, never the target
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    del X, dY, bufs
    if be.name == "hip" and not args.no_gat:
        out["gat"] = gat_layer(args, agg.g, hg, dev, timer, sync)
    del agg
    if not args.no_rmat:
        out["rmat"] = rmat_family(args, dev, be, timer, sync, "rmat")
    # the banded graph's SpMM is the headline kernel (same name) on another graph: at N = 1
    # only on request, so a rocprof run of the default command averages the headline graph's
    # launches alone (profiles/r03_bench_n1_banded.json holds its N = 1 line)
    if args.banded and not args.no_banded:
        out["banded"] = rmat_family(args, dev, be, timer, sync, "banded")
    return out


GAT_HEADS, GAT_HEAD_F = 8, 32   # BASELINE configs[2]: ogbn-products GAT, 8 heads x 32 (galac gat_heads(8))
GAT_IN_F = 100                  # ogbn-products node features (bench/dsl/gat_products_h8.txt feature_size)


def gat_layer(args, dg, hg, dev, timer, sync):
    """SDDMM + edge-softmax + aggregation throughput on the same graph: config 3's first GAT
    layer (bench/dsl/gat_products_h8.txt: 100 input features -> 8 heads x 32), forward +
    backward, from the 100-d input with the Linear included, as the generated program runs it
    (galac emits gala::gat_input_layer_apply for it):
        forward   the attention vectors folded through the Linear (uL, uR), the extended input
                  rows (gala_gat_in_prep_f32), then gala_gat_in_fwd_f32: per edge p =
                  exp(LeakyReLU(aL[r] + aR[c])) and the 512-B extended row of c into the
                  per-head input-space aggregates (matrix cores), projected per row by the
                  Linear into Y and Ym, with q = 1/(1e-12 + sum p) and sum m*alpha
                  -- in T mode (gala_gat_in_fwd_t_f32, the mirror's default on a symmetric
                  graph): a pass summing q for every row first, then the same walk also forms
                  the backward's per-column aggregates T_h[c] = sum alpha X_ext[r] (r in N(c))
                  from the rows it gathers anyway
        backward  gala_gat_in_bwd_t_f32: M_h += dY_h[c]^T T_h[c], d_aL from <dY, Y>, <dY, Ym>
                  (no walk over the graph); then G = d_aL^T X (gala_dense_grad_f32) and the
                  parameter gradients of W, b and both attention Linears.  `walk` times the
                  previous backward beside it: gala_gat_in_bwd_f32 gathering the extended rows
                  again over the transposed pattern
    (the reference's FFN_OP + attention Linears + the edge chains of cuda.h:505-562,679-845 and
    common.h:622-894, fused and regrouped in input space; tests/test_gpu_gat_input.py checks it
    against the oracle's pass-by-pass chain at this size).  `gathering_linear_output` times the
    previous formulation beside it: the Linear's 1-KB output rows gathered by the row-statistics
    pair (gala_gat_{fwd,bwd}_stats_f32).  value counts 2*E edges per step (the forward's and the
    backward's pass over every edge)."""
    import torch
    from gala import ops
    H, D = GAT_HEADS, GAT_HEAD_F
    F, FIN = H * D, GAT_IN_F
    N, E = hg.n_rows, hg.nnz
    gen = torch.Generator(device=dev).manual_seed(4321)
    Xin = torch.rand((N, FIN), device=dev, generator=gen) * 2 - 1
    dY = torch.rand((N, F), device=dev, generator=gen) * 2 - 1
    W = (torch.rand((F, FIN), device=dev, generator=gen) * 2 - 1) / 10
    b = (torch.rand(F, device=dev, generator=gen) - 0.5) * 0.2
    wL, wR = ((torch.rand(F, device=dev, generator=gen) - 0.5) * 0.6 for _ in range(2))
    bL, bR = ((torch.rand(H, device=dev, generator=gen) - 0.5) * 0.2 for _ in range(2))
    order = torch.from_numpy(ops.degree_order(hg.rowptr)).to(dev)   # the mirror's phase order
    st = {}

    def fwd():
        st["f"] = ops.gat_input_layer(dg, Xin, W, b, wL, bL, wR, bR, H, order=order, relu=True, tmode=True)

    def bwd():
        f = st["f"]
        daL, M = ops.gat_in_bwd(dg, f["xext"], dY, f["Y"], f["Ym"], f["sma"], H, FIN, order=order, relu=True,
                                T=f["T"])
        Gw, Gb = ops.dense_grad(Xin, daL)
        sLR = (wL + wR).reshape(H, D)
        dW = M[:, :, :FIN] + sLR.unsqueeze(2) * Gw.unsqueeze(1)
        db = M[:, :, FIN] + sLR * Gb.unsqueeze(1)
        dw = (W.reshape(H, D, FIN) * Gw.unsqueeze(1)).sum(2) + b.reshape(H, D) * Gb.unsqueeze(1)
        st["b"] = (dW, db, dw, Gb)

    def step():
        fwd()
        bwd()
    steps = max(args.steps // 2, 2)
    t_step = timed_steps(step, steps, 2, sync, lambda: None, lambda x: x)
    f0 = st["f"]
    xext, Y0, Ym0, sma0, T0 = f0["xext"], f0["Y"], f0["Ym"], f0["sma"], f0["T"]

    def k_fwd():   # the aggregation call alone (its extended rows prepared): q pass + T-mode walk
        ops.gat_in_fwd(dg, xext, W, b, H, FIN, order=order, relu=True, T=T0)

    def k_bwd():
        ops.gat_in_bwd(dg, xext, dY, Y0, Ym0, sma0, H, FIN, order=order, relu=True, T=T0)

    def k_fwd_walk():   # the walk formulation: forward without T, backward gathering again
        ops.gat_in_fwd(dg, xext, W, b, H, FIN, order=order, relu=True)

    def k_bwd_walk():
        ops.gat_in_bwd(dg, xext, dY, Y0, Ym0, sma0, H, FIN, order=order, relu=True)
    # the layer, its kernels (both formulations) and the same-process gather probe of the
    # 512-B extended rows, interleaved over three rounds (medians: all move by up to 10 % with
    # the GPU's load state).  The walk's forward writes q into the extended rows
    # as the T-mode q pass does (the same values), so the two share the rows.
    rounds = {"fwd": [], "bwd": [], "k_fwd": [], "k_bwd": [], "k_fwd_walk": [], "k_bwd_walk": [], "ceil": []}
    for _ in range(3):
        rounds["fwd"].append(timer(fwd, 5))
        rounds["bwd"].append(timer(bwd, 5))
        rounds["k_fwd"].append(timer(k_fwd, 5))
        rounds["k_bwd"].append(timer(k_bwd, 5))
        rounds["k_fwd_walk"].append(timer(k_fwd_walk, 5))
        rounds["k_bwd_walk"].append(timer(k_bwd_walk, 5))
        k_fwd()   # the T tiles and q of the T-mode forward back in place for the next round
        t_c = gather_ceiling(dg.col, xext, timer, reps=5)
        if t_c:
            rounds["ceil"].append(t_c)
    med = lambda xs: sorted(xs)[len(xs) // 2] if xs else None  # noqa: E731
    t_fwd, t_bwd, t_kf, t_kb = (med(rounds[k]) for k in ("fwd", "bwd", "k_fwd", "k_bwd"))
    # algorithmic bytes per call, SURVEY §8(d)'s model (every operand once, no per-edge
    # outputs): the q pass rowptr + col + aR (copied to a compact table: read + write + read),
    # aL, q into the rows; the forward rowptr + col + the extended rows + Y, Ym + q, sma + W +
    # the T tiles written (896 floats per row); the backward the T tiles + dY, Y, Ym + sma +
    # d_aL
    T_ROW = 896 * 4
    alg_q = 4 * (N + 1) + 4 * E + 3 * 4 * N * 8 + 2 * 4 * N * H
    alg = alg_q + 4 * (N + 1) + 4 * E + 512 * N + 2 * 4 * N * F + 2 * 4 * N * H + 4 * F * (FIN + 1) + T_ROW * N
    alg_b = T_ROW * N + 3 * 4 * N * F + 2 * 4 * N * H
    # the walk pair's own (the previous round's) byte model, for the kernels timed beside
    alg_w = 4 * (N + 1) + 4 * E + 512 * N + 2 * 4 * N * F + 3 * 4 * N * H + 4 * F * (FIN + 1)
    alg_wb = 4 * (N + 1) + 4 * E + 512 * N + 3 * 4 * N * F + 2 * 4 * N * H
    traffic_f = [load_traffic(k) for k in ("k_gat_in_fwd<true>", "k_gat_in_q", "k_gat_in_ar")]
    out = {"value": 2 * E / t_step, "unit": "edges/s", "ms_per_step": t_step * 1e3, "steps": steps,
           "layer": (f"GAT layer 1 of config 3: {FIN} input features -> {H} heads x {D} (F={F}), Linear + both "
                     f"attention Linears + REF softmax aggregation + the program's ReLU, input space; forward + "
                     f"backward with every parameter gradient"),
           "fwd_ms": t_fwd * 1e3, "bwd_ms": t_bwd * 1e3,
           "roofline": {"bound": "hbm", "achieved": alg / t_kf / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                        "frac": alg / t_kf / HBM_PEAK, "kernel_ms": t_kf * 1e3, "alg_bytes_per_launch": alg,
                        "traffic": sum(traffic_f) if all(t is not None for t in traffic_f) else None,
                        "kernel": "gala_gat_in_fwd_t_f32: gala::k_gat_in_ar + k_gat_in_q + k_gat_in_fwd<true> "
                                  "(8 heads x 32 from 100 inputs)",
                        "traffic_note": "PMC FETCH_SIZE*2+WRITE_SIZE per launch summed over the call's three "
                                        "kernels (profiles/traffic.json): 126 M gathered 512-B extended input rows, "
                                        "the 3.5-KB T tiles per row written"}}
    out["bwd_roofline"] = {"bound": "hbm", "achieved": alg_b / t_kb / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                           "frac": alg_b / t_kb / HBM_PEAK, "kernel_ms": t_kb * 1e3, "alg_bytes_per_launch": alg_b,
                           "traffic": load_traffic("k_gat_in_bwd<8, true>"),
                           "kernel": "gala::k_gat_in_bwd<8, true> (gala_gat_in_bwd_t_f32: the T tiles, no walk)"}
    t_kfw, t_kbw = med(rounds["k_fwd_walk"]), med(rounds["k_bwd_walk"])
    out["walk"] = {"note": "the previous formulation timed beside: gala_gat_in_fwd_f32 (no T) and "
                           "gala_gat_in_bwd_f32 gathering the extended rows again over the transposed pattern",
                   "fwd_kernel_ms": t_kfw * 1e3, "bwd_kernel_ms": t_kbw * 1e3,
                   "fwd_frac": alg_w / t_kfw / HBM_PEAK, "bwd_frac": alg_wb / t_kbw / HBM_PEAK,
                   "pair_ms_vs_tmode_pair_ms": [(t_kfw + t_kbw) * 1e3, (t_kf + t_kb) * 1e3]}
    with_traffic_rate(out["roofline"])
    with_traffic_rate(out["bwd_roofline"])
    t_ceil = med(rounds["ceil"])
    if t_ceil:
        out["roofline"]["gather_ceiling_ms"] = t_ceil * 1e3
        out["roofline"]["frac_of_gather_ceiling"] = med([c / f for c, f in zip(rounds["ceil"], rounds["k_fwd"])])
        # (the T-mode backward gathers nothing: the ceiling applies to the walk's)
        out["walk"]["gather_ceiling_ms"] = t_ceil * 1e3
        out["walk"]["fwd_frac_of_gather_ceiling"] = med([c / f for c, f in zip(rounds["ceil"], rounds["k_fwd_walk"])])
        out["walk"]["bwd_frac_of_gather_ceiling"] = med([c / b for c, b in zip(rounds["ceil"], rounds["k_bwd_walk"])])
    out["interleaved_ms"] = {k: [round(v * 1e3, 3) for v in vs] for k, vs in rounds.items()}
    del st, f0, xext, Y0, Ym0, sma0, T0
    torch.cuda.empty_cache()
    # the previous formulation on the same layer: the Linear's output (1-KB rows) gathered by
    # the row-statistics pair, timed from that output (kernels only)
    X = torch.rand((N, F), device=dev, generator=gen) * 2 - 1
    aL = torch.rand((N, H), device=dev, generator=gen) - 0.5
    st2 = {}

    def fwd2():
        st2["f"] = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=H, want_aR=True)

    def bwd2():
        Yv, q, Ym, sma, aRo = st2["f"]
        st2["b"] = ops.gat_bwd_stats(dg, aL, aRo, dY, q, Yv, Ym, sma, heads=H)
    fwd2()
    t2f, t2b = timer(fwd2, 5), timer(bwd2, 5)
    out["gathering_linear_output"] = {
        "fwd_ms": t2f * 1e3, "bwd_ms": t2b * 1e3,
        "kernels": "gala::k_gat_fwd<64,4,8,2,1,true,8> / k_gat_bwd_fused<64,4,8,8,1,false,true> "
                   "(gala_gat_{fwd,bwd}_stats_f32 over the 1-KB Linear output rows; Linear and weight "
                   "gradients not included)"}
    del st2
    torch.cuda.empty_cache()
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = gat_cpu_baseline(hg, X.cpu().numpy(), dY.cpu().numpy(), aL.cpu().numpy(),
                                                   wR.cpu().numpy(), bR.cpu().numpy(), H)
            out["cpu_baseline"]["note"] = ("the reference's REF GAT pass sequence over the Linear's output "
                                           "(the Linear and the weight gradients are not in the CPU sample)")
        except Exception as e:  # the baseline is reported, never the target
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    del X, dY
    return out


def rmat_traffic(hub: str):
    """PMC bytes of one R-MAT SpMM call (profiles/traffic.json's "rmat|" entries: the PMC
    passes of tools/rmat_prof.py, tools/gpu_job.sh pmccmd=rmat + tools/merge_traffic.py), or
    None. exact: the degree-ordered row kernel + the REF-order hub kernel beside it; chunked:
    the rows + hub chunks grid and the chunk fix-up."""
    names = (("k_spmm_rowgroup<4, 8, 1, 4, false, false, false, false>", "k_spmm_hub_exact<4, 32, false, false>")
             if hub == "exact" else ("k_spmm_rows_chunks<4, 8, 1, 4, false, false>", "k_spmm_fixup<4, 8, 1, false>"))
    a, b = (load_traffic("rmat|void gala::" + n) for n in names)
    return a + b if a is not None and b is not None else None


FAMILY_GRAPH = {
    "rmat": "R-MAT a=0.57 b=0.19 c=0.19 symmetrised + self loops",
    "banded": "banded (every edge's ends at most min(8192, n/256) ids apart: a graph with locality, as a "
              "locality-preserving vertex order gives; it shards naturally) symmetrised + self loops",
}


def rmat_family(args, dev, be, timer, sync, kind="rmat"):
    """The same step on another graph of the Products shape: R-MAT:
    skewed degrees, so the SpMM runs the degree-ordered row schedule and the hub-row chunks;
    or banded: neighbours within min(8192, n/256) ids, so a row's X rows share the L2 (the locality the
    uniform graph lacks)."""
    import torch
    F = args.F
    t0 = time.time()
    hg = products_graph(kind, args.scale)
    log(f"[bench] {kind} graph N={hg.n_rows} E={hg.nnz} in {time.time() - t0:.1f}s")
    agg = OneGpuGCN(hg, F, be)
    gen = torch.Generator(device=dev).manual_seed(1234)
    X = torch.rand((hg.n_rows, F), device=dev, generator=gen) * 2 - 1
    dY = torch.rand((hg.n_rows, F), device=dev, generator=gen) * 2 - 1
    bufs = [be.empty(hg.n_rows, F) for _ in range(4)]
    steps = max(args.steps // 2, 2)
    step = make_fused_step(agg, X, dY, bufs)
    t_step = timed_steps(step, steps, 2, sync, lambda: None, lambda x: x)
    t_kernel = timer(lambda: be.spmm(agg.g, agg.Xs, bufs[0], agg.norm, False), 10)
    alg = spmm_alg_bytes(hg.n_rows, hg.n_rows, hg.nnz, F)
    hubs = getattr(agg.g, "split_rows", 0)
    out = {"value": 4 * hg.nnz / t_step, "unit": "edges/s", "ms_per_step": t_step * 1e3, "steps": steps,
           "graph": f"{FAMILY_GRAPH[kind]}, N={hg.n_rows}, E={hg.nnz}, "
                    f"max degree {int((hg.rowptr[1:] - hg.rowptr[:-1]).max())}",
           "split_rows": hubs,
           "roofline": {"bound": "hbm", "achieved": alg / t_kernel / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                        "frac": alg / t_kernel / HBM_PEAK, "kernel_ms": t_kernel * 1e3,
                        "alg_bytes_per_launch": alg,
                        "traffic": (None if be.name != "hip" else rmat_traffic("exact") if kind == "rmat" else
                                    load_traffic("banded|void gala::k_spmm_rowgroup<4, 8, 1, 4, false, false, false, false>")),
                        "kernel": "gala_spmm_f32 (degree-ordered k_spmm_rowgroup + k_spmm_hub_exact on a side "
                                  "stream: the hub rows in the reference's order)" if kind == "rmat" else
                                  "gala_spmm_f32 (k_spmm_rowgroup, XCD-ordered row blocks)"}}
    with_traffic_rate(out["roofline"])
    if hubs and be.name == "hip":
        # REF order is the default (bit-identical to the reference's serial row loop); the fast
        # mode sums hub rows as chunk partials (GALA_SPMM_HUB_CHUNKED, within fp32 rounding)
        out["hub_order"] = "exact: hub rows summed sequentially in CSR order (REF, bit-identical)"
        be.hub = "chunked"
        try:
            tc_step = timed_steps(step, steps, 2, sync, lambda: None, lambda x: x)
            tc_kernel = timer(lambda: be.spmm(agg.g, agg.Xs, bufs[0], agg.norm, False), 10)
        finally:
            be.hub = "exact"
        tr = rmat_traffic("chunked") if kind == "rmat" else None
        out["chunked"] = {"hub_order": "chunked: 512-edge partials + ordered fix-up (GALA_SPMM_HUB_CHUNKED; fp32 "
                                       "summation rounding of REF)",
                          "value": 4 * hg.nnz / tc_step, "ms_per_step": tc_step * 1e3,
                          "kernel_ms": tc_kernel * 1e3, "frac": alg / tc_kernel / HBM_PEAK, "traffic": tr,
                          "kernel": "k_spmm_rows_chunks + k_spmm_fixup"}
        if tr:
            out["chunked"]["traffic_GBps"] = tr / tc_kernel / 1e9
    if be.name == "hip":
        t_ceil = gather_ceiling(agg.g.col, agg.Xs, timer)
        if t_ceil:
            out["roofline"]["gather_ceiling_ms"] = t_ceil * 1e3
            out["roofline"]["frac_of_gather_ceiling"] = t_ceil / t_kernel
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--F", type=int, default=32)
    ap.add_argument("--scale", type=float, default=1.0, help="graph size multiplier (debug)")
    ap.add_argument("--calib-steps", type=int, default=3, help="timed steps per strong-scaling candidate")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: the host-CPU backend over gloo (plumbing checks, not a measurement)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-rmat", action="store_true")
    ap.add_argument("--no-banded", action="store_true", help="N > 1: no banded family")
    ap.add_argument("--banded", action="store_true", help="N = 1: add the banded family line")
    ap.add_argument("--no-gat", action="store_true")
    ap.add_argument("--no-weak", action="store_true")
    ap.add_argument("--budget-s", type=float, default=float(os.environ.get("GALA_BENCH_BUDGET_S", "420")),
                    help="N > 1: wall-clock budget from the process start; secondary fields and candidates "
                         "that would not fit are skipped (noted in the line's 'budget'); the headline always runs")
    ap.add_argument("--data", help="dataset directory in the reference's npy format (Adj_src.npy, Adj_dst.npy) "
                                   "or a Matrix Market .mtx graph; default: Data/Products/ when present, else "
                                   "the synthetic graph")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    # the driver reads ONE JSON line on stdout: the libraries' own stdout banners (RCCL's
    # version lines, gloo's connection lines) go to stderr, the result line to the real stdout
    result_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    from gala.backend import make_backend

    if args.device == "cuda":
        local_rank = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
        sync = torch.cuda.synchronize
    else:
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731
    be = make_backend(dev)
    timer = Timer(dev.type == "cuda")
    # GALA_BENCH_DIST=1 runs the partitioned path even on one rank (its collectives then go
    # through RCCL at world 1: the API contract checks a one-GPU box can make)
    distributed = world > 1 or os.environ.get("GALA_BENCH_DIST") == "1"
    if distributed:
        import datetime
        import torch.distributed as dist
        backend = os.environ.get("GALA_DIST_BACKEND", "nccl" if dev.type == "cuda" else "gloo")
        kw = dict(timeout=datetime.timedelta(seconds=int(os.environ.get("GALA_DIST_TIMEOUT", "300"))))
        if "MASTER_ADDR" not in os.environ:      # one rank without a launcher
            kw.update(init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend, **kw)
        out = run_multi(args, rank, world, dev, be, timer, sync)
    else:
        out = run_single(args, dev, be, timer, sync)
    if dev.type == "cpu":
        out["device"] = "cpu (host-CPU backend plumbing run; not a GPU measurement)"
    if TRAFFIC_STALE:   # PMC bytes withheld: the kernel changed since profiles/traffic.json's pass
        out["traffic_withheld_stale"] = sorted(set(TRAFFIC_STALE))
    if rank == 0:
        os.write(result_fd, (json.dumps(out) + "\n").encode())
    if distributed:
        from gala.comm import shutdown
        shutdown()
        # no library destructors after the process group is closed: a gloo rank could abort
        # in one at interpreter exit (gala/dist_run.py); the result line is already written
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


if __name__ == "__main__":
    main()
