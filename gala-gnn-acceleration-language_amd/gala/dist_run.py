"""Multi-rank runtime for galac programs: one process per GPU (torch.distributed, RCCL on
the GPU, gloo on the host), each rank training the same model on its row partition of
the graph.  BASELINE config 5 ("ogbn-papers100M GCN 3-layer across 8 MI355X") is
    galac bench/dsl/gcn3_papers10.txt --ir-json prog.json
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m gala.dist_run prog.json --synthetic

The generated C++ programs (galac's emitter) are single-device, like the reference's
gala.cu.  This runtime executes the same post-pass IR (galac --ir-json) instead:
  * node values are row-partitioned: rank p holds rows [bounds[p], bounds[p+1)) of every
    [N, F] value (gala/dist.py row_bounds: balanced by stored edges + rows);
  * every aggregation -- GCN_AGGREGATE post * A (pre * x), AGGREGATE_MUL_SUM -- is
    gala/dist.py's DistAggregator in exact mode: the halo rows arrive (RCCL all-gather or
    point-to-point), then ONE SpMM over the own rows, bit-identical to the one-GPU result;
    its backward is the same operator on the gradient (undirected graphs: slot 2g+1 is the
    forward graph, cuda.h:1253-1257, so pre and post swap places) or, for a directed
    program, the same aggregation over A^T's own partition (the same vertex ranges);
  * sampled programs: G.sample(k) (inplace_sample_graph_ab, tiling.h:454-508) samples the
    whole graph identically on every rank before it is partitioned; aggrFn.sample(k)
    (kernel sampling, cuda.h:313-321) runs the sampled SpMM over each rank's rows, whose
    CSR edge lists are whole, so every row samples the same edges as on one GPU (row
    partition only; .dynamic() redraws ra / rb before each forward from one seeded stream
    that every rank shares);
  * FFN weights are replicated (same seed on every rank); each rank's loss is its own
    training rows' share of the global mean cross entropy, and the weight gradients are
    summed over the ranks (one all-reduce per weight) before the identical Adam steps
    (lr 0.01, weight decay 5e-4, codegen/gala.cu:606-607).
  * `--layout vcut` is north_star's vertex cut instead (gala/vertex_cut.py
    VertexCutAggregator.apply): each rank holds the edges whose source it owns, computes
    partial rows for every destination and one RCCL reduce-scatter (`--exchange dense`) or
    an all-to-all of only the rows it holds edges of (`sparse`; `auto` picks by the graph's
    touched fraction) sums them into the owners' rows -- no halo; the sums regroup per
    rank, so results agree with one GPU to fp32 rounding.
  * GAT programs (GAT_AGGREGATE, REF softmax; config 3's gat_heads(H) included): each GAT
    layer is a training pair wrapped as an autograd Function (row-statistics forward, REF
    backward with dX, d_aL and, when the source logit is the layer's attention Linear of X,
    that Linear's gradients) -- gala/dist.py HaloGat on the halo layout (the one-GPU kernels
    over a gathered table: bit-identical to one rank), VertexCutGat on the vertex cut;
    per-head attention Linears (gat_heads) are the block-diagonal `HeadLinear`.
Training subgraphs (graph g > 0) run on the whole graph: they only drop rows no training
row depends on, so the training rows' values are unchanged.  The column-tiled layout
(col_tile) is a single-device layout and is not used.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from . import dist as gdist
from . import layout
from .backend import make_backend
from .comm import Comm

# (N, undirected edges, features, classes, train fraction) of the published shapes,
# as host/gala_datasets.h
SHAPES = {
    "Cora": (2708, 5278, 1433, 7, 140.0 / 2708),
    "Pubmed": (19717, 44324, 500, 3, 60.0 / 19717),
    "CoraFull": (19793, 63421, 8710, 70, 0.70),
    "Arxiv": (169343, 583122, 128, 40, 0.537),
    "Products": (2449029, 61859140, 100, 47, 0.080),
    "Reddit": (232965, 57307946, 602, 41, 0.660),
    "Papers100M": (111059956, 807842936, 128, 172, 0.011),
}
SUPPORTED = {"INPUT", "DEGREES", "FULL", "POWER", "ROW_BROADCAST", "GCN_AGGREGATE", "AGGREGATE_MUL_SUM", "FFN", "RELU",
             "ADD", "SCALAR_ADD_EPS_MULTIPLY", "GAT_AGGREGATE", "AGGREGATE_EDGE_MUL"}


def dataset_shape(name: str):
    """(N, undirected edges, features, classes, train fraction) of a dataset name, as
    host/gala_datasets.h: the published shapes, and papers100M_<p> for the p% node
    subgraph of ogbn-papers100M (get_large_sampled_datasets.py:68; an induced subgraph
    keeps about p^2 of the edges)."""
    if name in SHAPES:
        return SHAPES[name]
    pre = "papers100M_"
    if name.startswith(pre) and len(name) > len(pre):
        p = float(name[len(pre):]) / 100.0
        n0, m0, F, C, frac = SHAPES["Papers100M"]
        return int(n0 * p), int(m0 * p * p), F, C, frac
    return None


def _hash_uniform(rows: np.ndarray, cols: int, seed: int) -> np.ndarray:
    """Deterministic U[-1, 1) features of the given rows (counter hash of (seed, row, col)),
    so every rank draws exactly its own rows, whatever the number of ranks."""
    k = (rows.astype(np.uint64)[:, None] * np.uint64(cols) + np.arange(cols, dtype=np.uint64)[None, :])
    h = gdist._splitmix64(k ^ (np.uint64(seed) << np.uint64(40)))
    return ((h >> np.uint64(40)).astype(np.float64) / float(1 << 24) * 2.0 - 1.0).astype(np.float32)


def _hash_int(rows: np.ndarray, seed: int, mod: int) -> np.ndarray:
    h = gdist._splitmix64(rows.astype(np.uint64) ^ (np.uint64(seed) << np.uint64(44)))
    return ((h >> np.uint64(33)) % np.uint64(mod)).astype(np.int64)


class _EdgeMul:
    """AGGREGATE_EDGE_MUL's edge values r[row] * c[col] (the sparse rewrite's
    norm_i * norm_j, middle-end.h; cuda.h:870-952), kept factored: an AGGREGATE_MUL_SUM over
    them runs as r * A (c * x), which is what the rewrite started from, so no per-edge array
    and no halo of c is needed (agrees with the edge-weighted sum to fp32 rounding)."""

    def __init__(self, row, col):
        self.row, self.col = row, col

    def detach(self):
        return self


class _Agg(torch.autograd.Function):
    """post * A (pre * x) on the partition; backward pre * B (post * dy) with B the
    aggregation of slot 2g+1: A itself for an undirected program (cuda.h:1253-1257), A^T
    (its own partition) for a directed one.  samp (nsamp, ra, rb): kernel sampling, the
    same (ra, rb) in the backward (the reference reads the global ra / rb there too)."""

    @staticmethod
    def forward(ctx, x, agg, agg_b, pre, post, samp):
        out = torch.empty_like(x)
        agg.apply(x.contiguous(), out, pre, post, samp=samp)
        ctx.agg_b, ctx.pre, ctx.post, ctx.samp = agg_b, pre, post, samp
        return out

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty_like(dy)
        ctx.agg_b.apply(dy.contiguous(), dx, ctx.post, ctx.pre, samp=ctx.samp)
        return dx, None, None, None, None, None


class _AggRelu(torch.autograd.Function):
    """post * A (pre * relu(act * x)) on the partition, the ReLU prologue fused into the
    aggregation's elementwise pass (as the generated programs' gcn_aggregate_relu_apply);
    backward: relu_scale_backward(pre * B (post * dy)), B as in _Agg."""

    @staticmethod
    def forward(ctx, x, act, agg, agg_b, pre, post, samp):
        out = torch.empty_like(x)
        agg.apply(x.contiguous(), out, pre, post, relu=True, act=act, samp=samp)
        ctx.save_for_backward(x)
        ctx.agg_b, ctx.act, ctx.pre, ctx.post, ctx.samp = agg_b, act, pre, post, samp
        return out

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        g = torch.empty_like(dy)
        ctx.agg_b.apply(dy.contiguous(), g, ctx.post, ctx.pre, samp=ctx.samp)
        dx = torch.empty_like(x)
        ctx.agg_b.be.relu_scale_backward(ctx.act, x.contiguous(), g, dx)
        return dx, None, None, None, None, None, None


def _mirror():
    """The C++ operator mirror (gala._gala_torch): the same FFN / attention-Linear autograd
    ops a generated program calls (narrow-output MFMA forward, dense-gradient kernels)."""
    from . import _gala_torch
    return _gala_torch


class FfnLinear(torch.nn.Linear):
    """FFN_OP through the operator mirror's ffn_apply (host/gala_torch.cpp Ffn)."""

    def forward(self, x):
        return _mirror().ffn_apply(x.contiguous(), self.weight, self.bias)


class HeadLinear(torch.nn.Module):
    """gat_heads(H)'s attention vector Linear(F, 1) per head: out[:, h] = <x[:, head h],
    w[head h]> + b[h] (weight [1, F], bias [H]; galac's HeadAttn, tests/_ir_ref.py _ffn)."""

    def __init__(self, in_features: int, heads: int):
        super().__init__()
        k = 1.0 / np.sqrt(in_features // heads)
        self.heads = heads
        self.weight = torch.nn.Parameter(torch.empty(1, in_features).uniform_(-k, k))
        self.bias = torch.nn.Parameter(torch.empty(heads).uniform_(-k, k))

    def forward(self, x):
        return _mirror().head_attn_apply(x.contiguous(), self.weight, self.bias)


class _VcutGatFfn(torch.autograd.Function):
    """GAT aggregation over ranks (HaloGat or VertexCutGat) with the source logit recomputed from x (the
    DSL's attnR = ffn(res, out=1) of the aggregated res): inputs aL [n, H], x [n, F], the
    attention Linear's w [1, F] and b [H]; REF backward (VertexCutGat.backward)."""

    @staticmethod
    def forward(ctx, aL, x, w, b, layer):
        ctx.layer = layer
        return layer.forward_train(aL.detach().contiguous(), None, x.detach().contiguous(),
                                   w.detach().reshape(-1).contiguous(), b.detach().reshape(-1).contiguous())

    @staticmethod
    def backward(ctx, dy):
        dX, d_aL, dW, db = ctx.layer.backward(dy.contiguous())
        return d_aL, dX, dW.view(1, -1), db.view(-1), None


class _VcutGat(torch.autograd.Function):
    """GAT aggregation over ranks (HaloGat or VertexCutGat) with a given source logit aR [n, H]; the REF
    backward returns the row sums as both d_aL and d_aR (common.h:622-675)."""

    @staticmethod
    def forward(ctx, aL, aR, x, layer):
        ctx.layer = layer
        return layer.forward_train(aL.detach().contiguous(), aR.detach().contiguous(), x.detach().contiguous())

    @staticmethod
    def backward(ctx, dy):
        dX, d_aL = ctx.layer.backward(dy.contiguous())
        return d_aL, d_aL.clone(), dX, None


def check_program(ir: dict, layout_mode: str = "halo") -> None:
    """Raise NotImplementedError when this runtime cannot run the (post-pass) program on the
    given layout; the message names what is missing."""
    ops = {nd["op"] for nd in ir["nodes"]}
    bad = ops - SUPPORTED
    if bad:
        raise NotImplementedError(f"gala.dist_run: unsupported ops {sorted(bad)} (GCN / GIN / SAGE / GAT programs)")
    s = ir["sched"]
    if "GAT_AGGREGATE" in ops:
        if s.get("gat_mode", 0) != 0:
            raise NotImplementedError("gala.dist_run: FIXED-mode GAT (its backward needs A^T)")
        if not s["undirected"]:
            # the reference's directed REF backward applies the forward-order alpha to the
            # transposed pattern's edge positions (common.h:835-894 on slot 2g+1): every rank
            # would need the whole alpha; the generated single-device program runs them
            raise NotImplementedError("gala.dist_run: directed GAT programs (run the generated program)")
        if s["kernel_sample"]:
            raise NotImplementedError("gala.dist_run: kernel-sampled GAT programs")
    if s["kernel_sample"] and layout_mode == "vcut":
        raise NotImplementedError("gala.dist_run: kernel sampling on the vertex cut (a row's samples are "
                                  "picked among all its edges, which the cut splits by owner); use --layout halo")


class Program:
    """One rank's share of a galac program (post-pass IR)."""

    def __init__(self, ir: dict, graph: layout.HostGraph, X_own: torch.Tensor, labels_own: torch.Tensor,
                 train_own: torch.Tensor, rank: int, world: int, device, seed: int = 0, group=None,
                 layout_mode: str = "halo", exchange: str = "auto", train_all=None):
        """train_all: () -> bool [N] of every vertex's training flag, needed only by a
        directed program with training subgraphs (its levels are built from the global mask)."""
        check_program(ir, layout_mode)
        s = ir["sched"]
        self.directed = not s["undirected"]
        self.ksamp, self.dynamic = int(s["kernel_sample"]), bool(s["dynamic_sample"])
        self.ir, self.device = ir, torch.device(device)
        self.be = make_backend(self.device)
        self.comm = Comm(group) if dist.is_initialized() else None
        self.rank, self.world = rank, world
        self.layout = layout_mode
        if layout_mode not in ("halo", "vcut"):
            raise ValueError(f"gala.dist_run: layout {layout_mode!r} (halo | vcut)")
        self._exchange = exchange
        self.part, self.agg = self._partition(graph, None)
        own_rowptr = self.part.deg_graph.rowptr if layout_mode == "vcut" else self.part.graph.rowptr
        self._gat = {}
        # the aggregation pair (forward, slot 2g+1 backward) of every graph g of the program
        self.aggs = {0: (self.agg, self._partition(layout.transpose(graph)[0], self.part.bounds)[1]
                         if self.directed else self.agg)}
        L = int(ir.get("num_graphs", 1)) - 1
        if self.directed and L > 0:
            # training subgraphs (getMaskSubgraphs, tests/common.h:21-110): on an undirected
            # graph a level keeps every row a training row depends on, so graph 0 gives the
            # training rows the same values; on a directed one it does not, so each level
            # gets its own partitions (the same vertex ranges)
            levels = layout.mask_subgraphs(graph, np.asarray(train_all(), np.int32), L)
            for c in range(L):
                sub = levels[L - 1 - c]
                self.aggs[1 + c] = (self._partition(sub, self.part.bounds)[1],
                                    self._partition(layout.transpose(sub)[0], self.part.bounds)[1])
        # kernel sampling: (nsamp, ra, rb), ra / rb redrawn before every forward when dynamic
        # (rt::next_forward; the same seeded draws on every rank)
        self.samp = (self.ksamp, 5, 7) if self.ksamp else None
        self._rng = np.random.default_rng(seed + 17)
        self.samples = []
        self.deg = torch.from_numpy(np.diff(own_rowptr).astype(np.float32)).to(self.device).view(-1, 1)
        self.X, self.labels, self.train = X_own, labels_own, train_own
        # replicated weights, identical on every rank (same seed, same order as the IR)
        torch.manual_seed(seed)
        self.params = {}
        self.modules = torch.nn.ModuleDict()
        for w in ir["weights"]:
            if w["type"] == "linear" and int(w.get("heads", 1)) > 1 and w["out"] == 1:
                self.modules[w["name"]] = HeadLinear(w["in"], int(w["heads"]))
            elif w["type"] == "linear":
                self.modules[w["name"]] = FfnLinear(w["in"], w["out"])
            else:
                self.modules[w["name"]] = torch.nn.ParameterList([torch.nn.Parameter(torch.tensor([float(w["init"])]))])
        self.modules.to(self.device)
        n_train = torch.tensor([float(train_own.sum().item())], dtype=torch.float64,
                               device=self.device if (self.comm and self.comm.rccl) else "cpu")
        if self.comm is not None:
            dist.all_reduce(n_train, group=group)
        self.n_train = float(n_train.item())
        self.invariants = None

    def _partition(self, g, bounds):
        """(partition, aggregator) of graph g on this rank in the program's layout."""
        if self.layout == "vcut":
            from . import vertex_cut as vc
            part = vc.vertex_cut_partition(g, self.rank, self.world, bounds=bounds, exchange=self._exchange)
            return part, vc.VertexCutAggregator(part, 1, self.be, self.comm)
        part = gdist.partition_graph(g, self.rank, self.world, bounds=bounds)
        return part, gdist.DistAggregator(part, 1, self.be, self.comm, exact=True)

    def _param(self, name):
        m = self.modules[name]
        return m[0] if isinstance(m, torch.nn.ParameterList) else m

    def _vec(self, v):
        return None if v is None else v.reshape(-1).contiguous()

    def _gat_layer(self, nd, F, H):
        """The GAT layer of one GAT_AGGREGATE node (its buffers are width-specific): HaloGat on
        the row partition (bit-identical to one rank), VertexCutGat on the vertex cut."""
        from . import vertex_cut as vc
        key = nd["out"]
        if key not in self._gat:
            cls = vc.VertexCutGat if self.layout == "vcut" else gdist.HaloGat
            self._gat[key] = cls(self.part, F, H, self.be, self.comm, slope=float(nd["param"]))
        return self._gat[key]

    def forward(self):
        if self.samp is not None and self.dynamic:
            ra, rb = (int(v) for v in self._rng.integers(0, 101, 2))
            self.samp = (self.ksamp, ra, rb)
        if self.samp is not None:
            self.samples.append(self.samp[1:])
        vals = {}
        hoisted = self.invariants is None
        for nd in self.ir["nodes"]:
            out = nd["out"]
            if nd.get("hoisted") and not hoisted:
                vals[out] = self.invariants[out]
                continue
            op, a = nd["op"], [vals[i] if i >= 0 else None for i in nd["in"]]
            if op == "INPUT":
                y = self.X
            elif op == "DEGREES":
                y = self.deg
            elif op == "FULL":    # FULL_OP: the sampled degree, nsamples per row (one segment)
                y = torch.full((self.deg.shape[0], 1), float(nd["param"]), device=self.device)
            elif op == "POWER":
                y = torch.pow(a[0], nd["param"])
            elif op == "ROW_BROADCAST":
                y = a[0] * a[1]
            elif op == "GCN_AGGREGATE":
                x = a[0]
                fw, bw = self.aggs.get(nd["graph"], self.aggs[0])
                if nd["param"] == 1:  # ReLU prologue: relu(act * x), fused into the aggregation
                    act = a[3] if len(a) > 3 else None
                    if act is not None and act.requires_grad:
                        x = torch.relu(act * x)
                        y = _Agg.apply(x, fw, bw, self._vec(a[1]), self._vec(a[2]), self.samp)
                    else:
                        y = _AggRelu.apply(x, self._vec(act), fw, bw, self._vec(a[1]), self._vec(a[2]), self.samp)
                else:
                    y = _Agg.apply(x, fw, bw, self._vec(a[1]), self._vec(a[2]), self.samp)
            elif op == "AGGREGATE_MUL_SUM":
                w = a[1] if len(a) > 1 else None
                if w is not None and not isinstance(w, _EdgeMul):
                    raise NotImplementedError("gala.dist_run: AGGREGATE_MUL_SUM over computed edge values")
                fw, bw = self.aggs.get(nd["graph"], self.aggs[0])
                pre, post = (w.col, w.row) if w is not None else (None, None)
                y = _Agg.apply(a[0], fw, bw, pre, post, self.samp)
            elif op == "AGGREGATE_EDGE_MUL":
                if a[0].requires_grad or a[1].requires_grad:
                    raise NotImplementedError("gala.dist_run: AGGREGATE_EDGE_MUL of trained values")
                y = _EdgeMul(self._vec(a[0]), self._vec(a[1]))
            elif op == "GAT_AGGREGATE":
                aL, x = a[0], a[2]
                n = x.shape[0]
                H = aL.numel() // max(n, 1)
                layer = self._gat_layer(nd, x.shape[1], H)
                if nd["weight"]:     # gat_aggregate_ffn: attnR = the Linear of x, recomputed
                    m = self.modules[nd["weight"]]
                    y = _VcutGatFfn.apply(aL.reshape(n, H), x, m.weight, m.bias, layer)
                else:
                    y = _VcutGat.apply(aL.reshape(n, H), a[1].reshape(n, H), x, layer)
            elif op == "FFN":
                y = self.modules[nd["weight"]](a[0])
            elif op == "RELU":
                y = torch.relu(a[0])
            elif op == "ADD":
                y = a[0] + a[1]
            elif op == "SCALAR_ADD_EPS_MULTIPLY":
                y = (1 + self._param(nd["weight"])) * a[0]
            vals[out] = y
        if hoisted:  # training-invariant values (code motion): computed once
            self.invariants = {nd["out"]: vals[nd["out"]].detach() for nd in self.ir["nodes"] if nd.get("hoisted")}
        return vals[self.ir["output"]]

    def loss(self, pred):
        """This rank's share of the global mean cross entropy over the training rows."""
        logp = torch.log_softmax(pred[self.train], 1)
        return -logp.gather(1, self.labels[self.train].view(-1, 1)).sum() / self.n_train

    def reduce_grads(self):
        if self.comm is None:
            return
        for p in self.modules.parameters():
            if p.grad is not None:
                self.comm.wait([self.comm.all_reduce(p.grad)])


def load(ir_path):
    with open(ir_path) as f:
        d = json.load(f)
    return d.get("post", d)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("ir", help="galac --ir-json output (its post-pass IR is run)")
    ap.add_argument("--data", help="dataset directory in the reference's npy format, or a Matrix Market .mtx "
                                   "graph (then with synthetic features, labels and training rows)")
    ap.add_argument("--synthetic", action="store_true", help="a seeded graph of the dataset's published shape")
    ap.add_argument("--scale", type=float, default=1.0, help="synthetic graph size multiplier")
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--dump", help="rank 0 writes an npz: the first forward's predictions (all rows), the losses, "
                                   "the first epoch's weight gradients (grad:<name>), rowptr/col, the initial "
                                   "weights, the kernel-sampling (ra, rb) of every forward")
    ap.add_argument("--dump-stride", type=int, default=1,
                    help="dump the predictions of every k-th row only (rows in 'rows'; large graphs)")
    ap.add_argument("--layout", default="halo", choices=["halo", "vcut"],
                    help="halo: row partition + exact halo SpMM; vcut: vertex cut + reduce-scatter")
    ap.add_argument("--dist", action="store_true",
                    help="run the collectives even on one rank (RCCL at world 1 on one GPU)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "dense", "sparse"],
                    help="vcut: dense reduce-scatter, sparse DCSR all-to-all, or auto (touched fraction)")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.device == "cuda":
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    distributed = world > 1 or args.dist
    if distributed:
        backend = os.environ.get("GALA_DIST_BACKEND", "nccl" if dev.type == "cuda" else "gloo")
        kw = {}
        if "MASTER_ADDR" not in os.environ:      # one rank without a launcher
            import socket
            so = socket.socket()
            so.bind(("127.0.0.1", 0))
            kw = dict(init_method=f"tcp://127.0.0.1:{so.getsockname()[1]}", rank=0, world_size=1)
            so.close()
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend, **kw)
    ir = load(args.ir)
    s = ir["sched"]
    if args.data and args.data.endswith(".mtx"):
        # a Matrix Market graph (readSM / MtxIO semantics; the pattern), synthetic features
        g = layout.load_mtx(args.data)
        g.val = None
        shape = dataset_shape(s["dataset"])
        frac = shape[4] if shape else 0.1
        X_all = lab_all = tr_all = None
    elif args.data:
        g = layout.load_npy_dataset(args.data)
        X_all = np.load(os.path.join(args.data, "Feat.npy"), mmap_mode="r")
        lab_all = np.load(os.path.join(args.data, "Lab.npy")).reshape(-1)
        tr_all = np.load(os.path.join(args.data, "TnMsk.npy")).reshape(-1)
    else:
        shape = dataset_shape(s["dataset"])
        if shape is None:
            raise SystemExit(f"gala.dist_run: no published shape for dataset {s['dataset']!r}; pass --data")
        n0, m0, _, _, frac = shape
        n, m = max(int(n0 * args.scale), 2), max(int(m0 * args.scale), 1)
        g = layout.gen_graph("uniform", n, m, seed=args.seed)
        X_all = lab_all = tr_all = None
    g_in = g                     # the dump's graph: the program's input, before data sampling
    if int(s["data_sample"]) > 0:   # G.sample(k): inplace_sample_graph_ab(5, 7) on every rank alike
        g = layout.sample_ab(g, int(s["data_sample"]), 5, 7)
    F, C = int(s["feat_size"]), int(s["label_size"])
    bounds = gdist.row_bounds(g.rowptr, world)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    rows = np.arange(r0, r1)
    if X_all is None:
        X = _hash_uniform(rows, F, args.seed)
        labels = _hash_int(rows, args.seed + 1, C)
        train = (_hash_int(rows, args.seed + 2, 1 << 20) < int(frac * (1 << 20))) | (rows == 0)
    else:
        X = np.ascontiguousarray(X_all[r0:r1], np.float32)
        labels = lab_all[r0:r1].astype(np.int64)
        train = tr_all[r0:r1] > 0
    if tr_all is None:
        def train_all():
            every = np.arange(g.n_rows)
            return (_hash_int(every, args.seed + 2, 1 << 20) < int(frac * (1 << 20))) | (every == 0)
    else:
        def train_all():
            return tr_all > 0
    prog = Program(ir, g, torch.from_numpy(X).to(dev), torch.from_numpy(labels).to(dev),
                   torch.from_numpy(train).to(dev), rank, world, dev, seed=args.seed, layout_mode=args.layout,
                   exchange=args.exchange, train_all=train_all)
    init_weights = {k: v.detach().cpu().numpy().tolist() for k, v in prog.modules.state_dict().items()}
    opt = torch.optim.Adam(prog.modules.parameters(), lr=0.01, weight_decay=5e-4)
    iters = args.iters if args.iters is not None else max(int(s.get("iterations", 0)), 1)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    fwd_t, ep_t, losses = [], [], []
    for epoch in range(iters):
        sync()
        t0 = time.perf_counter()
        pred = prog.forward()
        sync()
        t1 = time.perf_counter()
        opt.zero_grad()
        loss = prog.loss(pred)
        loss.backward()
        prog.reduce_grads()
        if epoch == 0:   # the first epoch's summed weight gradients (the dump's grad:<name>)
            first_grads = {k: v.grad.detach().cpu().numpy() for k, v in prog.modules.named_parameters()
                           if v.grad is not None}
        opt.step()
        sync()
        t2 = time.perf_counter()
        lt = loss.detach().reshape(1).to(torch.float64)
        if distributed:
            lt = lt.to(dev) if prog.comm.rccl else lt.cpu()
            dist.all_reduce(lt)
        losses.append(float(lt.item()))
        if epoch == 0:
            first_pred = pred.detach()
        fwd_t.append(t1 - t0)
        ep_t.append(t2 - t0)
    keep = slice(min(4, iters - 1), None)  # the reference drops its first epochs (gala.cu:613-637)
    if args.dump:
        sizes = [int(bounds[q + 1] - bounds[q]) for q in range(world)]
        pr = first_pred
        if world > 1:   # equal-sized blocks for all_gather: pad every rank's rows
            gdev = dev if prog.comm.rccl else torch.device("cpu")
            pad = torch.full((max(sizes), pr.shape[1]), float("nan"), device=gdev)
            pad[:pr.shape[0]] = pr.to(gdev)
            parts = [torch.empty_like(pad) for _ in sizes]
            dist.all_gather(parts, pad)
            pr = torch.cat([t[:n] for t, n in zip(parts, sizes)])
        pr = pr.cpu()
        if rank == 0:
            rows_d = np.arange(0, g.n_rows, max(args.dump_stride, 1))
            np.savez(args.dump, prediction=pr.numpy()[rows_d], rows=rows_d, losses=np.array(losses),
                     rowptr=g_in.rowptr, col=g_in.col, weights=np.array(json.dumps(init_weights)),
                     samples=np.array(prog.samples, np.int64).reshape(-1, 2),
                     **{"grad:" + k: v for k, v in first_grads.items()})
    messages = None
    if distributed:   # every rank: the maxima over ranks are collectives
        from .comm import message_stats

        def reduce_max(x):
            t = torch.tensor([x], dtype=torch.float64, device=dev if prog.comm.rccl else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
        messages = message_stats(reduce_max)
    if rank == 0:
        print(json.dumps({"ranks": world, "backend": dist.get_backend() if distributed else None,
                          "messages": messages,
                          "vertices": g.n_rows, "edges": g.nnz, "layout": args.layout,
                          "halo": prog.part.halo_mode if args.layout == "halo" else None,
                          "exchange": prog.part.exchange if args.layout == "vcut" else None,
                          "fwd_mean_s": float(np.mean(fwd_t[keep])), "epoch_mean_s": float(np.mean(ep_t[keep])),
                          "loss_first": losses[0], "loss_last": losses[-1]}), flush=True)
        print(f"{np.mean(fwd_t[keep]):.6g},{np.mean(ep_t[keep]):.6g}", flush=True)
    if distributed:
        from .comm import shutdown
        print(f"[gala.dist_run rank {rank}] epochs done", file=sys.stderr, flush=True)
        shutdown()
        print(f"[gala.dist_run rank {rank}] process group closed", file=sys.stderr, flush=True)


if __name__ == "__main__":
    rc = main() or 0
    # End the process without running library destructors: after the process group is
    # closed, about one gloo rank in forty aborted here at interpreter exit ("terminate
    # called without an active exception", a C++ thread still joinable in some library's
    # static teardown); everything the run produced is written and flushed by now.
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)
