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
    forward graph, cuda.h:1253-1257, so pre and post swap places);
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
    "Arxiv": (169343, 583122, 128, 40, 0.537),
    "Products": (2449029, 61859140, 100, 47, 0.080),
    "Reddit": (232965, 57307946, 602, 41, 0.660),
    "Papers100M": (111059956, 807842936, 128, 172, 0.011),
}
SUPPORTED = {"INPUT", "DEGREES", "POWER", "ROW_BROADCAST", "GCN_AGGREGATE", "AGGREGATE_MUL_SUM", "FFN", "RELU",
             "ADD", "SCALAR_ADD_EPS_MULTIPLY", "GAT_AGGREGATE"}


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


class _Agg(torch.autograd.Function):
    """post * A (pre * x) on the partition; backward pre * A (post * dy) (undirected)."""

    @staticmethod
    def forward(ctx, x, agg, pre, post):
        out = torch.empty_like(x)
        agg.apply(x.contiguous(), out, pre, post)
        ctx.agg, ctx.pre, ctx.post = agg, pre, post
        return out

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty_like(dy)
        ctx.agg.apply(dy.contiguous(), dx, ctx.post, ctx.pre)
        return dx, None, None, None


class _AggRelu(torch.autograd.Function):
    """post * A (pre * relu(act * x)) on the partition, the ReLU prologue fused into the
    aggregation's elementwise pass (as the generated programs' gcn_aggregate_relu_apply);
    backward: relu_scale_backward(pre * A (post * dy)) (undirected)."""

    @staticmethod
    def forward(ctx, x, act, agg, pre, post):
        out = torch.empty_like(x)
        agg.apply(x.contiguous(), out, pre, post, relu=True, act=act)
        ctx.save_for_backward(x)
        ctx.agg, ctx.act, ctx.pre, ctx.post = agg, act, pre, post
        return out

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        g = torch.empty_like(dy)
        ctx.agg.apply(dy.contiguous(), g, ctx.post, ctx.pre)
        dx = torch.empty_like(x)
        ctx.agg.be.relu_scale_backward(ctx.act, x.contiguous(), g, dx)
        return dx, None, None, None, None


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


class Program:
    """One rank's share of a galac program (post-pass IR)."""

    def __init__(self, ir: dict, graph: layout.HostGraph, X_own: torch.Tensor, labels_own: torch.Tensor,
                 train_own: torch.Tensor, rank: int, world: int, device, seed: int = 0, group=None,
                 layout_mode: str = "halo", exchange: str = "auto"):
        ops = {nd["op"] for nd in ir["nodes"]}
        bad = ops - SUPPORTED
        if bad:
            raise NotImplementedError(f"gala.dist_run: unsupported ops {sorted(bad)} (GCN / GIN / SAGE / GAT programs)")
        if "GAT_AGGREGATE" in ops:
            if ir["sched"].get("gat_mode", 0) != 0:
                raise NotImplementedError("gala.dist_run: FIXED-mode GAT (its backward needs A^T)")
        if not ir["sched"]["undirected"]:
            raise NotImplementedError("gala.dist_run: directed programs (the backward needs A^T)")
        if ir["sched"]["kernel_sample"] or ir["sched"]["data_sample"]:
            raise NotImplementedError("gala.dist_run: sampled programs")
        self.ir, self.device = ir, torch.device(device)
        self.be = make_backend(self.device)
        self.comm = Comm(group) if dist.is_initialized() else None
        self.rank, self.world = rank, world
        self.layout = layout_mode
        if layout_mode == "vcut":
            from . import vertex_cut as vc
            self.part = vc.vertex_cut_partition(graph, rank, world, exchange=exchange)
            self.agg = vc.VertexCutAggregator(self.part, 1, self.be, self.comm)
            self._gat = {}
            own_rowptr = self.part.deg_graph.rowptr
        elif layout_mode == "halo":
            self.part = gdist.partition_graph(graph, rank, world)
            self.agg = gdist.DistAggregator(self.part, 1, self.be, self.comm, exact=True)
            own_rowptr = self.part.graph.rowptr
            self._gat = {}
        else:
            raise ValueError(f"gala.dist_run: layout {layout_mode!r} (halo | vcut)")
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
            elif op == "POWER":
                y = torch.pow(a[0], nd["param"])
            elif op == "ROW_BROADCAST":
                y = a[0] * a[1]
            elif op == "GCN_AGGREGATE":
                x = a[0]
                if nd["param"] == 1:  # ReLU prologue: relu(act * x), fused into the aggregation
                    act = a[3] if len(a) > 3 else None
                    if act is not None and act.requires_grad:
                        x = torch.relu(act * x)
                        y = _Agg.apply(x, self.agg, self._vec(a[1]), self._vec(a[2]))
                    else:
                        y = _AggRelu.apply(x, self._vec(act), self.agg, self._vec(a[1]), self._vec(a[2]))
                else:
                    y = _Agg.apply(x, self.agg, self._vec(a[1]), self._vec(a[2]))
            elif op == "AGGREGATE_MUL_SUM":
                y = _Agg.apply(a[0], self.agg, None, None)
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
    ap.add_argument("--data", help="dataset directory in the reference's npy format")
    ap.add_argument("--synthetic", action="store_true", help="a seeded graph of the dataset's published shape")
    ap.add_argument("--scale", type=float, default=1.0, help="synthetic graph size multiplier")
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--dump", help="rank 0 writes an npz: predictions (all rows), losses, rowptr/col")
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
    if args.data:
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
    prog = Program(ir, g, torch.from_numpy(X).to(dev), torch.from_numpy(labels).to(dev),
                   torch.from_numpy(train).to(dev), rank, world, dev, seed=args.seed, layout_mode=args.layout,
                   exchange=args.exchange)
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
                     rowptr=g.rowptr, col=g.col, weights=np.array(json.dumps(init_weights)))
    if rank == 0:
        print(json.dumps({"ranks": world, "backend": dist.get_backend() if distributed else None,
                          "vertices": g.n_rows, "edges": g.nnz, "layout": args.layout,
                          "halo": prog.part.halo_mode if args.layout == "halo" else None,
                          "exchange": prog.part.exchange if args.layout == "vcut" else None,
                          "fwd_mean_s": float(np.mean(fwd_t[keep])), "epoch_mean_s": float(np.mean(ep_t[keep])),
                          "loss_first": losses[0], "loss_last": losses[-1]}), flush=True)
        print(f"{np.mean(fwd_t[keep]):.6g},{np.mean(ep_t[keep]):.6g}", flush=True)
    if distributed:
        from .comm import shutdown
        shutdown()


if __name__ == "__main__":
    sys.exit(main())
