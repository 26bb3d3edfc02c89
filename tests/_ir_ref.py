"""TEST INFRASTRUCTURE: a float64 torch-CPU executor for galac's IR (galac --ir-json).

It gives the IR its mathematical meaning, independently of the generated C++ and of the
HIP operators, so that
  * CPU tests can check that the middle-end passes keep a program's meaning
    (pre-pass vs post-pass IR on the same weights), and
  * GPU tests can check a generated program end to end (its --dump of the first
    forward/backward against this executor on the dumped weights and data).
Op semantics follow the reference: AGGREGATE_MUL_SUM = A x in CSR order,
edge softmax p = min(e^s, 1e12), alpha = p / (1e-12 + sum_row p), LeakyReLU(0.2) on the
attention logits, (1 + eps) x for GIN's scalar, degrees = row edge counts of graph 0,
kernel sampling = the (ra*j + rb) mod deg edge of each row (cuda.h:313-321).
"""
import json
import struct

import numpy as np
import torch

from gala import layout


def read_dump(path):
    """Reads a gala_prog --dump file (gala_runtime.cpp rt::dump)."""
    out = {}
    with open(path, "rb") as f:
        assert f.read(8) == b"GALADMP1"
        (n,) = struct.unpack("<I", f.read(4))
        for _ in range(n):
            (nl,) = struct.unpack("<I", f.read(4))
            name = f.read(nl).decode()
            code = f.read(1)[0]
            (nd,) = struct.unpack("<I", f.read(4))
            shape = struct.unpack("<" + "q" * nd, f.read(8 * nd)) if nd else ()
            dt = {0: np.float32, 1: np.int64, 2: np.int32, 3: np.bool_}[code]
            cnt = int(np.prod(shape)) if nd else 1
            out[name] = np.frombuffer(f.read(cnt * np.dtype(dt).itemsize), dt).reshape(shape).copy()
    return out


def load_ir(path):
    with open(path) as f:
        return json.load(f)


def _csr(rowptr, col, n_cols, val=None):
    rowptr = torch.as_tensor(np.asarray(rowptr, np.int64))
    col = torch.as_tensor(np.asarray(col, np.int64))
    v = torch.ones(col.shape[0], dtype=torch.float64) if val is None else val
    return torch.sparse_csr_tensor(rowptr, col, v, (rowptr.shape[0] - 1, n_cols))


def _spmm(rowptr, col, x, w=None):
    """sum_e w_e x[col_e] per row, differentiable in x and w (duplicate edges kept).
    w [E] or [E, H]: head h weights columns hD:(h+1)D."""
    rows = _rows(rowptr)
    g = x[torch.as_tensor(np.asarray(col, np.int64))]
    if w is not None:
        H = w.numel() // max(g.shape[0], 1) if g.shape[0] else 1
        g = (g.view(g.shape[0], H, -1) * w.reshape(-1, H, 1)).reshape(g.shape)
    return torch.zeros(len(rowptr) - 1, x.shape[1], dtype=x.dtype).index_add(0, rows, g)


def _rows(rowptr):
    return torch.as_tensor(np.repeat(np.arange(len(rowptr) - 1), np.diff(rowptr)))


def sampled_graph(rowptr, col, nsamp, ra, rb):
    """The edges a kernel-sampled aggregation visits (cuda.h:313-321), in visit order."""
    n = len(rowptr) - 1
    deg = np.diff(rowptr)
    rp = np.zeros(n + 1, np.int64)
    cols = []
    for i in range(n):
        if deg[i] > 0:
            j = np.arange(nsamp)
            cols.append(col[rowptr[i] + (ra * j + rb) % deg[i]])
            rp[i + 1] = rp[i] + nsamp
        else:
            rp[i + 1] = rp[i]
    return rp, (np.concatenate(cols) if cols else np.zeros(0, np.int32))


class Graphs:
    """Graph g of a program: 0 = the whole graph, 1 + c = the c-th aggregation's mask
    subgraph (level L-1-c of getMaskSubgraphs).  The backward of an aggregation on graph g
    reads slot 2g+1 (common.h:928-978): the same matrix for graph 0 of an undirected
    program (cuda.h:1253-1257), the transpose otherwise (buildTranspose)."""

    def __init__(self, ir, rowptr, col, train_mask, ra=5, rb=7):
        s = ir["sched"]
        n = len(rowptr) - 1
        self.n = n
        self.undirected = bool(s["undirected"])
        g = layout.HostGraph(n, n, np.asarray(rowptr, np.int32), np.asarray(col, np.int32))
        if s["data_sample"] > 0:
            g = layout.sample_ab(g, s["data_sample"], 5, 7)
        graphs = [g]
        L = ir["num_graphs"] - 1
        if L > 0:
            levels = layout.mask_subgraphs(g, np.asarray(train_mask, np.int32), L)
            graphs += [levels[L - 1 - c] for c in range(L)]
        self.host = graphs
        self.ks = s["kernel_sample"]
        self.ra, self.rb = ra, rb
        self.deg0 = torch.as_tensor(np.diff(graphs[0].rowptr).astype(np.float64)).view(-1, 1)

    def edges(self, gi):
        g = self.host[gi]
        if self.ks > 0:
            return sampled_graph(g.rowptr, g.col, self.ks, self.ra, self.rb)
        return g.rowptr, g.col

    def matrix(self, gi, val=None):
        rp, col = self.edges(gi)
        return _csr(rp, col, self.n, val)

    def backward_edges(self, gi):
        """The pattern of slot 2g+1: graph g itself for graph 0 of an undirected program,
        its transpose (buildTranspose) otherwise."""
        if gi == 0 and self.undirected:
            return self.edges(gi)
        g = self.host[gi]
        t, _ = layout.transpose(layout.HostGraph(g.n_rows, g.n_cols, g.rowptr, g.col))
        if self.ks > 0:
            return sampled_graph(t.rowptr, t.col, self.ks, self.ra, self.rb)
        return t.rowptr, t.col

    def backward_matrix(self, gi):
        rp, col = self.backward_edges(gi)
        return _csr(rp, col, self.n)


class _SlotSpmm(torch.autograd.Function):
    """A x forward, B dY backward: the emitted <K>_AutoGrad pair (B = slot 2g+1)."""

    @staticmethod
    def forward(ctx, x, A, B):
        ctx.B = B
        return A @ x

    @staticmethod
    def backward(ctx, dy):
        return ctx.B @ dy, None, None


class _GatRef(torch.autograd.Function):
    """GAT aggregation with the reference's backward chain (`ref` mode;
    common.h:835-894): every backward step runs on slot 2g+1's pattern (rp_b, col_b) with
    the forward's alpha taken by edge POSITION -- dX = A_b(alpha) dY, d alpha_e =
    <dY_row, X_col> (edge_sddmm), ds = alpha*dalpha - alpha*(1e-12 + sum_row alpha*dalpha),
    dz = LeakyReLU'(z) ds with z at the same position of the forward pattern,
    daL = daR = 1e-12 + sum_row dz.  On an undirected graph slot 2g+1 is the forward graph;
    on a directed one it is the transpose and the positions pair unrelated edges, as the
    reference does."""

    @staticmethod
    def forward(ctx, aL, aR, x, rp, col, n, slope, rp_b=None, col_b=None):
        rows = _rows(rp)
        colt = torch.as_tensor(col, dtype=torch.long)
        z = aL.view(-1)[rows] + aR.view(-1)[colt]
        alpha = _softmax(rp, _lrelu(z, slope))
        ctx.save_for_backward(x, alpha, z)
        rp_b, col_b = (rp, col) if rp_b is None else (rp_b, col_b)
        ctx.rp_b, ctx.col_b, ctx.n, ctx.slope = rp_b, torch.as_tensor(col_b, dtype=torch.long), n, slope
        return _csr(rp, col, n, alpha) @ x

    @staticmethod
    def backward(ctx, dy):
        x, alpha, z = ctx.saved_tensors
        rp, col, n = ctx.rp_b, ctx.col_b, ctx.n
        rows = _rows(rp)
        dx = _csr(rp, col.numpy(), n, alpha) @ dy
        dalpha = (dy[rows] * x[col]).sum(1)
        sds = alpha * dalpha
        acc = torch.zeros(n, dtype=dy.dtype).index_add(0, rows, sds) + 1e-12
        ds = sds - alpha * acc[rows]
        dz = torch.where(z > 0, ds, ds * ctx.slope)
        da = (torch.zeros(n, dtype=dy.dtype).index_add(0, rows, dz) + 1e-12).view(-1, 1)
        return da, da.clone(), dx, None, None, None, None, None, None


def run(ir, graphs: Graphs, X, params, segments=1):
    """Forward of one IR ({"pre"|"post"} part of galac --ir-json) in float64.
    params: name -> float64 tensor (fc0.weight, fc0.bias, eps0, ...)."""
    vals = {}
    for nd in ir["nodes"]:
        op, ins = nd["op"], nd["in"]
        a = [vals[i] if i >= 0 else None for i in ins]
        gi = nd["graph"]
        if op == "INPUT":
            y = X
        elif op == "DEGREES":
            y = graphs.deg0.clone()
        elif op == "FULL":
            y = torch.full((graphs.n, 1), float(nd["param"]) * segments, dtype=torch.float64)
        elif op == "POWER":
            y = torch.pow(a[0], nd["param"])
        elif op == "ROW_BROADCAST":
            y = a[0] * a[1]
        elif op == "AGGREGATE_MUL_SUM":
            if len(a) > 1:
                rp, col = graphs.edges(gi)
                y = _spmm(rp, col, a[0], a[1])
            else:
                y = _SlotSpmm.apply(a[0], graphs.matrix(gi), graphs.backward_matrix(gi))
        elif op == "GCN_AGGREGATE":
            x = a[0]
            if nd["param"] == 1:  # ReLU prologue: relu(act * x)
                act = a[3] if len(a) > 3 else None
                x = torch.relu(x if act is None else act * x)
            x = x if a[1] is None else a[1] * x
            y = _SlotSpmm.apply(x, graphs.matrix(gi), graphs.backward_matrix(gi))
            if a[2] is not None:
                y = a[2] * y
        elif op == "GAT_AGGREGATE":
            rp, col = graphs.edges(gi)
            rp_b, col_b = graphs.backward_edges(gi)
            H = a[0].numel() // graphs.n                  # heads (galac gat_heads)
            if nd["weight"]:  # gat_aggregate_ffn: attnR = Linear(X) of the aggregated rows
                a[1] = _ffn(a[2], params, nd["weight"], H)
            D = a[2].shape[1] // H
            aL, aR = a[0].reshape(graphs.n, H), a[1].reshape(-1, H)
            heads = []
            for h in range(H):                           # heads are independent
                xh = a[2][:, h * D:(h + 1) * D]
                if ir["sched"]["gat_mode"] == 0:
                    heads.append(_GatRef.apply(aL[:, h].reshape(-1, 1), aR[:, h].reshape(-1, 1), xh, rp, col,
                                               graphs.n, nd["param"], rp_b, col_b))
                else:
                    alpha = _softmax(rp, _lrelu(aL[:, h][_rows(rp)] + aR[:, h][torch.as_tensor(col, dtype=torch.long)],
                                                nd["param"]))
                    heads.append(_spmm(rp, col, xh, alpha))
            y = heads[0] if H == 1 else torch.cat(heads, 1)
        elif op == "FFN":
            y = _ffn(a[0], params, nd["weight"], _heads(ir, nd["weight"]))
        elif op == "RELU":
            y = torch.relu(a[0])
        elif op == "LEAKY_RELU":
            y = _lrelu(a[0], nd["param"])
        elif op == "AGGREGATE_EDGE_SUM":
            rp, col = graphs.edges(gi)
            H = a[0].numel() // graphs.n
            y = (a[0].reshape(-1, H)[_rows(rp)] + a[1].reshape(-1, H)[torch.as_tensor(col, dtype=torch.long)])
            y = y.reshape(-1) if H == 1 else y
        elif op == "AGGREGATE_EDGE_MUL":
            rp, col = graphs.edges(gi)
            y = a[0].view(-1)[_rows(rp)] * a[1].view(-1)[torch.as_tensor(col, dtype=torch.long)]
        elif op == "SOFTMAX":
            rp, _ = graphs.edges(gi)
            y = _softmax(rp, a[0])
        elif op == "SCALAR_ADD_EPS_MULTIPLY":
            y = (1 + params[nd["weight"]]) * a[0]
        elif op == "ADD":
            y = a[0] + a[1]
        else:
            raise NotImplementedError(op)
        vals[nd["out"]] = y
    return vals[ir["output"]]


def _lrelu(x, slope):
    return torch.where(x > 0, x, x * slope)


def _heads(ir, wname):
    for w in ir["weights"]:
        if w["name"] == wname:
            return int(w.get("heads", 1))
    return 1


def _ffn(x, params, wname, heads):
    """FFN: x W^T + b; with heads > 1 (gat_heads attention vectors) the per-head dot
    out[:, h] = x[:, head h] . W[0, head h] + b[h]."""
    W, b = params[wname + ".weight"], params[wname + ".bias"]
    if heads == 1 or W.shape[0] != 1 or b.numel() != heads:
        return x @ W.T + b
    D = x.shape[1] // heads
    return (x.reshape(x.shape[0], heads, D) * W.reshape(1, heads, D)).sum(2) + b.reshape(1, heads)


def _softmax(rowptr, s):
    """Per-row edge softmax of s [E] or [E, H] (each head on its own)."""
    p = torch.clamp(torch.exp(s), max=1e12)
    rows = _rows(rowptr)
    shape = (len(rowptr) - 1,) + tuple(s.shape[1:])
    r = torch.zeros(shape, dtype=s.dtype).index_add(0, rows, p) + 1e-12
    return p * (1.0 / r)[rows]


def init_params(ir, seed=0, zero_bias=False):
    """Random float64 weights for every weight the IR names (requires_grad)."""
    g = torch.Generator().manual_seed(seed)
    p = {}
    for w in ir["weights"]:
        if w["type"] == "linear":
            p[w["name"] + ".weight"] = (torch.rand(w["out"], w["in"], generator=g, dtype=torch.float64) - 0.5) / np.sqrt(w["in"])
            b = (torch.rand(w["out"] * int(w.get("heads", 1)), generator=g, dtype=torch.float64) - 0.5) / np.sqrt(w["in"])
            p[w["name"] + ".bias"] = torch.zeros_like(b) if zero_bias else b
        else:
            p[w["name"]] = torch.tensor([float(w["init"])], dtype=torch.float64)
    for t in p.values():
        t.requires_grad_(True)
    return p
