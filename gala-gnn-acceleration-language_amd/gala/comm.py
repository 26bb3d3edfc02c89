"""Collectives of the partitioned aggregation (one process per GPU, torch.distributed).

Backend "nccl" is RCCL on ROCm: every collective is issued asynchronously on RCCL's own
stream, which first waits for the caller's current stream (so rows written there are
visible), and `wait(works)` makes the caller's current stream wait for it in turn -- no
host synchronisation, so the compute stream can run SpMM work between a collective's
issue and its use.

Any other backend (gloo: the CPU test suite, and two ranks sharing one GPU in a
rehearsal) runs synchronously; device tensors are staged through host memory, because
gloo's device-tensor support varies by collective.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

# RCCL 2.26.6 (the torch 2.10 ROCm wheel's librccl) returns wrong rows from all_to_all_single
# and from batched point-to-point once the payload passes 1 GiB: at 2^30 + 512 B (and at 2, 5.7
# GiB) every row past the first half is wrong (tools/a2a_probe.py on MI355X,
# profiles/r04_rccl_a2a_probe.jsonl; 568 MB is exact, and reduce_scatter / all_gather are exact
# at every size).  That was the round-3 divergence of the sparse vertex-cut exchange at config
# 5's 11.1 M-row shape (5.7 GB per all-to-all).  Every all-to-all and point-to-point message is
# therefore cut into rounds of at most MAX_MSG_BYTES (512 MiB: half the smallest failing size).
MAX_MSG_BYTES = 1 << 29


# Message sizes every collective kind sent in this process (for the first multi-GPU run to
# show whether the MAX_MSG_BYTES cut held): per kind the calls, the largest tensor one RCCL
# call was handed (an all-to-all round's send payload, one point-to-point piece), the largest
# payload before cutting, and the most rounds / pieces one exchange took.  The host-staged
# (gloo) path records the plan RCCL would have run.
MSG_KINDS = ("all_gather", "reduce_scatter", "all_reduce", "all_to_all", "p2p")
_MSG = {}


def _note(kind: str, call_bytes: int, payload_bytes: int, rounds: int = 1) -> None:
    s = _MSG.setdefault(kind, {"calls": 0, "max_call_bytes": 0, "max_payload_bytes": 0, "max_rounds": 0})
    s["calls"] += 1
    s["max_call_bytes"] = max(s["max_call_bytes"], int(call_bytes))
    s["max_payload_bytes"] = max(s["max_payload_bytes"], int(payload_bytes))
    s["max_rounds"] = max(s["max_rounds"], int(rounds))


def reset_message_stats() -> None:
    _MSG.clear()


def message_stats(reduce_max=None) -> dict:
    """{kind: {calls, max_call_bytes, max_payload_bytes, max_rounds}} for the kinds sent, plus
    cut_at_bytes.  reduce_max (a collective every rank calls alike, e.g. a MAX all-reduce of
    one number): the maxima over all ranks (every rank must call this together)."""
    out = {}
    for kind in MSG_KINDS:
        s = dict(_MSG.get(kind, {"calls": 0, "max_call_bytes": 0, "max_payload_bytes": 0, "max_rounds": 0}))
        if reduce_max is not None:
            s = {k: int(reduce_max(float(v))) for k, v in s.items()}
        if s["calls"]:
            out[kind] = s
    out["cut_at_bytes"] = MAX_MSG_BYTES
    return out


class _Works:
    """Several async collectives waited on as one (a chunked all-to-all)."""

    def __init__(self, works):
        self.works = [w for w in works if w is not None]

    def wait(self):
        for w in self.works:
            w.wait()


def a2a_rounds(in_splits, out_splits, world: int, row_bytes: int, max_rows=None, strict=True):
    """The rounds of an all-to-all cut at MAX_MSG_BYTES: a list of (ins, outs), ins[q] the
    (start, stop) rows of the input sent to rank q in that round, outs[q] the rows of the output
    received from rank q.  Round j carries rows [j*r, (j+1)*r) of every block, r =
    MAX_MSG_BYTES // (world * row_bytes), so one round's message is at most MAX_MSG_BYTES; the
    round count comes from max_rows, a bound on every rank's blocks that all ranks pass alike
    (they must issue the same collectives), or from this rank's largest block.  One round when
    nothing needs cutting.  strict=False (the uncut host-staged path, which only records the
    plan) takes the larger of the two instead of refusing a block past max_rows; the ranks'
    agreement on the bound is checked collectively once per exchange plan
    (Comm.check_block_bound)."""
    in_splits, out_splits = [int(v) for v in in_splits], [int(v) for v in out_splits]
    r = max(MAX_MSG_BYTES // (world * row_bytes), 1)
    biggest = max(in_splits + out_splits + [0])
    if strict and max_rows is not None and biggest > int(max_rows):
        # rows past rounds * r would never be sent, and the output would keep stale rows
        raise ValueError(f"a2a_rounds: a block of {biggest} rows exceeds max_rows={int(max_rows)}")
    m = biggest if max_rows is None else max(int(max_rows), biggest)
    rounds = max(-(-m // r), 1)
    io, oo = [0] * world, [0] * world
    for q in range(1, world):
        io[q] = io[q - 1] + in_splits[q - 1]
        oo[q] = oo[q - 1] + out_splits[q - 1]
    out = []
    for j in range(rounds):
        ins = [(io[q] + min(j * r, in_splits[q]), io[q] + min((j + 1) * r, in_splits[q])) for q in range(world)]
        outs = [(oo[q] + min(j * r, out_splits[q]), oo[q] + min((j + 1) * r, out_splits[q])) for q in range(world)]
        out.append((ins, outs))
    return out


def p2p_pieces(rows: int, row_bytes: int):
    """The (start, stop) row pieces of a point-to-point message cut at MAX_MSG_BYTES (both
    ends cut a message of the same shape alike)."""
    r = max(MAX_MSG_BYTES // row_bytes, 1)
    return [(0, rows)] if rows <= r else [(i, min(i + r, rows)) for i in range(0, rows, r)]


def _bytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def _row_bytes(t: torch.Tensor) -> int:
    """Bytes of one row (dim 0) of t, also for a tensor with no rows."""
    n = 1
    for d in t.shape[1:]:
        n *= int(d)
    return max(n, 1) * t.element_size()


class Comm:
    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.rccl = dist.get_backend(group) == "nccl"

    # -- helpers --------------------------------------------------------------------------
    @staticmethod
    def _host(t: torch.Tensor) -> torch.Tensor:
        return t.detach().cpu().contiguous() if t.is_cuda else t

    @staticmethod
    def _back(dst: torch.Tensor, src: torch.Tensor) -> None:
        if dst.data_ptr() != src.data_ptr():
            dst.copy_(src)

    @staticmethod
    def wait(works) -> None:
        for w in works or ():
            if w is not None:
                w.wait()

    # -- collectives ----------------------------------------------------------------------
    def all_gather(self, out: torch.Tensor, inp: torch.Tensor):
        """out = concat over ranks of inp (out may contain inp: in-place all-gather)."""
        _note("all_gather", _bytes(out), _bytes(out))
        if self.rccl:
            return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(ho, self._host(inp).clone(), group=self.group)
        self._back(out, ho)
        return None

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor):
        """out = sum over ranks of inp's block `rank` (blocks of out.shape[0] rows)."""
        _note("reduce_scatter", _bytes(inp), _bytes(inp))
        if self.rccl:
            return dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True)
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(ho, self._host(inp), op=dist.ReduceOp.SUM, group=self.group)
        self._back(out, ho)
        return None

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM):
        _note("all_reduce", _bytes(t), _bytes(t))
        if self.rccl:
            return dist.all_reduce(t, op=op, group=self.group, async_op=True)
        h = self._host(t).clone()
        dist.all_reduce(h, op=op, group=self.group)
        self._back(t, h)
        return None

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        _note("all_to_all", _bytes(inp), _bytes(inp))
        if self.rccl:
            dist.all_to_all_single(out, inp, group=self.group)
            return
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(ho, self._host(inp), group=self.group)
        self._back(out, ho)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, max_rows=None):
        """Uneven all-to-all of rows: inp's blocks of in_splits[q] rows go to rank q, out
        receives out_splits[q] rows from rank q (in rank order).  Async on RCCL.
        max_rows: a bound on every block's rows that ALL ranks pass alike (it fixes the
        number of rounds when the exchange is cut at MAX_MSG_BYTES); default: this rank's
        largest block, which is only safe when no rank's exchange needs cutting."""
        rb = _row_bytes(inp)
        # only the RCCL path cuts (and so depends on the agreed bound); a block past it raises
        # here on the ranks that hold it -- check_block_bound, run when the plan is built, makes
        # every rank raise together before any exchange is posted
        rounds = a2a_rounds(in_splits, out_splits, self.world, rb, max_rows, strict=self.rccl)
        _note("all_to_all", max(sum(b - a for a, b in ins) for ins, _ in rounds) * rb,
              sum(int(v) for v in in_splits) * rb, len(rounds))
        if self.rccl:
            if len(rounds) == 1:
                return dist.all_to_all_single(out, inp, output_split_sizes=[int(v) for v in out_splits],
                                              input_split_sizes=[int(v) for v in in_splits], group=self.group,
                                              async_op=True)
            works = [dist.all_to_all([out[a:b] for a, b in outs], [inp[a:b] for a, b in ins], group=self.group,
                                     async_op=True) for ins, outs in rounds]
            return _Works(works)
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(ho, self._host(inp), output_split_sizes=list(out_splits),
                               input_split_sizes=list(in_splits), group=self.group)
        self._back(out, ho)
        return None

    def check_block_bound(self, biggest: int, max_rows: int) -> None:
        """Collective: raise ValueError on EVERY rank when any rank's largest all-to-all block
        (biggest rows) exceeds the max_rows bound all ranks cut their exchanges by.  A rank
        that raised alone would leave its peers waiting inside the next collective."""
        dev = torch.device("cuda", torch.cuda.current_device()) if self.rccl else torch.device("cpu")
        t = torch.tensor([int(biggest)], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        worst = int(t.item())
        if worst > int(max_rows):
            raise ValueError(f"all_to_all: a block of {worst} rows (some rank) exceeds max_rows={int(max_rows)}")

    def exchange(self, sends, recvs):
        """Grouped point-to-point: sends = [(tensor, peer)], recvs = [(tensor, peer)]."""
        for t, _ in sends:
            pc = p2p_pieces(t.shape[0], _row_bytes(t))
            _note("p2p", max((b - a) for a, b in pc) * _row_bytes(t), _bytes(t), len(pc))
        if self.rccl:
            # messages past MAX_MSG_BYTES go as row pieces, in order (both ends cut alike)
            def pieces(t):
                return [t[a:b] for a, b in p2p_pieces(t.shape[0], _row_bytes(t))]
            ops = [dist.P2POp(dist.isend, p, q, self.group) for t, q in sends for p in pieces(t)]
            ops += [dist.P2POp(dist.irecv, p, q, self.group) for t, q in recvs for p in pieces(t)]
            return dist.batch_isend_irecv(ops) if ops else []
        hs = [(self._host(t), q) for t, q in sends]
        hr = [(torch.empty(t.shape, dtype=t.dtype), t, q) for t, q in recvs]
        ops = [dist.P2POp(dist.isend, t, q, self.group) for t, q in hs]
        ops += [dist.P2POp(dist.irecv, h, q, self.group) for h, _, q in hr]
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        for h, t, _ in hr:
            self._back(t, h)
        return []

    def barrier(self) -> None:
        dist.barrier(group=self.group)


def shutdown() -> None:
    """Tear the process group down on every rank together.  A rank that destroys its gloo
    group while a peer is still busy (rank 0 writing a dump) can die in gloo's teardown
    ('terminate called without an active exception'), so all ranks meet at a barrier first."""
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
