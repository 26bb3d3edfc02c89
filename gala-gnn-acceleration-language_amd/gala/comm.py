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
        if self.rccl:
            return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(ho, self._host(inp).clone(), group=self.group)
        self._back(out, ho)
        return None

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor):
        """out = sum over ranks of inp's block `rank` (blocks of out.shape[0] rows)."""
        if self.rccl:
            return dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True)
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(ho, self._host(inp), op=dist.ReduceOp.SUM, group=self.group)
        self._back(out, ho)
        return None

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM):
        if self.rccl:
            return dist.all_reduce(t, op=op, group=self.group, async_op=True)
        h = self._host(t).clone()
        dist.all_reduce(h, op=op, group=self.group)
        self._back(t, h)
        return None

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if self.rccl:
            dist.all_to_all_single(out, inp, group=self.group)
            return
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(ho, self._host(inp), group=self.group)
        self._back(out, ho)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        """Uneven all-to-all of rows: inp's blocks of in_splits[q] rows go to rank q, out
        receives out_splits[q] rows from rank q (in rank order).  Async on RCCL."""
        if self.rccl:
            return dist.all_to_all_single(out, inp, output_split_sizes=list(out_splits),
                                          input_split_sizes=list(in_splits), group=self.group, async_op=True)
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(ho, self._host(inp), output_split_sizes=list(out_splits),
                               input_split_sizes=list(in_splits), group=self.group)
        self._back(out, ho)
        return None

    def exchange(self, sends, recvs):
        """Grouped point-to-point: sends = [(tensor, peer)], recvs = [(tensor, peer)]."""
        if self.rccl:
            ops = [dist.P2POp(dist.isend, t, q, self.group) for t, q in sends]
            ops += [dist.P2POp(dist.irecv, t, q, self.group) for t, q in recvs]
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
