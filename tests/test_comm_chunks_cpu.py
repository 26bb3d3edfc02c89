"""CPU: gala.comm's message cutting.  RCCL 2.26.6 corrupts all-to-all and point-to-point
payloads past 1 GiB (profiles/r04_rccl_a2a_probe.jsonl), so every RCCL all-to-all is cut
into rounds and every p2p message into row pieces of at most MAX_MSG_BYTES.

The cutting plans (gala.comm.a2a_rounds / p2p_pieces, what Comm.all_to_all and Comm.exchange
issue over RCCL) are checked by playing every rank's rounds against each other: in every
round the block rank p sends to rank q has exactly the rows q posts for p, every round's
message stays within the cap, and the assembled outputs equal the uncut exchange -- uneven
splits, empty blocks, a rank with nothing to send, ranks whose own blocks need fewer rounds
than the shared bound.
"""
import numpy as np
import pytest

from gala import comm as gcomm


def _play(splits, row_bytes, cap, max_rows):
    world = splits.shape[0]
    old = gcomm.MAX_MSG_BYTES
    gcomm.MAX_MSG_BYTES = cap
    try:
        plans = [gcomm.a2a_rounds(splits[p], splits[:, p], world, row_bytes, max_rows) for p in range(world)]
    finally:
        gcomm.MAX_MSG_BYTES = old
    assert len({len(pl) for pl in plans}) == 1            # every rank issues the same collectives
    F = 3
    inputs = []
    for p in range(world):
        n = int(splits[p].sum())
        inputs.append(np.arange(n * F).reshape(n, F) + 10_000 * p)
    outs = [np.full((int(splits[:, p].sum()), F), -1) for p in range(world)]
    for j in range(len(plans[0])):
        sent = 0
        for p in range(world):
            ins, _ = plans[p][j]
            sent = max(sent, sum(b - a for a, b in ins) * row_bytes)
            for q in range(world):
                a, b = ins[q]
                oa, ob = plans[q][j][1][p]
                assert b - a == ob - oa                      # sender and receiver agree
                outs[q][oa:ob] = inputs[p][a:b]
        assert sent <= max(cap, world * row_bytes)           # one round's message within the cap
    for q in range(world):                                   # the uncut exchange
        want = [inputs[p][int(splits[p, :q].sum()):int(splits[p, :q + 1].sum())] for p in range(world)]
        np.testing.assert_array_equal(outs[q], np.concatenate(want))
    return len(plans[0])


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("seed", range(4))
def test_all_to_all_rounds_play_out_as_the_uncut_exchange(world, seed):
    rng = np.random.default_rng(seed)
    splits = rng.integers(0, 40, (world, world))
    if world > 2:
        splits[2, :] = 0                 # a rank that sends nothing
        splits[0, 1] = 0                 # an empty block
    rb = 12                              # bytes per row
    m = int(splits.max())
    # uncut: one round
    assert _play(splits, rb, 1 << 30, m) == 1
    # cut to about 3 rows per peer and round: many rounds, the count from the shared bound
    n = _play(splits, rb, 3 * rb * world, m)
    assert n == max(-(-m // 3), 1)
    # a cap below one row per peer still moves one row per peer and round
    assert _play(splits, rb, 1, m) == max(m, 1)


def test_p2p_pieces_cover_the_message_in_order():
    old = gcomm.MAX_MSG_BYTES
    try:
        gcomm.MAX_MSG_BYTES = 5 * 16
        for rows in (0, 1, 4, 5, 6, 23):
            pieces = gcomm.p2p_pieces(rows, 16)
            assert pieces[0][0] == 0 and pieces[-1][1] == rows
            assert all(b - a <= 5 for a, b in pieces) or rows <= 5
            assert all(p[1] == n[0] for p, n in zip(pieces, pieces[1:]))
        gcomm.MAX_MSG_BYTES = 1 << 30
        assert gcomm.p2p_pieces(1 << 20, 128) == [(0, 1 << 20)]
        assert len(gcomm.p2p_pieces(3 << 20, 1024)) == 3     # 3 GiB of 1-KB rows: 3 pieces
    finally:
        gcomm.MAX_MSG_BYTES = old


def _bound_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    from gala.comm import Comm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = Comm()
        c.check_block_bound(5, 8)                       # every block within the bound: no error
        try:                                            # only rank 1 holds a block past it
            c.check_block_bound(12 if rank == 1 else 3, 8)
            q.put((rank, "no error"))
        except ValueError as e:
            q.put((rank, str(e)))
        # the uncut (gloo) exchange records a plan past the bound instead of refusing it
        rounds = gcomm.a2a_rounds([12, 3, 0], [3, 3, 3], world, 4, max_rows=8, strict=False)
        assert len(rounds) == 1
        dist.barrier()
    finally:
        dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)


def test_block_bound_raises_on_every_rank():
    """a2a_rounds refused an oversize block only on the ranks that held it, so its
    peers went on into the all-to-all and hung.  Comm.check_block_bound (run when a sparse
    vertex-cut plan is built) all-reduces the largest block: every rank raises together."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bound_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(got) == [0, 1, 2]
    assert all("12 rows" in v and "max_rows=8" in v for v in got.values()), got
    with pytest.raises(ValueError):
        gcomm.a2a_rounds([12, 3], [3, 3], 2, 4, max_rows=8)
