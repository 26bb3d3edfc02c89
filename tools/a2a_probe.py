#!/usr/bin/env python3
"""Probe: do RCCL's uneven all_to_all_single and reduce_scatter_tensor copy large row blocks
exactly at world 1?  (the sparse vertex-cut exchange diverged at config
5's 11.1 M-row shape on MI355X, the dense reduce-scatter did not.)  Prints one JSON line per
(collective, rows, width): whether the received rows equal the sent rows bit for bit, and
the first mismatching row."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gala-gnn-acceleration-language_amd"))
from gala.comm import Comm  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    comm = Comm()
    for rows in (1_110_599, 2_097_153, 4_194_305, 11_105_995):
        x = torch.arange(rows, device="cuda", dtype=torch.float32).view(-1, 1).repeat(1, W)
        x += torch.arange(W, device="cuda", dtype=torch.float32).view(1, -1) * 1e-3
        for name in ("a2a_split", "a2a_even", "reduce_scatter", "all_gather", "p2p_self", "comm_a2a", "comm_p2p"):
            out = torch.full_like(x, -1.0)
            t0 = time.time()
            if name == "a2a_split":
                dist.all_to_all_single(out, x, output_split_sizes=[rows], input_split_sizes=[rows])
            elif name == "a2a_even":
                dist.all_to_all_single(out, x)
            elif name == "reduce_scatter":
                dist.reduce_scatter_tensor(out, x)
            elif name == "all_gather":
                dist.all_gather_into_tensor(out, x)
            elif name == "p2p_self":
                for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, x, 0), dist.P2POp(dist.irecv, out, 0)]):
                    w.wait()
            elif name == "comm_a2a":   # gala.comm: cut into rounds of at most MAX_MSG_BYTES
                comm.all_to_all(out, x, [rows], [rows], max_rows=rows).wait()
            else:
                for w in comm.exchange([(x, 0)], [(out, 0)]):
                    w.wait()
            torch.cuda.synchronize()
            ok = bool(torch.equal(out, x))
            rec = {"op": name, "rows": rows, "W": W, "bytes": rows * W * 4, "equal": ok,
                   "s": round(time.time() - t0, 4)}
            if not ok:
                bad = (out != x).any(1).nonzero().view(-1)
                rec["bad_rows"] = int(bad.numel())
                rec["first_bad_row"] = int(bad[0])
                rec["last_bad_row"] = int(bad[-1])
            print(json.dumps(rec), flush=True)
            del out
        del x
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
