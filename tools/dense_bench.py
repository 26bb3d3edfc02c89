#!/usr/bin/env python3
"""GPU: FFN weight/bias gradient kernel (gala_dense_grad_f32) vs torch (mm + sum(0)) on the
generated programs' shapes.  Prints one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gala-gnn-acceleration-language_amd"))
from gala import ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    shapes = [(2449029, 100, 32), (2449029, 32, 47), (2449029, 32, 1), (2449029, 47, 1), (232965, 602, 256),
              (232965, 256, 41), (169343, 128, 128), (11105995, 128, 128), (11105995, 128, 172)]
    for N, K, M in shapes:
        X = torch.rand(N, K, device="cuda")
        dY = torch.rand(N, M, device="cuda")
        t_gala = timed(lambda: ops.dense_grad(X, dY))
        t_torch = timed(lambda: (dY.t().mm(X), dY.sum(0)))
        byts = 4 * N * (K + M)
        line = {"N": N, "K": K, "M": M, "gala_ms": round(t_gala, 4), "torch_ms": round(t_torch, 4),
                "gala_GBps": round(byts / t_gala / 1e6, 1)}
        W = torch.rand(M, K, device="cuda")  # forward Y = X W^T + b, where supported
        b = torch.rand(M, device="cuda")
        try:
            line["fwd_gala_ms"] = round(timed(lambda: ops.ffn_fwd(X, W, b)), 4)
            line["fwd_torch_ms"] = round(timed(lambda: torch.addmm(b, X, W.t())), 4)
        except Exception:
            pass
        print(json.dumps(line), flush=True)
        del X, dY


if __name__ == "__main__":
    main()
