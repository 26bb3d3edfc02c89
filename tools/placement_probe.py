#!/usr/bin/env python3
"""Does where a gathered table lands decide the gather rate?  The same-process gather probe
(tools/libgala_probe.so: X[col[e]] for the Products-shaped uniform graph's 126 M edges, F =
256, a 2.5 GB table) on several copies of the same table allocated at different points of the
process, under torch's default caching allocator and (child process) with
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True.  One JSON line per (allocator, copy): probe
ms, 10 calls, 3 alternated rounds.  Measurement only.   python tools/placement_probe.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(tag):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "gala-gnn-acceleration-language_amd"))
    sys.path.insert(0, ROOT)
    import bench
    from gala import ops
    hg = bench.products_graph("uniform", 1.0)
    dg = ops.DeviceGraph.from_host(hg)
    N, F = hg.n_rows, 256
    timer = bench.Timer(True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    tabs = {"first": torch.rand((N, F), device="cuda", generator=gen)}
    pad = torch.empty(3 << 28, dtype=torch.uint8, device="cuda")   # 768 MB between copies
    tabs["after_pad"] = tabs["first"].clone()
    del pad
    tabs["in_freed_gap"] = tabs["first"].clone()
    big = torch.empty(40 << 30, dtype=torch.uint8, device="cuda")  # 40 GB, then a copy past it
    tabs["past_40GB"] = tabs["first"].clone()
    del big
    bench.gather_ceiling(dg.col, tabs["first"], timer, reps=3)    # warm-up
    res = {k: [] for k in tabs}
    for _ in range(3):
        for k, X in tabs.items():
            res[k].append(bench.gather_ceiling(dg.col, X, timer) * 1e3)
    for k, v in res.items():
        print(json.dumps({"allocator": tag, "copy": k, "ptr_mod_2MB": tabs[k].data_ptr() % (2 << 20),
                          "probe_ms": [round(x, 3) for x in v]}), flush=True)


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    for tag, extra in (("caching", {}), ("expandable_segments", {"PYTORCH_HIP_ALLOC_CONF": "expandable_segments:True"}),
                       ("caching", {})):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), tag], env=dict(os.environ, **extra),
                           capture_output=True, text=True, timeout=600)
        sys.stdout.write(r.stdout)
        if r.returncode:
            print(json.dumps({"allocator": tag, "rc": r.returncode, "stderr": r.stderr[-1500:]}))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
