#!/usr/bin/env python3
"""Per-launch HBM traffic of the hot kernels from rocprofv3 PMC passes.

Usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json>
Each dir holds a `rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace --output-format csv`
run.  FETCH_SIZE/WRITE_SIZE are in KiB.  Correction per MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads (TCC_EA0_RDREQ x 64 B
for 128-B requests), so fetch bytes are reported raw and x2; WRITE_SIZE is exact for
16-B/lane streaming stores.
"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gala-gnn-acceleration-language_amd", "csrc")


def source_digests():
    """sha256 of every kernel source and header the PMC pass ran (bench.py reports a kernel's
    traffic only while the digests of its sources still match)."""
    out = {}
    for f in sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))
                    + [os.path.join(ROOT, "include", "gala_hip.h")]):
        out[os.path.relpath(f, ROOT)] = hashlib.sha256(open(f, "rb").read()).hexdigest()
    return out


def read_counter(d, name):
    vals = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != name:
                continue
            vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch = read_counter(fdir, "FETCH_SIZE")
    write = read_counter(wdir, "WRITE_SIZE")
    digests = source_digests()
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), KiB -> bytes",
           "correction": "hbm_bytes_per_launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
           "kernels": {}}
    for k in set(fetch) | set(write):
        if not (k.startswith("void gala::") or "gala" in k):
            continue
        f = sorted(fetch.get(k, [0.0]))
        w = sorted(write.get(k, [0.0]))
        fm = f[len(f) // 2] * 1024
        wm = w[len(w) // 2] * 1024
        res["kernels"][k] = {"launches": len(f), "fetch_bytes_raw": fm, "write_bytes": wm,
                             "hbm_bytes_per_launch": 2 * fm + wm, "sources_sha256": digests}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
