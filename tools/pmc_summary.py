#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 runs (kernel-trace --stats dir + PMC dirs): average
duration, per-dispatch counter averages, VGPR count, and HBM bytes per launch with the
gfx950 FETCH_SIZE correction (x2, MI355X_MICROARCH.md §HBM).

Usage: pmc_summary.py <out.json> <trace_dir> <pmc_dir> [<pmc_dir> ...]
Only kernels whose name contains 'gala' are kept."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    out, trace, pmcs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(trace, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "gala" in r["Name"]:
                res[short(r["Name"])].update(calls=int(r["Calls"]), avg_ms=float(r["AverageNs"]) / 1e6)
    for d in pmcs:
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "gala" not in r["Kernel_Name"]:
                    continue
                k = short(r["Kernel_Name"])
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                res[k]["vgpr"] = int(r["VGPR_Count"])
        for k, cs in vals.items():
            for c, v in cs.items():
                res[k][c] = sum(v) / len(v)
    for k, v in res.items():
        if "FETCH_SIZE" in v or "WRITE_SIZE" in v:
            v["hbm_bytes_per_launch"] = 2 * v.get("FETCH_SIZE", 0) * 1024 + v.get("WRITE_SIZE", 0) * 1024
    doc = {"source": "rocprofv3 --kernel-trace --stats and separate --pmc passes; counters are per-dispatch "
                     "averages; FETCH_SIZE/WRITE_SIZE in KiB, hbm_bytes_per_launch = 2*FETCH + WRITE (gfx950)",
           "kernels": res}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
