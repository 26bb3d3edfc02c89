#!/usr/bin/env python3
"""Merge one PMC traffic summary (tools/pmc_traffic.py output) into profiles/traffic.json.

Usage: merge_traffic.py SRC.json SOURCE_NOTE [PREFIX]
Every kernel of SRC replaces the entry of the same name (PREFIX + name when given: the
banded and R-MAT families run the headline's row kernel, so their entries are kept apart as
"banded|<name>" / "rmat|<name>"), tagged with SOURCE_NOTE.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, note = sys.argv[1], sys.argv[2]
    prefix = sys.argv[3] if len(sys.argv) > 3 else ""
    dst = os.path.join(ROOT, "profiles", "traffic.json")
    d = json.load(open(dst))
    for k, v in json.load(open(src))["kernels"].items():
        d["kernels"][prefix + k] = dict(v, source=note)
    json.dump(d, open(dst, "w"), indent=1)
    print(f"merged {len(json.load(open(src))['kernels'])} kernels into {dst}")


if __name__ == "__main__":
    main()
