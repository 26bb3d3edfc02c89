#!/usr/bin/env python3
"""Top-kernel summary (name, calls, total_ms, avg_us, percent) of a rocprofv3 rocpd
database (rocprofv3 --kernel-trace --stats writes <name>_results.db on this image).

    python tools/rocpd_top.py gpurun_out/prof/x_results.db [N] > profiles/rNN_x_top.csv
"""
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name) if not name.startswith("Cijk") else name[:48]
    return name[:160]


def main() -> int:
    db, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30
    c = sqlite3.connect(db)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_ms", "avg_us", "percent"])  # rocpd durations are in us
    for name, calls, total, avg, pct in c.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels "
            "order by total_duration desc limit ?", (n,)):
        w.writerow([short(name), calls, f"{total / 1000:.3f}", f"{avg:.1f}", f"{pct:.2f}"])
    return 0


if __name__ == "__main__":
    sys.exit(main())
