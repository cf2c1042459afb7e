#!/usr/bin/env python
"""Per-kernel statistics from a rocprofv3 SQLite result (rocprofv3 --kernel-trace writes
<dir>/<name>_results.db on this ROCm): the same columns as rocprofv3's kernel_stats.csv
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev).

  python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--out stats.csv] [--top 30]
"""
import argparse
import csv
import math
import sqlite3
import sys


def kernel_stats(db_path: str) -> list[dict]:
    db = sqlite3.connect(db_path)
    by = {}
    for name, dur in db.execute("select name, duration from kernels"):
        by.setdefault(name, []).append(float(dur))
    total = sum(sum(v) for v in by.values()) or 1.0
    rows = []
    for name, v in by.items():
        n, s = len(v), sum(v)
        mean = s / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        rows.append({"Name": name, "Calls": n, "TotalDurationNs": round(s), "AverageNs": round(mean, 3),
                     "Percentage": round(100 * s / total, 2), "MinNs": round(min(v)), "MaxNs": round(max(v)),
                     "StdDev": round(sd, 3)})
    return sorted(rows, key=lambda r: -r["TotalDurationNs"])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--out", default=None)
    ap.add_argument("--top", type=int, default=0)
    ap.add_argument("--header", default=None, help="a '# ...' comment line written first")
    a = ap.parse_args(argv)
    rows = kernel_stats(a.db)
    if a.top:
        rows = rows[: a.top]
    f = open(a.out, "w", newline="") if a.out else sys.stdout
    if a.header:
        f.write(a.header.rstrip() + "\n")
    w = csv.DictWriter(f, fieldnames=list(rows[0]), quoting=csv.QUOTE_NONNUMERIC)
    w.writeheader()
    w.writerows(rows)
    return 0


if __name__ == "__main__":
    sys.exit(main())
