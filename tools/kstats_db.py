#!/usr/bin/env python
"""Kernel statistics (rocprofv3 --kernel-trace, rocpd sqlite DB, ROCm 7) in the column layout
of rocprofv3's kernel_stats.csv: Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs,
MaxNs, StdDev -- sorted by total time.  python tools/kstats_db.py <results.db> [out.csv]"""
import csv
import shutil
import sqlite3
import subprocess
import statistics
import sys
from collections import defaultdict


def demangle(names: list[str]) -> list[str]:
    """Itanium-demangle code-object symbols (``_ZN...E.kd``) with c++filt when available."""
    tool = shutil.which("c++filt") or shutil.which("llvm-cxxfilt")
    raw = [n[:-3] if n.endswith(".kd") else n for n in names]
    if not tool or not raw:
        return raw
    out = subprocess.run([tool], input="\n".join(raw), capture_output=True, text=True).stdout.splitlines()
    return out if len(out) == len(raw) else raw


def kernel_stats(db: str) -> list[list]:
    c = sqlite3.connect(db)
    rows = list(c.execute("select id, kernel_name from rocpd_info_kernel_symbol"))
    kname = dict(zip([r[0] for r in rows], demangle([r[1] for r in rows])))
    dur = defaultdict(list)
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        dur[kname.get(kid, str(kid))].append(e - s)
    tot = sum(sum(v) for v in dur.values()) or 1
    rows = []
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        rows.append([k, len(v), sum(v), round(sum(v) / len(v), 3), round(100 * sum(v) / tot, 3), min(v), max(v),
                     round(statistics.pstdev(v), 3)])
    return rows


def main() -> int:
    rows = kernel_stats(sys.argv[1])
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    w.writerows(rows)
    return 0


if __name__ == "__main__":
    sys.exit(main())
