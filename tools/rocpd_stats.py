"""Kernel statistics (the rocprofv3 --stats table) from a rocprofv3 rocpd SQLite database.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--top 40] > profiles/x.csv
"""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--header", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on s.id = d.kernel_id").fetchall()
    by = {}
    for name, dur in rows:
        by.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in by.values())
    if a.header:
        print(f"# {a.header}")
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","MedianNs"')
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        s = sum(v)
        print(f'"{name}",{len(v)},{s},{s / len(v):.1f},{100 * s / total:.3f},{min(v)},{max(v)},{statistics.median(v):.0f}')


if __name__ == "__main__":
    main()
