#!/usr/bin/env python
"""Summarise a rocprofv3 --pmc sqlite results DB (rocpd schema, ROCm 7): median counter value
per (kernel, counter) over dispatches, plus the median dispatch duration."""
import sqlite3
import statistics
import sys
from collections import defaultdict


def summarise(db: str, match: str = "") -> None:
    c = sqlite3.connect(db)
    kname = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    pname = {r[0]: r[1] for r in c.execute("select id, name from rocpd_info_pmc")}
    vals = defaultdict(lambda: defaultdict(list))
    q = ("select d.kernel_id, p.pmc_id, p.value from rocpd_pmc_event p "
         "join rocpd_kernel_dispatch d on d.event_id = p.event_id")
    try:
        rows = list(c.execute(q))
    except sqlite3.OperationalError:
        rows = []
    for kid, pid, v in rows:
        vals[kname.get(kid, str(kid))][pname.get(pid, str(pid))].append(v)
    dur = defaultdict(list)
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        dur[kname.get(kid, str(kid))].append((e - s) / 1e3)
    for k, cs in vals.items():
        if match and match not in k:
            continue
        print(f"  {k.split('(')[0][-70:]}  median {statistics.median(dur[k]):.1f} us over {len(dur[k])} dispatches")
        for n, v in sorted(cs.items()):
            print(f"     {n:28s} {statistics.median(v):16.1f}")


if __name__ == "__main__":
    for db in sys.argv[1:]:
        print(f"=== {db}")
        summarise(db, "attn")
