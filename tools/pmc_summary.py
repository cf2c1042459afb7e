#!/usr/bin/env python
"""Summarise rocprofv3 --pmc CSVs: median per (kernel, counter) over dispatches."""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def load(pattern):
    d = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(pattern):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-60:]
            d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    for case in sys.argv[1:]:
        d = load(f"gpurun_out/pmc/{case}_p*/run_counter_collection.csv")
        print(f"=== {case}")
        for k, cs in d.items():
            print(f"  {k}")
            for c, v in sorted(cs.items()):
                print(f"     {c:28s} {statistics.median(v):16.1f}")


if __name__ == "__main__":
    main()
