#!/usr/bin/env python
"""Timeline summary of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

For the stage-pipelined bench (two compute streams running different layers of
consecutive batches) the per-kernel stats do not say which stage bounds the step.
This reads ``*kernel_trace.csv``, keeps the last ``--window-ms`` of the trace (the
timed steady state), and prints per stream: busy time (union of its kernel
intervals) as a share of the wall window, its idle gaps, the time both streams
are busy at once, and the kernels that own most of each stream's busy time.

    python tools/trace_timeline.py gpurun_out/trace [--window-ms 200]
"""
from __future__ import annotations

import argparse
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def _union(iv: list[tuple[int, int]]) -> list[tuple[int, int]]:
    out: list[list[int]] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [(a, b) for a, b in out]


def _length(iv) -> int:
    return sum(b - a for a, b in iv)


def _intersect(x, y) -> int:
    i = j = tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def _short(name: str) -> str:
    m = re.search(r"kdl(?:\d+)?([a-z0-9_]+?_kernel)", name)
    return m.group(1) if m else name[:60]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path", type=Path)
    ap.add_argument("--window-ms", type=float, default=200.0)
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args(argv)
    files = sorted(a.path.rglob("*kernel_trace.csv")) if a.path.is_dir() else [a.path]
    if not files:
        print(f"no *kernel_trace.csv under {a.path}", file=sys.stderr)
        return 1
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = r.get("Stream_Id") or r.get("Queue_Id") or "0"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), key, r["Kernel_Name"]))
    t_end = max(r[1] for r in rows)
    t0 = t_end - int(a.window_ms * 1e6)
    rows = [r for r in rows if r[0] >= t0]
    wall = t_end - min(r[0] for r in rows)
    by_stream: dict[str, list] = defaultdict(list)
    for s, e, key, name in rows:
        by_stream[key].append((s, e, name))
    unions = {k: _union([(s, e) for s, e, _ in v]) for k, v in by_stream.items()}
    allu = _union([iv for u in unions.values() for iv in u])
    print(f"window {wall / 1e6:.2f} ms, {len(rows)} kernels, {len(by_stream)} streams; "
          f"some stream busy {100 * _length(allu) / wall:.1f} %")
    keys = sorted(by_stream, key=lambda k: -_length(unions[k]))
    for k in keys:
        v = by_stream[k]
        busy = _length(unions[k])
        per = defaultdict(int)
        for s, e, name in v:
            per[_short(name)] += e - s
        top = sorted(per.items(), key=lambda kv: -kv[1])[:a.top]
        gaps = [b0 - a1 for (a0, a1), (b0, b1) in zip(unions[k], unions[k][1:])]
        gaps.sort()
        med_gap = gaps[len(gaps) // 2] / 1e3 if gaps else 0.0
        print(f"stream {k}: {len(v)} kernels, busy {busy / 1e6:.2f} ms = {100 * busy / wall:.1f} % of wall, "
              f"sum of durations {sum(e - s for s, e, _ in v) / 1e6:.2f} ms, median gap {med_gap:.1f} us")
        for name, t in top:
            print(f"    {name:40s} {t / 1e6:8.3f} ms  {100 * t / busy:5.1f} %")
    if len(keys) >= 2:
        both = _intersect(unions[keys[0]], unions[keys[1]])
        print(f"streams {keys[0]} and {keys[1]} both busy {100 * both / wall:.1f} % of wall")
    return 0


if __name__ == "__main__":
    sys.exit(main())
