#!/usr/bin/env python
"""HBM ceilings on this device for the streaming-GEMM byte mixes: write-only (fill), read-only
(sum), read+write (copy) at a few sizes, median of --reps timings (GB/s = bytes / time).

  python tools/hbm_probe.py [--mb 1106 207 507] [--reps 10]
"""
import argparse
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, nargs="+", default=[1106.0, 415.0, 173.0])
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch

    def t(fn):
        fn()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        return statistics.median(ts)

    for mb in a.mb:
        n = int(mb * 1e6) // 2
        x = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        y = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        x.fill_(1.0)
        acc = torch.empty((), dtype=torch.float32, device="cuda")
        tw = t(lambda: x.fill_(0.5))
        tr = t(lambda: torch.sum(x, dim=(0,), dtype=torch.float32, out=acc))
        tc = t(lambda: y.copy_(x))
        b = 2 * n
        print(f"{mb:8.0f} MB  write {b / tw / 1e12:5.2f} TB/s  read {b / tr / 1e12:5.2f} TB/s  "
              f"copy {2 * b / tc / 1e12:5.2f} TB/s (r+w)", flush=True)


if __name__ == "__main__":
    main()
