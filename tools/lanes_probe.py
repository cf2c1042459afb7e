#!/usr/bin/env python
"""Split-batch concurrency probe: one batch-32 graph vs two batch-16 graphs
replayed on two streams at once (independent engines, same weights). Tells
whether the latency-bound small layers leave enough of the chip idle for a
second lane to fill."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from kdl.engine import registry  # noqa: E402
from kdl.engine.tuning import tuning_path  # noqa: E402


def timeit(fn, iters, streams):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in streams:
        s.wait_event(e0)
    for _ in range(iters):
        fn()
    for s in streams:
        torch.cuda.current_stream().wait_stream(s)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="xception")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--lanes", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    info = registry.get(a.model)
    params = info.init_params(0)
    B = 32
    big = info.engine(params, B, dev)
    tp = tuning_path(a.model, B)
    big.load_tuning(tp) if tp.exists() else big.autotune(B)
    t32 = timeit(lambda: big.launch(B), a.iters, [big.stream])
    print(f"one lane  b32: {t32 * 1e3:8.1f} us/batch  {B / t32 * 1e3:8.0f} img/s", flush=True)
    for nl in (2, 4):
        b = B // nl
        lanes = [info.engine(params, b, dev) for _ in range(nl)]
        tpb = tuning_path(a.model, b)
        for i, e in enumerate(lanes):
            if tpb.exists():
                e.load_tuning(tpb)
            elif i == 0:
                e.autotune(b)
            else:
                e.apply_tuning(lanes[0].tuning())
        t1 = timeit(lambda: lanes[0].launch(b), a.iters, [lanes[0].stream])
        print(f"one lane  b{b}: {t1 * 1e3:8.1f} us/batch", flush=True)
        tl = timeit(lambda: [e.launch(b) for e in lanes], a.iters, [e.stream for e in lanes])
        print(f"{nl} lanes x b{b}: {tl * 1e3:8.1f} us per {B} images  {B / tl * 1e3:8.0f} img/s", flush=True)
        # same b32-tuned tile choices on the lanes (autotune at b16 times layers alone)
        for e in lanes:
            e.apply_tuning(big.tuning())
        tl2 = timeit(lambda: [e.launch(b) for e in lanes], a.iters, [e.stream for e in lanes])
        print(f"{nl} lanes x b{b} (b32 tiles): {tl2 * 1e3:8.1f} us  {B / tl2 * 1e3:8.0f} img/s", flush=True)
        del lanes


if __name__ == "__main__":
    main()
