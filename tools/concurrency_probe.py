#!/usr/bin/env python
"""Probe: does splitting a batch across concurrent streams fill the chip better?
Also times hipBLASLt (torch.matmul) on the middle-flow GEMM shape for reference."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from kdl.engine.tuning import tuning_path  # noqa: E402
from kdl.engine.xception import XceptionEngine  # noqa: E402
from kdl.models import xception as X  # noqa: E402


def timeit(fn, iters=40, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    p = X.init_params(seed=0)
    dev = torch.device("cuda", 0)
    res = {}
    e32 = XceptionEngine(p, max_batch=32, device=dev)
    e32.load_tuning(tuning_path("xception", 32))
    res["1x32"] = timeit(lambda: e32.launch(32))
    engs = []
    for n, b in ((2, 16), (4, 8)):
        es = [XceptionEngine(p, max_batch=b, device=dev) for _ in range(n)]
        tp = tuning_path("xception", b)
        if tp.exists():
            es[0].load_tuning(tp)
        else:
            es[0].autotune(b)
        for e in es[1:]:
            e.load_tuning_dict(es[0].tuning()) if hasattr(e, "load_tuning_dict") else None
        engs.append(es)
        for e in es:
            for s0, s1 in zip(es[0].conv_steps(), e.conv_steps()):
                s1.layer.split, s1.layer.cfg = s0.layer.split, s0.layer.cfg
            e.invalidate()

        def run(es=es, b=b):
            for e in es:
                e.launch(b)
        res[f"{n}x{b}"] = timeit(run)
        res[f"1x{b}"] = timeit(lambda: es[0].launch(b))
    e2 = XceptionEngine(p, max_batch=32, device=dev)
    for s0, s1 in zip(e32.conv_steps(), e2.conv_steps()):
        s1.layer.split, s1.layer.cfg = s0.layer.split, s0.layer.cfg

    def run2():
        e32.launch(32)
        e2.launch(32)
    res["2x32"] = timeit(run2)
    for k, v in res.items():
        n, b = map(int, k.split("x"))
        print(f"{k:6s} {v:7.3f} ms/step  {n * b / v * 1e3:9.0f} img/s")
    a = torch.randn(11552, 736, device=dev, dtype=torch.bfloat16)
    w = torch.randn(736, 728, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: a @ w, iters=200)
    print(f"hipBLASLt 11552x736x728: {t * 1e3:.1f} us  {2 * 11552 * 736 * 728 / t / 1e9:.0f} TFLOP/s")
    a = torch.randn(11552 * 4, 736, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: a @ w, iters=100)
    print(f"hipBLASLt 46208x736x728: {t * 1e3:.1f} us  {2 * 46208 * 736 * 728 / t / 1e9:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
