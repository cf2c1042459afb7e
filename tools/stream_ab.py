#!/usr/bin/env python
"""A/B of the streaming pointwise GEMM (STREAM_BASE, and STREAM_NT with nontemporal stores;
gemm_stream.hip) against each layer's tuned
config on every eligible conv of a model (isolated launches, median of --reps timings of --iters
launches each), with the effective HBM rate (x + y + residual bytes) of both.

  python tools/stream_ab.py [--model efficientnet_b7] [--batch 32] [--write tuning.json]
--write: a copy of the model's tuning with the faster stream id on every layer where it won by > 3 %.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="efficientnet_b7")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--write", default=None)
    a = ap.parse_args()
    import torch
    from kdl.engine import registry
    from kdl.engine.tuning import tuning_path
    from kdl.ops.conv import MODE_DW, STREAM_BASE, STREAM_NT
    info = registry.get(a.model)
    e = info.engine(info.init_params(0), a.batch, torch.device("cuda", 0))
    tp = tuning_path(info.tuning or a.model, a.batch)
    e.load_tuning(tp)
    e.forward(torch.randint(0, 256, tuple(e.inp.shape), dtype=torch.uint8, device="cuda"))
    s = e.stream
    tun = e.tuning()
    new = dict(tun)
    tot_old = tot_new = 0.0

    def timeit(step, cfg, split):
        ts = []
        with torch.cuda.stream(s):
            for _ in range(2):
                e._emit_conv(None, step, a.batch, split=split, cfg=cfg)
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.iters):
                    e._emit_conv(None, step, a.batch, split=split, cfg=cfg)
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / a.iters)
        return statistics.median(ts)

    for step in e.conv_steps():
        lay = step.layer
        if not getattr(lay, "stream_ok", lambda: False)():
            continue
        ssplit = lay.mode == MODE_DW          # separable convs: the stream GEMM runs as their split lowering
        H, W, OH, OW = step.geom
        M = a.batch * OH * OW
        nbytes = 2 * M * (step.extra.get("ldx", lay.cin_pad) + lay.ldy * (2 if step.res else 1))
        if step.res and not lay.stream_ok(res=True):
            continue
        t0 = timeit(step, lay.cfg, lay.split)
        t1 = timeit(step, STREAM_BASE, ssplit)
        t2 = timeit(step, STREAM_NT, ssplit)
        best, tb = min(((STREAM_BASE, t1), (STREAM_NT, t2)), key=lambda x: x[1])
        tot_old += t0
        tot_new += min(t0, tb)
        if tb < 0.97 * t0:
            new[step.name] = [int(ssplit), best]
        print(f"{step.name:26s} M {M:8d} K {lay.K:4d} ldy {lay.ldy:4d} cfg {lay.cfg:4d} {t0:7.1f} us "
              f"({nbytes / t0 / 1e6:5.2f} TB/s)  stream {t1:7.1f} us ({nbytes / t1 / 1e6:5.2f} TB/s)  "
              f"nt {t2:7.1f} us ({nbytes / t2 / 1e6:5.2f} TB/s)  {t0 / tb:5.2f}x", flush=True)
    print(f"eligible layers: tuned {tot_old:.0f} us -> best-of {tot_new:.0f} us "
          f"({tot_old - tot_new:.0f} us saved per batch of {a.batch})", flush=True)
    if a.write:
        with open(a.write, "w") as f:
            json.dump(new, f, indent=1)
        print(f"wrote {a.write} ({sum(1 for k in new if new[k] != tun.get(k))} layers on the streaming GEMM)")


if __name__ == "__main__":
    main()
