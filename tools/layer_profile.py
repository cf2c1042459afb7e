#!/usr/bin/env python
"""Per-step device time of a model's forward (eager replay of every step, median over
iters, one MI355X), with each step's kind, tuned (split, cfg), FLOPs and achieved rate,
sorted by time: where the kernel time goes, layer by layer.

  python tools/layer_profile.py [--model xception] [--batch 32] [--iters 20] [--top 40]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="xception")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import torch
    from kdl.engine import registry
    from kdl.engine.tuning import tuning_path
    info = registry.get(a.model)
    p = info.init_params(0)
    e = info.engine(p, a.batch, torch.device("cuda", 0))
    e.load_tuning(tuning_path(info.tuning or a.model, a.batch))
    x = torch.randint(0, 256, tuple(e.inp.shape), dtype=torch.uint8, device="cuda")
    e.inp.copy_(x) if e.inp.dtype == torch.uint8 else e.inp.copy_(x.float() / 127.5 - 1)
    e.forward(e.inp)
    prof = e.profile(a.batch, a.iters)
    steps = {s.name: s for s in e.steps}
    tot = sum(t for _, t in prof)
    rows = []
    for name, ms in prof:
        st = steps.get(name)
        kind = st.kind if st else "?"
        tun = e.tuning().get(name) if hasattr(e, "tuning") else None
        flops = None
        lay = getattr(st, "layer", None) if st else None
        if lay is not None and st.geom:
            H, W, OH, OW = st.geom
            flops = 2.0 * a.batch * OH * OW * lay.n * lay.K
        rows.append((ms, name, kind, tun, flops))
    print(f"{a.model} batch {a.batch}: {len(prof)} steps, eager sum {tot * 1e3:.1f} us", flush=True)
    for ms, name, kind, tun, flops in sorted(rows, reverse=True)[: a.top]:
        rate = f"{flops / (ms * 1e-3) / 1e12:7.1f} TF/s" if flops else " " * 12
        print(f"{name:28s} {kind:6s} {str(tun):12s} {ms * 1e3:8.1f} us {100 * ms / tot:5.1f} % {rate}", flush=True)


if __name__ == "__main__":
    main()
