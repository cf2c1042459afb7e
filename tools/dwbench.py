#!/usr/bin/env python
"""Depthwise-3x3 kernel sweep on the Xception shapes (batch 32): checks numerics
vs torch fp32 and times the host heuristic plus explicit (cg, rb, tw, seg) tiles."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from kdl.ops import _lib  # noqa: E402

SHAPES = {  # name: (H, W, C, relu_in)
    "b2s1": (147, 147, 64, 0), "b2s2": (147, 147, 128, 0), "b3s1": (74, 74, 128, 1),
    "b3s2": (74, 74, 256, 0), "b4s1": (37, 37, 256, 1), "b4s2": (37, 37, 736, 0),
    "mid": (19, 19, 736, 1), "b14s1": (10, 10, 1024, 0), "b14s2": (10, 10, 1536, 0),
}


def ref(x, w, relu):
    B, H, W, C = x.shape
    xf = x.float().permute(0, 3, 1, 2)
    if relu:
        xf = xf.relu()
    k = w.t().reshape(C, 1, 3, 3)
    return F.conv2d(F.pad(xf, (1, 1, 1, 1)), k, groups=C).permute(0, 2, 3, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--direct", action="store_true",
                    help="also time + check the direct row-streaming kernel (algo 2) over (seg, rb, pd)")
    a = ap.parse_args()
    C_ = _lib.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    for name in a.shapes.split(","):
        H, W, C, relu = SHAPES[name]
        B = a.batch
        x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(9, C, device=dev) * 0.3).float().contiguous()
        y = torch.empty_like(x)
        base = dict(x=x.data_ptr(), w=w.data_ptr(), y=y.data_ptr(), B=B, H=H, W=W, C=C, relu_in=relu)

        def run(**kw):
            C_.dw3x3({**base, **kw}, s)

        def tm(**kw):
            for _ in range(3):
                run(**kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run(**kw)
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / 20 * 1e3
        run()
        r = ref(x, w, relu)
        err = ((y.float() - r).abs().max() / r.abs().max()).item()
        t = tm()
        gb = 2 * B * H * W * C * 2 / 1e9
        print(f"{name:6s} B{B} {H}x{W}x{C}: auto {t:7.1f} us  {gb / t * 1e6 / 1e3:5.2f} TB/s  err {err:.2e}",
              flush=True)
        assert err < 1e-2, err
        if a.direct:
            res = []
            for seg in (2, 3, 4):
                for rb in (0, 2, 3, 4, 5, 7, 10, 19, 37):
                    for pd in (1, 2):
                        if rb > H:
                            continue
                        kw = dict(algo=2, seg=seg, rb=rb, pd=pd)
                        y.zero_()
                        run(**kw)
                        e2 = ((y.float() - r).abs().max() / r.abs().max()).item()
                        assert e2 < 1e-2, (kw, e2)
                        res.append((tm(**kw), kw))
            res.sort(key=lambda q: q[0])
            d0 = [q for q in res if q[1]["rb"] == 0 and q[1]["pd"] == 1]
            print(f"    direct default-rb: " + "  ".join(f"seg{q[1]['seg']} {q[0]:.1f}" for q in d0), flush=True)
            for q in res[:4]:
                print(f"    direct {q[0]:7.1f} us {gb / q[0] * 1e3:5.2f} TB/s  {q[1]}", flush=True)
        if not a.sweep:
            continue
        C8 = C // 8
        best = []
        tws = sorted({W, (W + 1) // 2, (W + 2) // 3, (W + 3) // 4} - {0})
        for cg in [d for d in (4, 7, 8, 13, 16) if C8 % d == 0]:
            for tw in tws:
                for seg in (5, 7):
                    for rb in (2, 4, 6, 8, 10, 12, 16, 19):
                        if rb > H or (9 * cg * 32 + (rb + 2) * (tw + 2) * cg * 16) > 96 * 1024:
                            continue
                        try:
                            tt = tm(cg=cg, rb=rb, tw=tw, seg=seg)
                        except RuntimeError:
                            continue
                        best.append((tt, cg, rb, tw, seg))
        best.sort()
        for b_ in best[:5]:
            print(f"    {b_[0]:7.1f} us  cg={b_[1]} rb={b_[2]} tw={b_[3]} seg={b_[4]}", flush=True)


if __name__ == "__main__":
    main()
