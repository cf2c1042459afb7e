#!/usr/bin/env python
"""Max-pool 3x3/2 TF-same + residual add on the Xception shapes (batch 32): the
pixel-per-thread kernel (algo 1) vs the row-streaming kernel (algo 2) over (seg, rb),
every config numerics-checked against the fp32 reference."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from kdl.models.layers import tf_same_pad  # noqa: E402
from kdl.ops import _lib  # noqa: E402
from kdl.ops.reference import pool_add_ref  # noqa: E402

SHAPES = {"b2": (147, 128), "b3": (74, 256), "b4": (37, 736), "b13": (19, 1024)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    C_ = _lib.lib()
    s = torch.cuda.current_stream().cuda_stream
    B = a.batch
    for name, (H, C) in SHAPES.items():
        OH, pt, _ = tf_same_pad(H, 3, 2)
        x = torch.randn(B * H * H * C, device="cuda").to(torch.bfloat16)
        res = torch.randn(B * OH * OH * C, device="cuda").to(torch.bfloat16)
        y = torch.empty(B * OH * OH * C, dtype=torch.bfloat16, device="cuda")
        base = dict(x=x.data_ptr(), res=res.data_ptr(), y=y.data_ptr(), B=B, H=H, W=H, OH=OH, OW=OH, C=C,
                    pad_top=pt, pad_left=pt)
        ref = pool_add_ref(x, res, B, H, H, OH, OH, C, pt)

        def tm(kw, n=20):
            y.fill_(float("nan"))
            C_.pool_add({**base, **kw}, s)
            torch.cuda.synchronize()
            err = (y.float().view(-1, C) - ref).abs().max().item()
            assert err <= 2e-2 * ref.abs().max().item(), (kw, err)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                C_.pool_add({**base, **kw}, s)
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / n * 1e3
        gb = (B * H * H * C + 2 * B * OH * OH * C) * 2 / 1e9
        t1 = tm(dict(algo=1))
        print(f"{name:4s} {H}x{H}x{C} -> {OH}: pixel {t1:6.1f} us {gb / t1 * 1e3:5.2f} TB/s", flush=True)
        res_ = []
        for seg in (1, 2, 4):
            for rb in (0, 1, 2, 3, 4, 6, 10, 19):
                if rb > OH:
                    continue
                kw = dict(algo=2, seg=seg, rb=rb)
                res_.append((tm(kw), kw))
        res_.sort(key=lambda q: q[0])
        d0 = [q for q in res_ if q[1]["rb"] == 0]
        print("    rows default-rb: " + "  ".join(f"seg{q[1]['seg']} {q[0]:.1f}" for q in d0), flush=True)
        for q in res_[:4]:
            print(f"    rows {q[0]:6.1f} us {gb / q[0] * 1e3:5.2f} TB/s  {q[1]}", flush=True)


if __name__ == "__main__":
    main()
