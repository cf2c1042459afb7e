#!/usr/bin/env python
"""Time the fused MBConv kernel (mbconv_ed) against its unfused pair on B7 block shapes,
with timing ablations (abl bits: 1 no depthwise, 2 no expand MFMA)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from kdl.ops import _lib  # noqa: E402
from kdl.ops.conv import MODE_PW, ConvGemmLayer, Geometry  # noqa: E402

SHAPES = {"f2": (64, 288, 3, 1, 150), "f3": (96, 480, 5, 1, 75), "f4": (160, 960, 3, 1, 38)}


def main():
    C_ = _lib.lib()
    s = _lib.stream_ptr()
    gen = torch.Generator().manual_seed(0)
    B = 32
    for name, (cin, C, K, S, H) in SHAPES.items():
        pad = (K - 1) // 2
        OH = (H + 2 * pad - K) // S + 1
        Cs = cin // 4
        x = torch.randn(B * H * H * cin, generator=gen).to(torch.bfloat16).cuda()
        lay = ConvGemmLayer("e", MODE_PW, torch.randn(C, cin, dtype=torch.float64) / cin ** 0.5, torch.zeros(C),
                            cin_pad=cin, n=C, relu_out=4, device="cuda")
        wk = (torch.randn(K * K, C) / K).cuda()
        bd = torch.zeros(C).cuda()
        w1 = (torch.randn(Cs, C) / C ** 0.5).cuda()
        y = torch.zeros(B * OH * OH * C, dtype=torch.bfloat16, device="cuda")
        from kdl.engine.efficientnet import mbconv_blobs
        blob = mbconv_blobs(lay, (wk, bd), w1, K, C_.mbconv_blob_bytes(cin, K, Cs))
        mg = dict(B=B, H=H, W=H, C=C, OH=OH, OW=OH, K=K, S=S, pad=pad, Cs=Cs, ldx=cin, cin=cin, blob=blob.data_ptr())
        rb, tw, nt = C_.mbconv_ed_tiles(mg)
        pool = torch.zeros(B * nt * Cs, device="cuda")
        e = torch.zeros(B * H * H * C, dtype=torch.bfloat16, device="cuda")
        nt0 = C_.dwk_tiles(mg)[3]
        pool0 = torch.zeros(B * nt0 * Cs, device="cuda")

        def fused(abl=0):
            C_.mbconv_ed(dict(mg, x=x.data_ptr(), we=lay.wp.data_ptr(), be=lay.bias.data_ptr(), wd=wk.data_ptr(),
                              bd=bd.data_ptr(), y=y.data_ptr(), pool=pool.data_ptr(), w1=w1.data_ptr(), abl=abl), s)

        def unfused():
            lay.emit(None, x.data_ptr(), e.data_ptr(), Geometry(B, H, H, H, H), ldx=cin)
            C_.dwk(dict(mg, x=e.data_ptr(), w=wk.data_ptr(), bias=bd.data_ptr(), y=y.data_ptr(),
                        pool=pool0.data_ptr(), w1=w1.data_ptr(), act=2), s)

        def t(fn, it=10):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(it):
                fn()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / it * 1e3
        print(f"{name}: tile {rb}x{tw} ({nt} tiles/img)  fused {t(fused):8.1f} us  no-dw {t(lambda: fused(1)):8.1f}"
              f"  no-expand {t(lambda: fused(2)):8.1f}  neither {t(lambda: fused(3)):8.1f}  unfused {t(unfused):8.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
