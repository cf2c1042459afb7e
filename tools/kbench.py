#!/usr/bin/env python
"""Per-kernel micro-benchmark on the GPU: time every tile config of the fused
conv-GEMM on Xception layer shapes (random data, interleaved rounds in one
process, cdna guide §5.4 rule 24)."""
from __future__ import annotations

import argparse
import statistics

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from kdl.ops import _lib
from kdl.ops.conv import MODE_DW, MODE_PW, MODE_CONV, Geometry, cfg_tile

SHAPES = {
    # name: (mode, cin, n, H, stride)
    "mid_sep": (MODE_DW, 728, 728, 19, 1),
    "mid_sep_nr": (MODE_DW, 728, 728, 19, 1),   # without the pre-ReLU (sepconv2 / 3 of a middle block)
    "mid_pw": (MODE_PW, 728, 728, 19, 1),
    "b2_sep2": (MODE_DW, 128, 128, 147, 1),
    "b2_sep1": (MODE_DW, 64, 128, 147, 1),
    "b3_sep1": (MODE_DW, 128, 256, 74, 1),
    "b3_sep2": (MODE_DW, 256, 256, 74, 1),
    "b4_sep2": (MODE_DW, 728, 728, 37, 1),
    "b14_sep2": (MODE_DW, 1536, 2048, 10, 1),
    "b14_sep1_nr": (MODE_DW, 1024, 1536, 10, 1),   # block14_sepconv1 (no ReLU before it)
    "stem2": (MODE_CONV, 32, 64, 149, 1),
    "b4_res": (MODE_PW, 256, 728, 37, 2),      # block4 residual 1x1/2 (conv2d_2)
    "b13_res": (MODE_PW, 728, 1024, 19, 2),    # block13 residual 1x1/2 (conv2d_3)
    # the split lowering's pointwise GEMMs of blocks 4 / 13 / 14 (after their depthwise kernels)
    "b4_pw1": (MODE_PW, 256, 728, 37, 1),
    "b4_pw2": (MODE_PW, 728, 728, 37, 1),
    "b13_pw2": (MODE_PW, 728, 1024, 19, 1),
    "b14_pw2": (MODE_PW, 1536, 2048, 10, 1),
    # ablations of the middle-flow GEMM: K x2 / x0.5, M x2 (via --batch)
    "mid_pw_k2": (MODE_PW, 1456, 728, 19, 1),
    "mid_pw_kh": (MODE_PW, 352, 728, 19, 1),
    "mid_pw_n2": (MODE_PW, 728, 1456, 19, 1),
    # core-efficiency probes (large square GEMMs; M = batch*64*64)
    "sq4k": (MODE_PW, 4096, 4096, 64, 1),
    "sq2k": (MODE_PW, 2048, 2048, 64, 1),
    # ViT-B/16 linears (M = 32 x 14 x 14 = 6272 rows ~ the engine's 32 x 197 = 6304)
    "vit_qkv": (MODE_PW, 768, 2304, 14, 1),
    "vit_proj": (MODE_PW, 768, 768, 14, 1),
    "vit_mlp0": (MODE_PW, 768, 3072, 14, 1),
    "vit_mlp3": (MODE_PW, 3072, 768, 14, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--cfgs", default=None, help="comma list of (fused) config ids to time instead of all variants; "
                                                  "s<id> for the split lowering")
    ap.add_argument("--vendor", action="store_true",
                    help="MODE_PW shapes: also time torch.matmul bf16 (hipBLASLt; GEMM only, no bias / ReLU)")
    a = ap.parse_args()
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
    from test_kernels_gpu import _layer, _rand_act  # reuse the test constructors
    gen = torch.Generator().manual_seed(0)
    C = _lib.lib()
    s = torch.cuda.current_stream()
    for name in a.shapes.split(","):
        mode, cin, n, H, stride = SHAPES[name]
        lay = _layer(mode, cin, n, gen, stride=stride, relu_in=mode == MODE_DW and not name.endswith("_nr"))
        B = a.batch
        if mode == MODE_CONV:
            g = Geometry(B, H, H, H - 2, H - 2)
        elif mode == MODE_PW:
            oh = (H - 1) // stride + 1
            g = Geometry(B, H, H, oh, oh)
        else:
            g = Geometry(B, H, H, H, H)
        x = _rand_act((B, H, H), lay.cin_pad, cin, gen)
        y = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device="cuda")
        macs = g.M * n * (9 * cin if mode == MODE_CONV else cin)
        tmp = torch.zeros(g.M * lay.cin_pad, dtype=torch.bfloat16, device="cuda")
        variants = lay.variants(H)
        if a.cfgs:
            variants = [(c.startswith("s"), int(c.lstrip("s"))) for c in a.cfgs.split(",")]
        times = {v: [] for v in variants}
        for _ in range(a.rounds):
            for split, cfg in variants:
                def run():
                    lay.emit(None, _lib.ptr(x), _lib.ptr(y), g, tmp=_lib.ptr(tmp), split=split, cfg=cfg)
                run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                e1.synchronize()
                times[(split, cfg)].append(e0.elapsed_time(e1) / a.iters * 1e3)
        print(f"== {name}: M={g.M} K={lay.K} N={n} ({macs / 1e9:.2f} GMAC)")
        if a.vendor and mode == MODE_PW:
            xa = torch.randn((g.M, cin), dtype=torch.bfloat16, device="cuda")
            wb = torch.randn((cin, n), dtype=torch.bfloat16, device="cuda")
            out = torch.empty((g.M, n), dtype=torch.bfloat16, device="cuda")
            vt = []
            for _ in range(a.rounds):
                torch.matmul(xa, wb, out=out)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    torch.matmul(xa, wb, out=out)
                e1.record()
                e1.synchronize()
                vt.append(e0.elapsed_time(e1) / a.iters * 1e3)
            t = statistics.median(vt)
            print(f"   hipBLASLt (torch.matmul bf16, GEMM only): {t:8.1f} us  {2 * macs / t / 1e6:7.1f} TF/s")
        for (split, cfg), ts in sorted(times.items(), key=lambda kv: min(kv[1]))[:a.top]:
            t = statistics.median(ts)
            print(f"   {'split' if split else 'fused'} cfg {cfg:2d} tile {cfg_tile(cfg)}: {t:8.1f} us  "
                  f"{2 * macs / t / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
