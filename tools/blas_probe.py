#!/usr/bin/env python
"""hipBLASLt (torch.matmul, bf16) timings on the GEMM shapes of tools/kbench.py,
as the library yardstick for the hand-written conv-GEMMs: M x K @ K x N."""
import argparse
import statistics

import torch

SHAPES = {"mid_pw": (11552, 736, 736), "b4_pw": (43808, 736, 736), "b2_pw": (691488, 128, 128),
          "b14_pw": (3200, 1536, 2048), "sq4k": (16384, 4096, 4096), "sq2k": (16384, 2048, 2048),
          # ViT-B/16 at batch 32 (M = 32 * 197 tokens)
          "vit_qkv": (6304, 768, 2304), "vit_proj": (6304, 768, 768), "vit_mlp0": (6304, 768, 3072),
          "vit_mlp3": (6304, 3072, 768)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--fp8", action="store_true")
    a = ap.parse_args()
    for name in a.shapes.split(","):
        M, K, N = SHAPES[name]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ts = []
        for _ in range(3):
            torch.matmul(x, w, out=y)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                torch.matmul(x, w, out=y)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / a.iters * 1e3)
        t = statistics.median(ts)
        print(f"== {name}: M={M} K={K} N={N}  hipBLASLt {t:8.1f} us  {2 * M * K * N / t / 1e6:7.1f} TF/s", flush=True)
        if a.fp8:
            try:
                xf = x.to(torch.float8_e4m3fn)
                wf = w.t().contiguous().to(torch.float8_e4m3fn).t()
                one = torch.ones((), device="cuda")
                ts = []
                for _ in range(3):
                    torch._scaled_mm(xf, wf, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        torch._scaled_mm(xf, wf, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) / a.iters * 1e3)
                t = statistics.median(ts)
                print(f"   fp8 e4m3 _scaled_mm {t:8.1f} us  {2 * M * K * N / t / 1e6:7.1f} TF/s", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"   fp8 _scaled_mm unavailable: {e}", flush=True)


if __name__ == "__main__":
    main()
