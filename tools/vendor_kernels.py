#!/usr/bin/env python
"""Which vendor kernels torch-ROCm runs for the ViT-B/16 GEMM shapes (batch 32: M = 6304), for
rocprofv3 --kernel-trace: hipBLASLt kernel names carry their macro tile (MT<M>x<N>x<K>), wave
tiling and MFMA shape -- the configurations our LDS-DMA GEMM tiles are compared against
(profiles/vit_gemm_vs_vendor_r4.jsonl). Probe only: never part of the product.

  rocprofv3 --kernel-trace --stats -d gpurun_out/vk -o run -- python tools/vendor_kernels.py
"""
import torch

M = 6304
SHAPES = {"qkv": (768, 2304), "out_proj": (768, 768), "mlp.0": (768, 3072), "mlp.3": (3072, 768)}


def main():
    dev = torch.device("cuda", 0)
    for name, (K, N) in SHAPES.items():
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        for _ in range(20):
            torch.matmul(a, b)
        torch.cuda.synchronize()
        if hasattr(torch, "_scaled_mm"):
            a8 = a.to(torch.float8_e4m3fn)
            b8 = b.t().contiguous().to(torch.float8_e4m3fn).t()
            one = torch.ones((), device=dev)
            try:
                for _ in range(20):
                    torch._scaled_mm(a8, b8, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            except RuntimeError as e:
                print(name, "fp8 _scaled_mm unavailable:", e)
        torch.cuda.synchronize()
        print("done", name, flush=True)


if __name__ == "__main__":
    main()
