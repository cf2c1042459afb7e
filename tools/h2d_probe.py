#!/usr/bin/env python
"""Pinned host->device copy bandwidth for the ingress sizes bench.py moves per step
(one rank's 32-image uint8 shard and rank 0's whole 8-GPU batch under --ingress scatter)."""
import torch

S = 299 * 299 * 3
for n in (32, 64, 128, 256):
    h = torch.randint(0, 256, (n * S,), dtype=torch.uint8).pin_memory()
    d = torch.empty_like(h, device="cuda")
    for _ in range(3):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        d.copy_(h, non_blocking=True)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"H2D {n:4d} images {n * S / 1e6:7.1f} MB: {ms:7.3f} ms  {n * S / ms / 1e6:6.1f} GB/s", flush=True)
