#!/usr/bin/env python
"""ViT-B/16 attention alone (B=32, T=197, 12 heads x 64): time of the whole-head and the
query-tiled kernels (KDL_ATTN_TILED=1 picks the latter at process start), for rocprof PMC."""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from kdl.ops import _lib  # noqa: E402

B, T, H, dh = int(os.environ.get('AP_B', 32)), 197, 12, 64
qkv = torch.randn(B * T, 3 * H * dh, device="cuda").to(torch.bfloat16)
out = torch.zeros(B * T, H * dh, dtype=torch.bfloat16, device="cuda")
C = _lib.lib()
args = dict(qkv=qkv.data_ptr(), out=out.data_ptr(), B=B, T=T, H=H, dh=dh, scale=1 / math.sqrt(dh))
s = _lib.stream_ptr()
for _ in range(5):
    C.attention(args, s)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    C.attention(args, s)
e1.record()
e1.synchronize()
print(f"attention B{B} T{T}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us "
      f"({'tiled' if os.environ.get('KDL_ATTN_TILED') else 'whole-head'})")
