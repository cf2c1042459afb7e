"""Time the classifier head (GAP + dense + dense) alone at batch 32 (kprof-style)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from kdl.ops import _lib  # noqa: E402
B, HW, F, H1, NC = 32, 100, 2048, 100, 10
x = torch.randn(B * HW * F, device="cuda").to(torch.bfloat16)
w1t, b1 = torch.randn(H1, F, device="cuda"), torch.randn(H1, device="cuda")
w2, b2 = torch.randn(H1, NC, device="cuda"), torch.randn(NC, device="cuda")
out, feat, hid = torch.zeros(B, NC, device="cuda"), torch.zeros(B, F, device="cuda"), torch.zeros(F // 64, B, H1, device="cuda")
d = dict(x=_lib.ptr(x), w1=_lib.ptr(w1t), b1=_lib.ptr(b1), w2=_lib.ptr(w2), b2=_lib.ptr(b2), out=_lib.ptr(out),
         feat=_lib.ptr(feat), hid=_lib.ptr(hid), B=B, HW=HW, ldx=F, F=F, H1=H1, NC=NC)
for _ in range(50):
    _lib.lib().head_dense(d, _lib.stream_ptr())
torch.cuda.synchronize()
print("ok")
