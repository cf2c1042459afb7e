#!/usr/bin/env python
"""Run ONE layer variant repeatedly (for rocprofv3 --pmc / --kernel-trace).

  rocprofv3 --pmc SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/prof -o run -- \
      python tools/kprof.py --shape mid_pw --cfg 8 --iters 20
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

from kdl.ops import _lib  # noqa: E402
from kdl.ops.conv import MODE_CONV, MODE_DW, MODE_PW, Geometry  # noqa: E402
from tools.kbench import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="mid_pw")
    ap.add_argument("--cfg", type=int, default=8)
    ap.add_argument("--split", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    from test_kernels_gpu import _layer, _rand_act
    gen = torch.Generator().manual_seed(0)
    mode, cin, n, H, stride = SHAPES[a.shape]
    lay = _layer(mode, cin, n, gen, stride=stride, relu_in=mode == MODE_DW)
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
    tmp = torch.zeros(g.M * lay.cin_pad, dtype=torch.bfloat16, device="cuda")
    for _ in range(a.iters):
        lay.emit(None, _lib.ptr(x), _lib.ptr(y), g, tmp=_lib.ptr(tmp), split=a.split, cfg=a.cfg)
    torch.cuda.synchronize()
    print("done", a.shape, a.cfg, a.split)


if __name__ == "__main__":
    main()
