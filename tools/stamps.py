#!/usr/bin/env python
"""Per-wave phase timing of the warp-specialized fused separable conv from in-kernel
s_memtime stamps (config 127 = 121 + stamping; sepconv_ws.hip STAMP).

For the first 64 blocks, every wave records, per k-step t, the time right after the
barrier (st0) and after its work for the step (st1). Printed: per role, the median
over waves/blocks of the k-step period, the work part and the barrier wait part, plus
prologue / epilogue spans. Clock: s_memtime counts shader-core cycles.

  python tools/stamps.py --shape mid_sep
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

from kdl.ops import _lib  # noqa: E402
from kdl.ops.conv import MODE_DW, Geometry  # noqa: E402
from tools.kbench import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="mid_sep")
    ap.add_argument("--cfg", type=int, default=127)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--no-relu", action="store_true", help="relu_in=False (sepconv2/3 of a block)")
    a = ap.parse_args()
    from test_kernels_gpu import _layer, _rand_act
    gen = torch.Generator().manual_seed(0)
    mode, cin, n, H, _ = SHAPES[a.shape]
    assert mode == MODE_DW
    lay = _layer(mode, cin, n, gen, relu_in=not a.no_relu)
    g = Geometry(a.batch, H, H, H, H)
    x = _rand_act((a.batch, H, H), lay.cin_pad, cin, gen)
    y = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(64 * 8 * 130, dtype=torch.int64, device="cuda")
    args = lay.args(_lib.ptr(x), _lib.ptr(y), g, cfg=a.cfg)
    args["stamps"] = st.data_ptr()
    C = _lib.lib()
    for _ in range(5):
        C.conv_gemm(MODE_DW, a.cfg, args, _lib.stream_ptr())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    C.conv_gemm(MODE_DW, a.cfg, args, _lib.stream_ptr())
    e1.record()
    torch.cuda.synchronize()
    kt = lay.K // 32
    s = st.view(64, 8, 130).cpu()
    print(f"{a.shape} cfg {a.cfg}: kernel {e0.elapsed_time(e1) * 1e3:.1f} us (event), KT={kt}")
    starts = s[:, 0, 0].tolist()
    print(f"block start spread (cycles): {max(starts) - min(starts)}")
    for role, waves in (("consumer", range(0, 4)), ("producer", range(4, 8))):
        per, work, wait, pro, epi, tot = [], [], [], [], [], []
        for b in range(64):
            for w in waves:
                r = s[b, w]
                st0 = r[2:2 + 2 * kt:2].tolist()
                st1 = r[3:3 + 2 * kt:2].tolist()
                tot.append(r[1].item())
                pro.append(st0[0])
                epi.append(r[1].item() - st1[kt - 1])
                for t in range(2, kt - 2):
                    per.append(st0[t + 1] - st0[t])
                    work.append(st1[t] - st0[t])
                    wait.append(st0[t + 1] - st1[t])
        med = statistics.median
        print(f"  {role}: step {med(per):7.0f}  work {med(work):7.0f}  wait {med(wait):7.0f}  "
              f"prologue {med(pro):7.0f}  loop-end->end {med(epi):7.0f}  total {med(tot):8.0f} cycles")
        # prologue milestones (cycles after kernel entry): setup done, loads issued, prologue barrier,
        # (producers) A(0) written
        ms = [[s[b, w, 120 + i].item() for b in range(64) for w in waves] for i in range(4)]
        print(f"    prologue milestones: " + "  ".join(f"p{i} {med(m):6.0f}" for i, m in enumerate(ms) if any(m)))


if __name__ == "__main__":
    main()
