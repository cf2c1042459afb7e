#!/usr/bin/env python
"""Per-layer numerics of a model engine on the GPU: run the steps one at a time
and compare every conv output with the fp32 reference of that layer computed
from the engine's own (bf16) input buffers. Localises kernel bugs vs. plain
bf16 drift through depth.

  python tools/layercheck.py --model resnet50 --batch 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from kdl.engine import registry  # noqa: E402
from kdl.ops import _lib  # noqa: E402
from kdl.ops.conv import Geometry  # noqa: E402
from kdl.ops.reference import conv_gemm_ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=2)
    a = ap.parse_args()
    info = registry.get(a.model)
    p = info.init_params(0)
    dev = torch.device("cuda", 0)
    eng = info.engine(p, a.batch, dev)
    B = a.batch
    x = torch.randint(0, 256, (B, info.input_size, info.input_size, 3), dtype=torch.uint8)
    eng.inp.copy_(x.to(dev))
    s = eng.stream
    worst = 0.0
    for step in eng.steps:
        prog = _lib.lib().Program()
        eng._emit(prog, step, B)
        prog.run(int(s.cuda_stream))
        torch.cuda.synchronize()
        if step.kind != "conv":
            continue
        H, W, OH, OW = step.geom
        g = Geometry(B, H, W, OH, OW)
        sh = eng.shapes[step.src]
        ldx = sh[2]
        xin = eng.bufs[step.src][: B * H * W * ldx]
        res = eng.bufs[step.res] if step.res else None
        ref = conv_gemm_ref(step.layer, xin, g, res[: g.M * eng.shapes[step.res][2]] if res is not None else None,
                            ldx=ldx)
        out = eng.bufs[step.dst]
        opad = step.extra.get("opad", 0)
        ld = eng.shapes[step.dst][2]
        if opad:
            out = out.view(B, OH + 2, OW + 2, ld)[:, 1:-1, 1:-1, :].reshape(g.M, ld)
        else:
            out = out[: g.M * ld].view(g.M, ld)
        err = ((out.float() - ref[:, :ld]).abs().max() / (ref.abs().max() + 1e-6)).item()
        worst = max(worst, err)
        flag = "  <-- BAD" if err > 2e-2 else ""
        print(f"{step.name:28s} rel err {err:.2e}{flag}", flush=True)
    print(f"worst {worst:.2e}")


if __name__ == "__main__":
    main()
