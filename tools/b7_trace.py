#!/usr/bin/env python
"""EfficientNet-B7 numerics trace: where does the engine's 15-17 %
max-logit error against the fp32 oracle come from?

Oracles (torch, any device), all from the same folded parameters:
  fp32        models/efficientnet.py's forward (BN folded in float64, applied in fp32)
  bf16        rounds to bf16 exactly where the engine stores bf16: the stem / expand / depthwise /
              project outputs and the folded weights, the SE-scaled project input bf16(D * s)
              (engine/efficientnet.py: the scale on the project GEMM's A operand), the pooled
              head features
  bf16+f32res the bf16 oracle with the block outputs (the residual stream) kept in fp32
  fp32+noise  the fp32 oracle on an input perturbed by ~bf16 rounding noise at the stem output
              (how much this random-init network amplifies a 2^-9 relative perturbation)

With --engine (GPU): the engine is run step by step and every block output is compared with
the bf16 oracle's (both fed from the engine's own previous block output) and with the fp32 one.

  python tools/b7_trace.py [--batch 2] [--size 600] [--device cpu|cuda] [--engine]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from kdl.models import efficientnet as E  # noqa: E402

bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731


def fold(p, conv, bn):
    w = p[conv].double()
    s = p[f"{bn}.weight"].double() / torch.sqrt(p[f"{bn}.running_var"].double() + E.BN_EPS)
    t = p[f"{bn}.bias"].double() - p[f"{bn}.running_mean"].double() * s
    return (w * s.view(-1, *([1] * (w.dim() - 1)))).float(), t.float()


class Folded:
    """BN-folded parameters of every layer (what the engine packs)."""

    def __init__(self, p, dev):
        self.stem = [t.to(dev) for t in fold(p, "features.0.0.weight", "features.0.1")]
        self.blk = []
        for b in E.blocks():
            n = b.names()
            d = {}
            if "expand" in n:
                d["expand"] = [t.to(dev) for t in fold(p, f"{n['expand']}.0.weight", f"{n['expand']}.1")]
            d["dw"] = [t.to(dev) for t in fold(p, f"{n['dw']}.0.weight", f"{n['dw']}.1")]
            se = n["se"]
            d["se"] = [p[f"{se}.{k}"].float().to(dev) for k in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")]
            d["project"] = [t.to(dev) for t in fold(p, f"{n['project']}.0.weight", f"{n['project']}.1")]
            self.blk.append((b, d))
        self.head = [t.to(dev) for t in fold(p, "features.8.0.weight", "features.8.1")]
        self.fc = (p["classifier.1.weight"].float().to(dev), p["classifier.1.bias"].float().to(dev))


def stem(F_, x_u8, mode):
    x = E.preprocess(x_u8)
    w, t = F_.stem
    y = F.silu(F.conv2d(x, bf(w) if mode != "fp32" else w, stride=2, padding=1) + t.view(1, -1, 1, 1))
    return bf(y) if mode != "fp32" else y


def block(b, d, x, mode, res_f32=False):
    """One MBConv; mode fp32 | bf16 (engine rounding points)."""
    r = (lambda t: t) if mode == "fp32" else bf
    y = x
    if "expand" in d:
        w, t = d["expand"]
        y = r(F.silu(F.conv2d(y, r(w)) + t.view(1, -1, 1, 1)))
    w, t = d["dw"]
    pre = F.silu(F.conv2d(y, w, stride=b.stride, padding=(b.k - 1) // 2, groups=b.cexp) + t.view(1, -1, 1, 1))
    D = r(pre)
    w1, b1, w2, b2 = d["se"]
    s = pre.mean(dim=(2, 3))                                   # SE pool from the fp32 depthwise values
    s = F.silu(s @ w1.view(b.csq, b.cexp).t() + b1)
    s = torch.sigmoid(s @ w2.view(b.cexp, b.csq).t() + b2)     # [B, cexp]
    wp, tp = d["project"]
    wp = wp.view(b.cout, b.cexp)
    if mode == "fp32":
        out = torch.einsum("bchw,oc->bohw", D * s[:, :, None, None], wp)
    else:                                                      # bf16(D * s) on the GEMM's A operand
        out = torch.einsum("bchw,oc->bohw", bf(D * s[:, :, None, None]), bf(wp))
    out = out + tp.view(1, -1, 1, 1)
    if b.residual:
        out = out + x
    return out if (mode == "fp32" or res_f32) else bf(out)


def head(F_, x, mode):
    w, t = F_.head
    r = (lambda t_: t_) if mode == "fp32" else bf
    y = r(F.silu(F.conv2d(x, r(w)) + t.view(1, -1, 1, 1)))
    f = y.mean(dim=(2, 3))
    f = r(f)
    wf, bfc = F_.fc
    return f @ (bf(wf) if mode != "fp32" else wf).t() + bfc


def run(F_, x_u8, mode, res_f32=False, noise=0.0, seed=0):
    h = stem(F_, x_u8, "fp32" if mode == "noise" else mode)
    if noise:
        g = torch.Generator(device="cpu").manual_seed(seed)
        h = h * (1 + noise * (torch.rand(h.shape, generator=g) * 2 - 1).to(h.device))
    outs = []
    m = "fp32" if mode == "noise" else mode
    for b, d in F_.blk:
        h = block(b, d, h, m, res_f32)
        outs.append(h)
    return head(F_, h, m), outs


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def maxrel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", type=int, default=E.INPUT_SIZE)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--engine", action="store_true")
    ap.add_argument("--out", default=None, help="write the JSON summary here")
    a = ap.parse_args()
    dev = torch.device(a.device)
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    p = E.init_params(seed=0)
    F_ = Folded(p, dev)
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (a.batch, a.size, a.size, 3), generator=g, dtype=torch.uint8).to(dev)
    with torch.no_grad():
        ref = E.efficientnet_forward({k: v.to(dev) for k, v in p.items()}, x)
        l32, o32 = run(F_, x, "fp32")
        lbf, obf = run(F_, x, "bf16")
        lrs, ors = run(F_, x, "bf16", res_f32=True)
        lno, ono = run(F_, x, "noise", noise=2 ** -9)
    summary = {"batch": a.batch, "size": a.size,
               "folded_fp32_vs_model_fp32_maxrel": maxrel(l32, ref),
               "logits_maxrel_vs_fp32": {"bf16 oracle": maxrel(lbf, l32), "bf16 + fp32 residual": maxrel(lrs, l32),
                                         "fp32 + 2^-9 stem noise": maxrel(lno, l32)},
               "top1_agree_vs_fp32": {"bf16 oracle": int((lbf.argmax(1) == l32.argmax(1)).sum()),
                                      "bf16 + fp32 residual": int((lrs.argmax(1) == l32.argmax(1)).sum()),
                                      "fp32 + 2^-9 stem noise": int((lno.argmax(1) == l32.argmax(1)).sum())}}
    print(json.dumps(summary, indent=1), flush=True)
    print(f"{'block':16s} {'bf16 vs fp32':>13s} {'bf16+f32res':>12s} {'noise vs fp32':>14s}  |x|", flush=True)
    rows = []
    for i, (b, _) in enumerate(F_.blk):
        row = (b.prefix, rel(obf[i], o32[i]), rel(ors[i], o32[i]), rel(ono[i], o32[i]), o32[i].abs().max().item())
        rows.append(row)
        print(f"{row[0]:16s} {row[1]:13.3e} {row[2]:12.3e} {row[3]:14.3e}  {row[4]:.1f}", flush=True)
    summary["blocks"] = rows
    if a.engine:
        summary["engine"] = engine_trace(p, F_, x, l32, lbf, o32, dev)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)


def engine_trace(p, F_, x, l32, lbf, o32, dev):
    """Run the engine step by step; after each block's project conv compare its output with
    (a) the bf16 oracle block fed with the ENGINE's previous block output (per-block kernel
    error, no drift) and (b) the fp32 oracle (accumulated drift)."""
    from kdl.engine.efficientnet import EfficientNetEngine
    from kdl.ops import _lib
    B = x.shape[0]
    eng = EfficientNetEngine(p, max_batch=B, device=dev, buckets=[B])
    logits = eng.forward(x).float()
    eng.inp.copy_(x)
    s = eng.stream
    out = {"logits_maxrel_engine_vs_fp32": maxrel(logits[:B], l32),
           "logits_maxrel_engine_vs_bf16_oracle": maxrel(logits[:B], lbf),
           "top1_engine_vs_fp32": int((logits[:B].argmax(1) == l32.argmax(1)).sum()), "blocks": []}
    print(json.dumps({k: v for k, v in out.items() if k != "blocks"}), flush=True)
    H = (eng.size + 2 - 3) // 2 + 1
    cur_name, cur_c = "X0", E.STEM
    prev = None
    bi = 0
    print(f"{'block':16s} {'eng vs bf16(eng in)':>20s} {'eng vs fp32':>12s}", flush=True)
    for step in eng.steps:
        prog = _lib.lib().Program()
        eng._emit(prog, step, B)
        prog.run(int(s.cuda_stream))
        torch.cuda.synchronize()
        if step.kind == "stem":
            prev = eng.bufs["X0"][: B * H * H * E.STEM].view(B, H, H, E.STEM).permute(0, 3, 1, 2).float()
            continue
        if step.kind != "conv" or bi >= len(F_.blk) or not step.name.endswith(
                F_.blk[bi][0].names()["project"]):
            continue
        b, d = F_.blk[bi]
        OH = step.geom[2]
        ld = step.layer.ldy
        got = eng.bufs[step.dst][: B * OH * OH * ld].view(B, OH, OH, ld)[..., : b.cout].permute(0, 3, 1, 2).float()
        with torch.no_grad():
            want = block(b, d, prev, "bf16")
        row = (b.prefix, rel(got, want), rel(got, o32[bi]))
        out["blocks"].append(row)
        print(f"{row[0]:16s} {row[1]:20.3e} {row[2]:12.3e}", flush=True)
        prev, bi = got, bi + 1
    return out


if __name__ == "__main__":
    main()
