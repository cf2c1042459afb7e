#!/usr/bin/env python
"""Same-box vendor baseline: each BASELINE.json family as plain torch-ROCm eager code.

What a PyTorch user would deploy without kdl: BatchNorm folded into the conv weights
and biases (what TF-Serving's grappler / any inference export does), bf16 (ResNet-50:
fp16) weights and activations in channels_last, MIOpen convolutions, hipBLASLt GEMMs,
``F.scaled_dot_product_attention`` for ViT, and the whole forward captured once into a
``torch.cuda.CUDAGraph`` and replayed -- batch 32, synthetic uint8 images, the same
random-init weights as ``bench.py``. Timed like ``bench.py``: warmup replays, then K
replays between two synchronizes (no host->device copy here: the kdl bench includes
its H2D, so this baseline is favoured by it).

    python tools/vendor_baseline.py [--models xception,resnet50,vit_b16,efficientnet_b7]
           [--steps 50] [--warmup 10] [--check]

Prints one JSON line per model; ``--check`` also compares the logits with the fp32
oracle (cosine), so a fast-but-wrong vendor path cannot slip through.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

CL = torch.channels_last


def _fold(w, gamma, beta, mean, var, eps):
    s = gamma / torch.sqrt(var + eps)
    return w * s.view(-1, *([1] * (w.dim() - 1))), beta - mean * s


def _to(dev, dt, w, cl=True):
    w = w.to(dev, dt)
    return w.contiguous(memory_format=CL) if cl and w.dim() == 4 else w.contiguous()


# ---------------------------------------------------------------------------- Xception
def xception(params, dev, dt):
    from kdl.models import xception as X
    from kdl.models.layers import KERAS_BN_EPS, tf_same_pad
    p = params
    bn = lambda n: (p[f"{n}/gamma"], p[f"{n}/beta"], p[f"{n}/moving_mean"], p[f"{n}/moving_variance"])  # noqa: E731
    W = {}
    for blk in X.SPEC:
        ops = list(blk.main) + ([blk.res_conv] if blk.res_conv is not None else [])
        for op in ops:
            if isinstance(op, X.Conv):
                w = p[f"{op.name}/kernel"].permute(3, 2, 0, 1)
                w, b = _fold(w, *bn(op.bn), KERAS_BN_EPS)
                W[op.name] = (_to(dev, dt, w), _to(dev, dt, b))
            else:
                dw = p[f"{op.name}/depthwise_kernel"][:, :, :, 0].permute(2, 0, 1).unsqueeze(1)
                pw = p[f"{op.name}/pointwise_kernel"][0, 0].t()[:, :, None, None]
                pw, b = _fold(pw, *bn(op.bn), KERAS_BN_EPS)
                W[op.name] = (_to(dev, dt, dw), _to(dev, dt, pw), _to(dev, dt, b))
    hd = X.DEFAULT_HEAD
    w1, b1 = _to(dev, dt, p[f"{hd.hidden}/kernel"].t()), _to(dev, dt, p[f"{hd.hidden}/bias"])
    w2, b2 = _to(dev, dt, p[f"{hd.out}/kernel"].t()), _to(dev, dt, p[f"{hd.out}/bias"])

    def conv(x, op):
        w, b = W[op.name]
        return F.conv2d(x, w, b, stride=op.stride, padding=0)

    def sep(x, op):
        dw, pw, b = W[op.name]
        x = F.conv2d(x, dw, padding=1, groups=op.cin)
        return F.conv2d(x, pw, b)

    def pool(x):
        _, t, bt = tf_same_pad(x.shape[2], 3, 2)
        return F.max_pool2d(F.pad(x, (t, bt, t, bt), value=float("-inf")), 3, 2)

    def fwd(x_u8):
        x = (x_u8.permute(0, 3, 1, 2).to(dt) * (1 / 127.5) - 1).contiguous(memory_format=CL)
        for blk in X.SPEC:
            if blk.kind == "plain":
                for op in blk.main:
                    if isinstance(op, X.Conv):
                        x = torch.relu(conv(x, op))
                    else:
                        x = sep(torch.relu(x) if op.relu_in else x, op)
                        x = torch.relu(x) if op.relu_out else x
                continue
            res = x if blk.res_conv is None else conv(x, blk.res_conv)
            y = x
            for op in blk.main:
                y = sep(torch.relu(y) if op.relu_in else y, op)
                y = torch.relu(y) if op.relu_out else y
            if blk.pool:
                y = pool(y)
            x = y + res
        g = x.mean(dim=(2, 3))
        return (torch.relu(F.linear(g, w1, b1)) @ w2.t() + b2).float()
    return fwd


# ---------------------------------------------------------------------------- ResNet-50
def resnet50(params, dev, dt):
    from kdl.models import resnet as R
    p = params

    def cb(conv, bnn):
        w, b = _fold(p[conv], p[f"{bnn}.weight"], p[f"{bnn}.bias"], p[f"{bnn}.running_mean"],
                     p[f"{bnn}.running_var"], R.BN_EPS)
        return _to(dev, dt, w), _to(dev, dt, b)
    stem = cb("conv1.weight", "bn1")
    blocks = []
    for b in R.blocks():
        e = dict(c1=cb(f"{b.prefix}.conv1.weight", f"{b.prefix}.bn1"), c2=cb(f"{b.prefix}.conv2.weight", f"{b.prefix}.bn2"),
                 c3=cb(f"{b.prefix}.conv3.weight", f"{b.prefix}.bn3"), stride=b.stride)
        if b.downsample:
            e["ds"] = cb(f"{b.prefix}.downsample.0.weight", f"{b.prefix}.downsample.1")
        blocks.append(e)
    fw, fb = _to(dev, dt, p["fc.weight"]), _to(dev, dt, p["fc.bias"])
    mean = torch.tensor(R.MEAN, device=dev).view(1, 3, 1, 1) * 255
    std = torch.tensor(R.STD, device=dev).view(1, 3, 1, 1) * 255

    def fwd(x_u8):
        x = ((x_u8.permute(0, 3, 1, 2).float() - mean) / std).to(dt).contiguous(memory_format=CL)
        x = torch.relu(F.conv2d(x, *stem, stride=2, padding=3))
        x = F.max_pool2d(x, 3, 2, 1)
        for e in blocks:
            y = torch.relu(F.conv2d(x, *e["c1"]))
            y = torch.relu(F.conv2d(y, *e["c2"], stride=e["stride"], padding=1))
            y = F.conv2d(y, *e["c3"])
            sc = F.conv2d(x, *e["ds"], stride=e["stride"]) if "ds" in e else x
            x = torch.relu(y + sc)
        return F.linear(x.mean(dim=(2, 3)), fw, fb).float()
    return fwd


# ---------------------------------------------------------------------------- EfficientNet-B7
def efficientnet_b7(params, dev, dt):
    from kdl.models import efficientnet as E
    p = params

    def cb(conv, bnn):
        w, b = _fold(p[conv], p[f"{bnn}.weight"], p[f"{bnn}.bias"], p[f"{bnn}.running_mean"],
                     p[f"{bnn}.running_var"], E.BN_EPS)
        return _to(dev, dt, w), _to(dev, dt, b)
    stem = cb("features.0.0.weight", "features.0.1")
    blks = []
    for b in E.blocks():
        n = b.names()
        e = dict(b=b, dw=cb(f"{n['dw']}.0.weight", f"{n['dw']}.1"),
                 pr=cb(f"{n['project']}.0.weight", f"{n['project']}.1"),
                 se=tuple(_to(dev, dt, p[f"{n['se']}.{k}"]) for k in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")))
        if "expand" in n:
            e["ex"] = cb(f"{n['expand']}.0.weight", f"{n['expand']}.1")
        blks.append(e)
    head = cb("features.8.0.weight", "features.8.1")
    cw, cbias = _to(dev, dt, p["classifier.1.weight"]), _to(dev, dt, p["classifier.1.bias"])
    mean = torch.tensor(E.MEAN, device=dev).view(1, 3, 1, 1) * 255
    std = torch.tensor(E.STD, device=dev).view(1, 3, 1, 1) * 255

    def fwd(x_u8):
        x = ((x_u8.permute(0, 3, 1, 2).float() - mean) / std).to(dt).contiguous(memory_format=CL)
        x = F.silu(F.conv2d(x, *stem, stride=2, padding=1))
        for e in blks:
            b = e["b"]
            y = F.silu(F.conv2d(x, *e["ex"])) if "ex" in e else x
            y = F.silu(F.conv2d(y, *e["dw"], stride=b.stride, padding=(b.k - 1) // 2, groups=b.cexp))
            w1, b1, w2, b2 = e["se"]
            s = y.mean(dim=(2, 3), keepdim=True)
            s = torch.sigmoid(F.conv2d(F.silu(F.conv2d(s, w1, b1)), w2, b2))
            y = F.conv2d(y * s, *e["pr"])
            x = y + x if b.residual else y
        x = F.silu(F.conv2d(x, *head))
        return F.linear(x.mean(dim=(2, 3)), cw, cbias).float()
    return fwd


# ---------------------------------------------------------------------------- ViT-B/16
def vit_b16(params, dev, dt):
    from kdl.models import vit as V
    p = {k: _to(dev, dt, v, cl=False) for k, v in params.items()}
    mean = torch.tensor(V.MEAN, device=dev).view(1, 3, 1, 1) * 255
    std = torch.tensor(V.STD, device=dev).view(1, 3, 1, 1) * 255
    H, D = V.HEADS, V.DIM

    def fwd(x_u8):
        x = ((x_u8.permute(0, 3, 1, 2).float() - mean) / std).to(dt)
        B = x.shape[0]
        t = F.conv2d(x, p["conv_proj.weight"], p["conv_proj.bias"], stride=V.PATCH).flatten(2).transpose(1, 2)
        x = torch.cat([p["class_token"].expand(B, -1, -1), t], dim=1) + p["encoder.pos_embedding"]
        N = x.shape[1]
        for i in range(V.DEPTH):
            L = V._layer(i)
            h = F.layer_norm(x, (D,), p[f"{L}.ln_1.weight"], p[f"{L}.ln_1.bias"], V.LN_EPS)
            qkv = F.linear(h, p[f"{L}.self_attention.in_proj_weight"], p[f"{L}.self_attention.in_proj_bias"])
            q, k, v = qkv.view(B, N, 3, H, D // H).permute(2, 0, 3, 1, 4)
            a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, N, D)
            x = x + F.linear(a, p[f"{L}.self_attention.out_proj.weight"], p[f"{L}.self_attention.out_proj.bias"])
            h = F.layer_norm(x, (D,), p[f"{L}.ln_2.weight"], p[f"{L}.ln_2.bias"], V.LN_EPS)
            h = F.gelu(F.linear(h, p[f"{L}.mlp.0.weight"], p[f"{L}.mlp.0.bias"]))
            x = x + F.linear(h, p[f"{L}.mlp.3.weight"], p[f"{L}.mlp.3.bias"])
        c = F.layer_norm(x[:, 0], (D,), p["encoder.ln.weight"], p["encoder.ln.bias"], V.LN_EPS)
        return F.linear(c, p["heads.head.weight"], p["heads.head.bias"]).float()
    return fwd


BUILDERS = {"xception": (xception, torch.bfloat16), "resnet50": (resnet50, torch.float16),
            "vit_b16": (vit_b16, torch.bfloat16), "efficientnet_b7": (efficientnet_b7, torch.bfloat16)}


def run(model: str, steps: int, warmup: int, batch: int, check: bool) -> dict:
    from kdl.engine import registry
    info = registry.get(model)
    dev = torch.device("cuda", 0)
    build, dt = BUILDERS[model]
    params = info.init_params(0)
    fwd = build(params, dev, dt)
    S = info.input_size
    g = torch.Generator().manual_seed(1234)
    x = torch.randint(0, 256, (batch, S, S, 3), generator=g, dtype=torch.uint8).to(dev)
    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):                       # MIOpen find / hipBLASLt heuristics outside capture
                fwd(x)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = fwd(x)
        for _ in range(warmup):
            graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            graph.replay()
        torch.cuda.synchronize()
        dt_s = time.perf_counter() - t0
    res = {"model": model, "impl": "torch-ROCm eager, BN folded, channels_last, hipGraph replay",
           "dtype": str(dt).replace("torch.", ""), "batch": batch, "steps": steps,
           "ms_per_step": round(dt_s * 1e3 / steps, 4), "images_per_s": round(batch * steps / dt_s, 1),
           "torch": torch.__version__}
    if check:
        with torch.no_grad():
            ref = info.oracle({k: v.to(dev) for k, v in params.items()}, x).float()
        res["cos_min_vs_fp32_oracle"] = round(F.cosine_similarity(out.float(), ref, dim=1).min().item(), 5)
        res["top1_agree"] = int((out.argmax(1) == ref.argmax(1)).sum())
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="xception,resnet50,vit_b16,efficientnet_b7")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args(argv)
    torch.backends.cudnn.benchmark = True
    for m in a.models.split(","):
        print(json.dumps(run(m, a.steps, a.warmup, a.batch, a.check)), flush=True)
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
