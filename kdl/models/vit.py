"""ViT-B/16 (torchvision ``vit_b_16`` layout) as an fp32 torch oracle.

BASELINE.json config "ViT-B/16 224x224 (pure-GEMM path on CDNA4 fp8 MFMA)"
(17.56 GMAC; MLP 63.5 %, QKV 23.8 %, proj 7.9 %, attention 4 %).
Not part of the reference's graph (the reference serves one Keras Xception via
TF-Serving, `tf-serving.dockerfile:2-5`); a third family behind the same API.

Parameters use torchvision state_dict names (``conv_proj.weight``,
``encoder.layers.encoder_layer_0.self_attention.in_proj_weight`` ...), so a real
checkpoint (``torch.load(..., weights_only=True)``) drops in. Pre-norm encoder,
LayerNorm eps 1e-6, exact (erf) GELU, class token + learned position embedding,
ImageNet mean/std preprocessing.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

INPUT_SIZE = 224
PATCH = 16
DIM = 768
DEPTH = 12
HEADS = 12
MLP = 3072
NUM_CLASSES = 1000
LN_EPS = 1e-6
TOKENS = (INPUT_SIZE // PATCH) ** 2 + 1        # 197
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
TOTAL_PARAMS = 86_567_656                     # torchvision vit_b_16


def _layer(i: int) -> str:
    return f"encoder.layers.encoder_layer_{i}"


def param_shapes(num_classes: int = NUM_CLASSES) -> dict[str, tuple]:
    s = {"class_token": (1, 1, DIM), "conv_proj.weight": (DIM, 3, PATCH, PATCH), "conv_proj.bias": (DIM,),
         "encoder.pos_embedding": (1, TOKENS, DIM)}
    for i in range(DEPTH):
        L = _layer(i)
        s.update({f"{L}.ln_1.weight": (DIM,), f"{L}.ln_1.bias": (DIM,),
                  f"{L}.self_attention.in_proj_weight": (3 * DIM, DIM),
                  f"{L}.self_attention.in_proj_bias": (3 * DIM,),
                  f"{L}.self_attention.out_proj.weight": (DIM, DIM),
                  f"{L}.self_attention.out_proj.bias": (DIM,),
                  f"{L}.ln_2.weight": (DIM,), f"{L}.ln_2.bias": (DIM,),
                  f"{L}.mlp.0.weight": (MLP, DIM), f"{L}.mlp.0.bias": (MLP,),
                  f"{L}.mlp.3.weight": (DIM, MLP), f"{L}.mlp.3.bias": (DIM,)})
    s.update({"encoder.ln.weight": (DIM,), "encoder.ln.bias": (DIM,),
              "heads.head.weight": (num_classes, DIM), "heads.head.bias": (num_classes,)})
    return s


def count_params(num_classes: int = NUM_CLASSES) -> int:
    return sum(math.prod(v) for v in param_shapes(num_classes).values())


def init_params(seed: int = 0, num_classes: int = NUM_CLASSES) -> dict[str, torch.Tensor]:
    """Random init of the exact architecture (truncated-normal-like scales as in
    torchvision; LN gains 1, biases small so the residual stream keeps a sane scale)."""
    g = torch.Generator().manual_seed(seed)
    p = {}
    for k, shp in param_shapes(num_classes).items():
        if k.endswith("ln_1.weight") or k.endswith("ln_2.weight") or k == "encoder.ln.weight":
            t = torch.ones(shp)
        elif k.endswith(".bias") and ("ln_" in k or k == "encoder.ln.bias"):
            t = torch.zeros(shp)
        elif k.endswith("bias"):
            t = torch.randn(shp, generator=g) * 0.02
        elif k == "conv_proj.weight":
            t = torch.randn(shp, generator=g) * (1.0 / (3 * PATCH * PATCH)) ** 0.5
        elif k in ("class_token", "encoder.pos_embedding"):
            t = torch.randn(shp, generator=g) * 0.02
        else:  # linear weights [out, in]
            t = torch.randn(shp, generator=g) * (1.0 / shp[1]) ** 0.5
        p[k] = t.float()
    return p


def preprocess(x_u8_nhwc: torch.Tensor) -> torch.Tensor:
    x = x_u8_nhwc.float().permute(0, 3, 1, 2) / 255.0
    return (x - torch.tensor(MEAN, device=x.device).view(1, 3, 1, 1)) / torch.tensor(STD, device=x.device).view(1, 3, 1, 1)


def embed(p, x_nchw):
    B = x_nchw.shape[0]
    t = F.conv2d(x_nchw, p["conv_proj.weight"], p["conv_proj.bias"], stride=PATCH)   # [B, D, 14, 14]
    t = t.flatten(2).transpose(1, 2)                                                 # [B, 196, D]
    cls = p["class_token"].expand(B, -1, -1)
    return torch.cat([cls, t], dim=1) + p["encoder.pos_embedding"]


def attention(p, L, x):
    B, N, D = x.shape
    qkv = x @ p[f"{L}.self_attention.in_proj_weight"].t() + p[f"{L}.self_attention.in_proj_bias"]
    q, k, v = qkv.view(B, N, 3, HEADS, D // HEADS).permute(2, 0, 3, 1, 4)            # [B, H, N, dh]
    a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D // HEADS), dim=-1) @ v
    a = a.transpose(1, 2).reshape(B, N, D)
    return a @ p[f"{L}.self_attention.out_proj.weight"].t() + p[f"{L}.self_attention.out_proj.bias"]


def encoder_layer(p, i, x):
    L = _layer(i)
    x = x + attention(p, L, F.layer_norm(x, (DIM,), p[f"{L}.ln_1.weight"], p[f"{L}.ln_1.bias"], LN_EPS))
    h = F.layer_norm(x, (DIM,), p[f"{L}.ln_2.weight"], p[f"{L}.ln_2.bias"], LN_EPS)
    h = F.gelu(h @ p[f"{L}.mlp.0.weight"].t() + p[f"{L}.mlp.0.bias"])
    return x + h @ p[f"{L}.mlp.3.weight"].t() + p[f"{L}.mlp.3.bias"]


@torch.no_grad()
def vit_forward(p, x_u8_nhwc: torch.Tensor) -> torch.Tensor:
    """fp32 oracle: uint8 NHWC [B,224,224,3] -> logits [B,1000]."""
    x = embed(p, preprocess(x_u8_nhwc))
    for i in range(DEPTH):
        x = encoder_layer(p, i, x)
    c = F.layer_norm(x[:, 0], (DIM,), p["encoder.ln.weight"], p["encoder.ln.bias"], LN_EPS)
    return c @ p["heads.head.weight"].t() + p["heads.head.bias"]


@torch.no_grad()
def activation_amax(p, x_u8_nhwc: torch.Tensor) -> list[dict[str, float]]:
    """Calibration for the fp8 engine: per encoder layer, the max |value| of the four
    tensors that feed fp8 GEMMs (ln_1 out -> QKV, attention out -> out_proj,
    ln_2 out -> mlp.0, GELU out -> mlp.3)."""
    out = []
    x = embed(p, preprocess(x_u8_nhwc))
    for i in range(DEPTH):
        L = _layer(i)
        h1 = F.layer_norm(x, (DIM,), p[f"{L}.ln_1.weight"], p[f"{L}.ln_1.bias"], LN_EPS)
        B, N, D = h1.shape
        qkv = h1 @ p[f"{L}.self_attention.in_proj_weight"].t() + p[f"{L}.self_attention.in_proj_bias"]
        q, k, v = qkv.view(B, N, 3, HEADS, D // HEADS).permute(2, 0, 3, 1, 4)
        a = (torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D // HEADS), dim=-1) @ v).transpose(1, 2).reshape(B, N, D)
        x = x + a @ p[f"{L}.self_attention.out_proj.weight"].t() + p[f"{L}.self_attention.out_proj.bias"]
        h2 = F.layer_norm(x, (DIM,), p[f"{L}.ln_2.weight"], p[f"{L}.ln_2.bias"], LN_EPS)
        g = F.gelu(h2 @ p[f"{L}.mlp.0.weight"].t() + p[f"{L}.mlp.0.bias"])
        x = x + g @ p[f"{L}.mlp.3.weight"].t() + p[f"{L}.mlp.3.bias"]
        out.append({"ln_1": h1.abs().max().item(), "attn": a.abs().max().item(),
                    "ln_2": h2.abs().max().item(), "gelu": g.abs().max().item()})
    return out


def macs_per_image() -> int:
    n = TOKENS
    per_layer = n * DIM * 3 * DIM + 2 * n * n * DIM + n * DIM * DIM + 2 * n * DIM * MLP
    return (n - 1) * DIM * 3 * PATCH * PATCH + DEPTH * per_layer + DIM * NUM_CLASSES
