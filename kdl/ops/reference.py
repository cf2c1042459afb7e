"""fp32 torch references of each fused kernel, for numerics tests.

They consume exactly the kernel's inputs (bf16 NHWC activations, the bf16-rounded
folded weights kept in ``ConvGemmLayer.w_ref``) and reproduce its intermediate
roundings (the depthwise output is rounded to bf16 before the MFMA), so the only
remaining difference is fp32 summation order.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .conv import MODE_CONV, MODE_DW, MODE_PW, ConvGemmLayer, Geometry


def _bf(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).float()


def conv_gemm_ref(lay: ConvGemmLayer, x: torch.Tensor, g: Geometry, res: torch.Tensor | None = None,
                  ldx: int | None = None) -> torch.Tensor:
    """Returns fp32 [M][ldy] (columns >= n are zero)."""
    ldx = ldx or lay.cin_pad
    xs = x.float().view(g.B, g.H, g.W, ldx)[..., :lay.cin_pad]
    w = lay.w_ref.to(x.device)
    if lay.mode == MODE_PW:
        a = xs[:, ::lay.stride, ::lay.stride, :].reshape(g.M, lay.cin_pad)
    elif lay.mode == MODE_CONV:
        cols = []
        st = lay.stride
        for dy in range(3):
            for dx in range(3):
                cols.append(xs[:, dy:dy + st * (g.OH - 1) + 1:st, dx:dx + st * (g.OW - 1) + 1:st, :])
        a = torch.cat(cols, dim=-1).reshape(g.M, 9 * lay.cin_pad)
    else:
        xin = torch.relu(xs) if lay.relu_in else xs
        xp = F.pad(xin.permute(0, 3, 1, 2), (1, 1, 1, 1))
        dw = lay.dww.to(x.device).t().reshape(lay.cin_pad, 1, 3, 3)
        a = F.conv2d(xp, dw, groups=lay.cin_pad).permute(0, 2, 3, 1).reshape(g.M, lay.cin_pad)
        a = _bf(a)
    y = a @ w.t() + lay.bias[: lay.n].to(x.device).float()
    if lay.relu_out == 1:
        y = torch.relu(y)
    out = torch.zeros(g.M, lay.ldy, device=x.device)
    out[:, : lay.n] = y
    if res is not None:
        out = _bf(out) + res.float().view(g.M, -1)[:, : lay.ldy]
    if lay.relu_out == 2:
        out = torch.relu(out)
    return out


def pool_add_ref(x: torch.Tensor, res: torch.Tensor | None, B, H, W, OH, OW, C, pad) -> torch.Tensor:
    xi = x.float().view(B, H, W, C).permute(0, 3, 1, 2)
    tot_h = max((OH - 1) * 2 + 3 - H, 0)
    tot_w = max((OW - 1) * 2 + 3 - W, 0)
    xi = F.pad(xi, (pad, tot_w - pad, pad, tot_h - pad), value=float("-inf"))
    y = F.max_pool2d(xi, 3, 2).permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float().view(B, OH, OW, C)
    return y.reshape(B * OH * OW, C)


def head_ref(x: torch.Tensor, B, HW, ldx, F_, w1, b1, w2, b2) -> torch.Tensor:
    """w1: Keras [F][H1], w2: [H1][NC]."""
    g = x.float().view(B, HW, ldx)[..., :F_].mean(1)
    h = torch.relu(g @ w1 + b1)
    return h @ w2 + b2
