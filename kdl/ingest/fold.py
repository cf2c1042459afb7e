"""BN-folded, bf16-packed Xception parameters (``kdl convert-savedmodel``).

Every BatchNormalization after a conv is folded into that conv's kernel (scale per
output channel, computed in double exactly as the engine does) and the kernel is
stored in bf16; the BN keeps only its shift (``<bn>/beta`` = beta - mean * scale).
The stem conv (block1_conv1) keeps its BN: its engine lowering folds the input
normalisation into the same weights before rounding. Depthwise kernels (BN acts after
the pointwise) and the dense head stay fp32.

The engine's packed weights come out bit-identical to packing the unfolded variables
(double product -> fp32 -> bf16 either way) and the fp32 oracle reads the folded form
too (``_bn`` adds the shift), so a folded version directory serves like the original
at half the file size and without the BN pass at load.
"""
from __future__ import annotations

import torch

from ..models import xception as X
from ..ops.pack import bn_scale_shift

FOLDED_KEY = "__kdl_bn_folded__"


def fold_xception(p: dict[str, torch.Tensor]) -> dict[str, torch.Tensor]:
    out = dict(p)
    for op in X.iter_convs():
        if op.name == "block1_conv1":
            continue
        s, t = bn_scale_shift(p, op.bn)
        key = f"{op.name}/kernel" if isinstance(op, X.Conv) else f"{op.name}/pointwise_kernel"
        w = p[key].double() * s          # HWIO / 11IO: the output channel is the last axis
        out[key] = w.float().to(torch.bfloat16)
        for v in ("gamma", "moving_mean", "moving_variance"):
            out.pop(f"{op.bn}/{v}", None)
        out[f"{op.bn}/beta"] = t.float()
    out[FOLDED_KEY] = torch.ones(1)
    return out


def unpack(p: dict[str, torch.Tensor]) -> dict[str, torch.Tensor]:
    """Loaded artifact -> in-memory params: bf16 kernels widened to fp32 (exact), marker dropped."""
    return {k: (v.float() if v.dtype == torch.bfloat16 else v) for k, v in p.items() if k != FOLDED_KEY}
