"""Keras Xception + the ML-Bookcamp clothing head, as an fp32 torch oracle.

The reference serves ``xception_v4_large_08_0.894.h5`` (`convert.py:4`) whose
SavedModel signature is ``input_8 f32[-1,299,299,3] -> dense_7 f32[-1,10]``
(`guide.md:220-231`); the output is logits (`guide.md:623-625`). The graph is
Keras' ``applications.Xception(include_top=False)`` followed by
GAP -> Dense(100, relu) -> Dropout -> Dense(10).

This module is the *specification* of the network shared by three consumers:

* the fp32 oracle forward (``xception_forward``) used by every numerics test,
* the MI355X engine builder (``kdl.engine.xception_plan``), which walks ``SPEC``
  and emits fused HIP kernel launches,
* SavedModel ingest (``kdl.ingest.keras_map``), which maps checkpoint variables
  to the Keras layer names used here.

Parameters are a flat ``dict[str, Tensor]`` keyed ``"<layer>/<var>"`` in Keras
layouts (conv HWIO, depthwise ``[3,3,C,1]``, pointwise ``[1,1,Cin,Cout]``,
dense ``[in,out]``) so a real Keras checkpoint drops in unchanged.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

from .layers import KERAS_BN_EPS, bn_eval, maxpool_same, pad_same_nchw

INPUT_SIZE = 299
BASE_PARAMS = 20_861_480  # Keras Xception(include_top=False)
from ..labels import LABELS  # noqa: E402,F401  (model_server.py:21-32)


@dataclass(frozen=True)
class Conv:
    name: str
    cin: int
    cout: int
    k: int
    stride: int
    padding: str  # 'valid' | 'same'
    bn: str


@dataclass(frozen=True)
class Sep:
    name: str
    cin: int
    cout: int
    bn: str
    relu_in: bool   # Keras "<name>_act" ReLU applied before the separable conv
    relu_out: bool  # ReLU applied right after the BN (block1/block14 style)


@dataclass
class Block:
    """One residual unit: ``main`` ops, then optional pool, plus residual."""
    kind: str                 # 'entry' | 'middle' | 'exit' | 'plain'
    main: list = field(default_factory=list)
    res_conv: Conv | None = None   # None -> identity residual (middle flow)
    pool: bool = False


def _build_spec() -> list[Block]:
    spec: list[Block] = []
    spec.append(Block("plain", [Conv("block1_conv1", 3, 32, 3, 2, "valid", "block1_conv1_bn"),
                                Conv("block1_conv2", 32, 64, 3, 1, "valid", "block1_conv2_bn")]))
    cin = 64
    res_names = [("conv2d", "batch_normalization"), ("conv2d_1", "batch_normalization_1"),
                 ("conv2d_2", "batch_normalization_2")]
    for i, (blk, cout) in enumerate([(2, 128), (3, 256), (4, 728)]):
        rc, rb = res_names[i]
        spec.append(Block(
            "entry",
            [Sep(f"block{blk}_sepconv1", cin, cout, f"block{blk}_sepconv1_bn", relu_in=blk != 2, relu_out=True),
             Sep(f"block{blk}_sepconv2", cout, cout, f"block{blk}_sepconv2_bn", relu_in=False, relu_out=False)],
            res_conv=Conv(rc, cin, cout, 1, 2, "same", rb), pool=True))
        cin = cout
    for blk in range(5, 13):
        spec.append(Block(
            "middle",
            [Sep(f"block{blk}_sepconv1", 728, 728, f"block{blk}_sepconv1_bn", relu_in=True, relu_out=True),
             Sep(f"block{blk}_sepconv2", 728, 728, f"block{blk}_sepconv2_bn", relu_in=False, relu_out=True),
             Sep(f"block{blk}_sepconv3", 728, 728, f"block{blk}_sepconv3_bn", relu_in=False, relu_out=False)]))
    spec.append(Block(
        "exit",
        [Sep("block13_sepconv1", 728, 728, "block13_sepconv1_bn", relu_in=True, relu_out=True),
         Sep("block13_sepconv2", 728, 1024, "block13_sepconv2_bn", relu_in=False, relu_out=False)],
        res_conv=Conv("conv2d_3", 728, 1024, 1, 2, "same", "batch_normalization_3"), pool=True))
    spec.append(Block("plain", [Sep("block14_sepconv1", 1024, 1536, "block14_sepconv1_bn", False, True),
                                Sep("block14_sepconv2", 1536, 2048, "block14_sepconv2_bn", False, True)]))
    return spec


SPEC: list[Block] = _build_spec()


@dataclass(frozen=True)
class Head:
    hidden: str = "dense_6"
    out: str = "dense_7"
    hidden_units: int = 100
    classes: int = 10
    features: int = 2048


DEFAULT_HEAD = Head()


def iter_convs():
    """Yield every Conv/Sep op of the base in forward order."""
    for b in SPEC:
        for op in b.main:
            yield op
        if b.res_conv is not None:
            yield b.res_conv


def param_shapes(head: Head = DEFAULT_HEAD, include_head: bool = True) -> dict[str, tuple]:
    shapes: dict[str, tuple] = {}

    def bn(name, c):
        for v in ("gamma", "beta", "moving_mean", "moving_variance"):
            shapes[f"{name}/{v}"] = (c,)

    for op in iter_convs():
        if isinstance(op, Conv):
            shapes[f"{op.name}/kernel"] = (op.k, op.k, op.cin, op.cout)
        else:
            shapes[f"{op.name}/depthwise_kernel"] = (3, 3, op.cin, 1)
            shapes[f"{op.name}/pointwise_kernel"] = (1, 1, op.cin, op.cout)
        bn(op.bn, op.cout)
    if include_head:
        shapes[f"{head.hidden}/kernel"] = (head.features, head.hidden_units)
        shapes[f"{head.hidden}/bias"] = (head.hidden_units,)
        shapes[f"{head.out}/kernel"] = (head.hidden_units, head.classes)
        shapes[f"{head.out}/bias"] = (head.classes,)
    return shapes


def count_params(head: Head = DEFAULT_HEAD, include_head: bool = True) -> int:
    n = 0
    for s in param_shapes(head, include_head).values():
        p = 1
        for d in s:
            p *= d
        n += p
    return n


# --------------------------------------------------------------------------- init
def init_params(seed: int = 0, head: Head = DEFAULT_HEAD, calibrate: bool = True,
                calib_batch: int = 2, calib_size: int = 299) -> dict[str, torch.Tensor]:
    """Random-init weights of the exact architecture (no network for checkpoints).

    He-normal convs; BN moving statistics are *calibrated* on a random batch so
    every BN output is ~N(beta, gamma^2) like in a trained net — otherwise 36
    random BNs drift the activation scale by orders of magnitude and bf16 checks
    become meaningless.
    """
    g = torch.Generator().manual_seed(seed)
    p: dict[str, torch.Tensor] = {}
    for name, shape in param_shapes(head).items():
        var = name.split("/")[1]
        if var == "kernel" and len(shape) == 4:
            fan_in = shape[0] * shape[1] * shape[2]
            t = torch.randn(shape, generator=g) * (2.0 / fan_in) ** 0.5
        elif var == "depthwise_kernel":
            t = torch.randn(shape, generator=g) * (2.0 / 9.0) ** 0.5
        elif var == "pointwise_kernel":
            t = torch.randn(shape, generator=g) * (2.0 / shape[2]) ** 0.5
        elif var == "kernel":  # dense
            t = torch.randn(shape, generator=g) * (2.0 / shape[0]) ** 0.5
        elif var == "bias":
            t = torch.randn(shape, generator=g) * 0.05
        elif var == "gamma":
            t = 0.6 + 0.4 * torch.rand(shape, generator=g)
        elif var == "beta":
            t = torch.randn(shape, generator=g) * 0.1
        elif var == "moving_mean":
            t = torch.zeros(shape)
        elif var == "moving_variance":
            t = torch.ones(shape)
        else:  # pragma: no cover
            raise KeyError(name)
        p[name] = t.float()
    if calibrate:
        x = torch.rand((calib_batch, calib_size, calib_size, 3), generator=g) * 2.0 - 1.0
        xception_forward(p, x, head=head, calibrate_bn=True)
    return p


# --------------------------------------------------------------------------- oracle
def _conv(x, p, op: Conv):
    w = p[f"{op.name}/kernel"].permute(3, 2, 0, 1)  # HWIO -> OIHW
    if op.padding == "same":
        x = pad_same_nchw(x, op.k, op.stride)
    return F.conv2d(x, w, stride=op.stride)


def _sep(x, p, op: Sep):
    dw = p[f"{op.name}/depthwise_kernel"][:, :, :, 0].permute(2, 0, 1).unsqueeze(1)  # [C,1,3,3]
    pw = p[f"{op.name}/pointwise_kernel"][0, 0].t()[:, :, None, None]              # [Cout,Cin,1,1]
    x = F.conv2d(pad_same_nchw(x, 3, 1), dw, groups=op.cin)
    return F.conv2d(x, pw)


def _bn(x, p, name, calibrate_bn):
    if f"{name}/gamma" not in p:        # folded artifact: the kernel carries the scale
        return x + p[f"{name}/beta"][None, :, None, None]
    if calibrate_bn:
        mean = x.mean(dim=(0, 2, 3))
        var = x.var(dim=(0, 2, 3), unbiased=False)
        p[f"{name}/moving_mean"] = mean.detach().clone()
        p[f"{name}/moving_variance"] = var.detach().clone()
    return bn_eval(x, p[f"{name}/gamma"], p[f"{name}/beta"],
                   p[f"{name}/moving_mean"], p[f"{name}/moving_variance"], KERAS_BN_EPS)


def base_forward(p, x_nchw, calibrate_bn: bool = False) -> torch.Tensor:
    x = x_nchw
    for b in SPEC:
        if b.kind == "plain":
            for op in b.main:
                if isinstance(op, Conv):
                    x = torch.relu(_bn(_conv(x, p, op), p, op.bn, calibrate_bn))
                else:
                    x = _bn(_sep(torch.relu(x) if op.relu_in else x, p, op), p, op.bn, calibrate_bn)
                    if op.relu_out:
                        x = torch.relu(x)
            continue
        res = x if b.res_conv is None else _bn(_conv(x, p, b.res_conv), p, b.res_conv.bn, calibrate_bn)
        y = x
        for op in b.main:
            y = _bn(_sep(torch.relu(y) if op.relu_in else y, p, op), p, op.bn, calibrate_bn)
            if op.relu_out:
                y = torch.relu(y)
        if b.pool:
            y = maxpool_same(y, 3, 2)
        x = y + res
    return x


def head_forward(p, feat_nchw, head: Head = DEFAULT_HEAD) -> torch.Tensor:
    g = feat_nchw.mean(dim=(2, 3))
    h = torch.relu(g @ p[f"{head.hidden}/kernel"] + p[f"{head.hidden}/bias"])
    return h @ p[f"{head.out}/kernel"] + p[f"{head.out}/bias"]  # logits, no softmax (guide.md:623-625)


@torch.no_grad()
def xception_forward(p, x_nhwc: torch.Tensor, head: Head = DEFAULT_HEAD,
                     calibrate_bn: bool = False) -> torch.Tensor:
    """fp32 oracle: preprocessed NHWC f32 [B,H,W,3] in [-1,1] -> logits [B,10]."""
    x = x_nhwc.float().permute(0, 3, 1, 2).contiguous()
    return head_forward(p, base_forward(p, x, calibrate_bn), head)
