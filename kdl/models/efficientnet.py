"""EfficientNet-B7 (torchvision ``efficientnet_b7`` layout) as an fp32 torch oracle.

BASELINE.json config "EfficientNet-B7 600x600 (large-activation path, LDS tiling
stress)" (37.75 GMAC, 66.0 M params, 55 MBConv blocks; pw expand
46.7 %, pw project 46.4 %, dw5x5 3.1 %, dw3x3 1.8 %; 34.6 MB/img peak bf16
activation). Not in the reference's graph (`tf-serving.dockerfile:2-5` serves one
Keras Xception); a fourth family behind the same Predict API.

torchvision state_dict names (``features.2.0.block.0.0.weight`` ...), so a real
checkpoint loads with ``torch.load(..., weights_only=True)``. MBConv = [1x1 expand
+ BN + SiLU] -> kxk depthwise (stride s, symmetric pad) + BN + SiLU -> squeeze-
excite (GAP -> 1x1 conv + SiLU -> 1x1 conv + sigmoid -> channel scale) -> 1x1
project + BN (+ identity residual when stride 1 and channels match; stochastic
depth is inactive at inference). BN eps 1e-3 as in the original TF EfficientNet.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

INPUT_SIZE = 600
NUM_CLASSES = 1000
BN_EPS = 1e-3
WIDTH, DEPTH = 2.0, 3.1
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
TOTAL_PARAMS = 66_347_960          # torchvision efficientnet_b7
# B0 stage table: (expand, kernel, stride, in, out, layers)
BASE = ((1, 3, 1, 32, 16, 1), (6, 3, 2, 16, 24, 2), (6, 5, 2, 24, 40, 2), (6, 3, 2, 40, 80, 3),
        (6, 5, 1, 80, 112, 3), (6, 5, 2, 112, 192, 4), (6, 3, 1, 192, 320, 1))


def make_divisible(v: float, divisor: int = 8) -> int:
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def ch(c: int) -> int:
    return make_divisible(c * WIDTH)


@dataclass(frozen=True)
class MBConv:
    prefix: str        # "features.2.0"
    cin: int
    cout: int
    expand: int
    k: int
    stride: int

    @property
    def cexp(self) -> int:
        return make_divisible(self.cin * self.expand) if self.expand != 1 else self.cin

    @property
    def csq(self) -> int:
        return max(1, self.cin // 4)

    @property
    def residual(self) -> bool:
        return self.stride == 1 and self.cin == self.cout

    def names(self) -> dict:
        b = f"{self.prefix}.block"
        i = 0
        out = {}
        if self.expand != 1:
            out["expand"] = f"{b}.{i}"
            i += 1
        out["dw"], out["se"], out["project"] = f"{b}.{i}", f"{b}.{i + 1}", f"{b}.{i + 2}"
        return out


def blocks() -> list[MBConv]:
    out = []
    for si, (e, k, s, cin, cout, n) in enumerate(BASE, start=1):
        layers = int(math.ceil(n * DEPTH))
        ci, co = ch(cin), ch(cout)
        for li in range(layers):
            out.append(MBConv(f"features.{si}.{li}", ci if li == 0 else co, co, e, k, s if li == 0 else 1))
    return out


STEM = ch(32)          # 64
HEAD = 4 * ch(320)     # 2560


def _bn(name, c):
    return {f"{name}.weight": (c,), f"{name}.bias": (c,), f"{name}.running_mean": (c,), f"{name}.running_var": (c,)}


def param_shapes(num_classes: int = NUM_CLASSES) -> dict[str, tuple]:
    s = {"features.0.0.weight": (STEM, 3, 3, 3), **_bn("features.0.1", STEM)}
    for b in blocks():
        n = b.names()
        if "expand" in n:
            s[f"{n['expand']}.0.weight"] = (b.cexp, b.cin, 1, 1)
            s.update(_bn(f"{n['expand']}.1", b.cexp))
        s[f"{n['dw']}.0.weight"] = (b.cexp, 1, b.k, b.k)
        s.update(_bn(f"{n['dw']}.1", b.cexp))
        s[f"{n['se']}.fc1.weight"] = (b.csq, b.cexp, 1, 1)
        s[f"{n['se']}.fc1.bias"] = (b.csq,)
        s[f"{n['se']}.fc2.weight"] = (b.cexp, b.csq, 1, 1)
        s[f"{n['se']}.fc2.bias"] = (b.cexp,)
        s[f"{n['project']}.0.weight"] = (b.cout, b.cexp, 1, 1)
        s.update(_bn(f"{n['project']}.1", b.cout))
    last = blocks()[-1].cout
    s["features.8.0.weight"] = (HEAD, last, 1, 1)
    s.update(_bn("features.8.1", HEAD))
    s["classifier.1.weight"] = (num_classes, HEAD)
    s["classifier.1.bias"] = (num_classes,)
    return s


def count_params(num_classes: int = NUM_CLASSES) -> int:
    return sum(math.prod(v) for k, v in param_shapes(num_classes).items()
               if not (k.endswith("running_mean") or k.endswith("running_var")))


def init_params(seed: int = 0, num_classes: int = NUM_CLASSES, calibrate: bool = True,
                calib_size: int = INPUT_SIZE, calib_batch: int = 2) -> dict[str, torch.Tensor]:
    """Random init; BN statistics calibrated on a random (smaller) batch so the
    activations keep a trained-like scale through 55 blocks. Calibrated variances
    are floored at 5 % of the layer's median: at 6x6 spatial a 4-image estimate of
    a near-dead channel's variance is ~0 and would blow that channel up by 100x on
    any other input."""
    g = torch.Generator().manual_seed(seed)
    p = {}
    for k, shp in param_shapes(num_classes).items():
        if k.endswith(".running_mean"):
            t = torch.zeros(shp)
        elif k.endswith(".running_var"):
            t = torch.ones(shp)
        elif len(shp) == 4:
            fan_in = shp[1] * shp[2] * shp[3]
            t = torch.randn(shp, generator=g) * (2.0 / fan_in) ** 0.5
        elif k.startswith("classifier") and k.endswith("weight"):
            t = torch.randn(shp, generator=g) * (1.0 / shp[1]) ** 0.5
        elif ".fc" in k or k.startswith("classifier"):      # SE / classifier biases
            t = torch.randn(shp, generator=g) * 0.1
        elif k.endswith(".weight"):                          # BN gamma
            t = 0.6 + 0.4 * torch.rand(shp, generator=g)
        else:                                                # BN beta
            t = torch.randn(shp, generator=g) * 0.1
        p[k] = t.float()
    if calibrate:
        x = torch.randint(0, 256, (calib_batch, calib_size, calib_size, 3), generator=g, dtype=torch.uint8)
        efficientnet_forward(p, x, calibrate_bn=True)
    return p


def preprocess(x_u8_nhwc: torch.Tensor) -> torch.Tensor:
    x = x_u8_nhwc.float().permute(0, 3, 1, 2) / 255.0
    return (x - torch.tensor(MEAN, device=x.device).view(1, 3, 1, 1)) / torch.tensor(STD, device=x.device).view(1, 3, 1, 1)


def _bnorm(x, p, name, calibrate):
    if calibrate:
        var = x.var(dim=(0, 2, 3), unbiased=False)
        p[f"{name}.running_mean"] = x.mean(dim=(0, 2, 3)).detach().clone()
        p[f"{name}.running_var"] = torch.maximum(var, 0.05 * var.median()).detach().clone()
    return F.batch_norm(x, p[f"{name}.running_mean"], p[f"{name}.running_var"], p[f"{name}.weight"],
                        p[f"{name}.bias"], False, 0.0, BN_EPS)


def mbconv(p, b: MBConv, x, calibrate=False):
    n = b.names()
    y = x
    if "expand" in n:
        y = F.silu(_bnorm(F.conv2d(y, p[f"{n['expand']}.0.weight"]), p, f"{n['expand']}.1", calibrate))
    y = F.conv2d(y, p[f"{n['dw']}.0.weight"], stride=b.stride, padding=(b.k - 1) // 2, groups=b.cexp)
    y = F.silu(_bnorm(y, p, f"{n['dw']}.1", calibrate))
    s = y.mean(dim=(2, 3), keepdim=True)
    s = F.silu(F.conv2d(s, p[f"{n['se']}.fc1.weight"], p[f"{n['se']}.fc1.bias"]))
    s = torch.sigmoid(F.conv2d(s, p[f"{n['se']}.fc2.weight"], p[f"{n['se']}.fc2.bias"]))
    y = _bnorm(F.conv2d(y * s, p[f"{n['project']}.0.weight"]), p, f"{n['project']}.1", calibrate)
    return y + x if b.residual else y


@torch.no_grad()
def features(p, x_nchw, calibrate_bn: bool = False):
    x = F.silu(_bnorm(F.conv2d(x_nchw, p["features.0.0.weight"], stride=2, padding=1), p, "features.0.1",
                      calibrate_bn))
    for b in blocks():
        x = mbconv(p, b, x, calibrate_bn)
    return F.silu(_bnorm(F.conv2d(x, p["features.8.0.weight"]), p, "features.8.1", calibrate_bn))


@torch.no_grad()
def efficientnet_forward(p, x_u8_nhwc: torch.Tensor, calibrate_bn: bool = False) -> torch.Tensor:
    """fp32 oracle: uint8 NHWC [B,600,600,3] -> logits [B,1000] (dropout inactive)."""
    f = features(p, preprocess(x_u8_nhwc), calibrate_bn)
    return f.mean(dim=(2, 3)) @ p["classifier.1.weight"].t() + p["classifier.1.bias"]


def macs_per_image(size: int = INPUT_SIZE) -> int:
    h = (size + 2 - 3) // 2 + 1
    total = h * h * STEM * 27
    for b in blocks():
        if b.expand != 1:
            total += h * h * b.cin * b.cexp
        oh = (h + 2 * ((b.k - 1) // 2) - b.k) // b.stride + 1
        total += oh * oh * b.cexp * b.k * b.k
        total += 2 * b.cexp * b.csq
        total += oh * oh * b.cexp * b.cout
        h = oh
    return total + h * h * blocks()[-1].cout * HEAD + HEAD * NUM_CLASSES
