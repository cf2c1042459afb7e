"""ResNet-50 (v1.5, torchvision layout) as an fp32 torch oracle.

BASELINE.json config "ResNet-50 224x224 fp16, 8 DP replicas" (SURVEY.md §2.6:
4.09 GMAC, 25.5 M params; 1x1 51.8 %, 3x3 45.2 %, 7x7 stem 2.9 % of FLOPs). Not
part of the reference's graph: the reference serves one Keras Xception through
TF-Serving (`tf-serving.dockerfile:2-5`); this is the second model family the
MI355X stack serves through the same Predict API.

Parameters are a flat dict with torchvision's state_dict names (``conv1.weight``,
``layer2.0.downsample.0.weight``, ``fc.weight`` ...), so a real torchvision
checkpoint (``torch.load(..., weights_only=True)``) drops in unchanged. v1.5 =
the stride-2 of a stage's first bottleneck sits on the 3x3 conv (torchvision),
not the first 1x1 (Keras/caffe v1). BN eps is PyTorch's 1e-5.

Preprocessing (torchvision): uint8 RGB -> x/255 -> (x - mean) / std per channel.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F

INPUT_SIZE = 224
NUM_CLASSES = 1000
BN_EPS = 1e-5
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
TOTAL_PARAMS = 25_557_032          # torchvision resnet50, trainable parameters
STAGES = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))   # (width, blocks, stride)
EXPANSION = 4


@dataclass(frozen=True)
class Bottleneck:
    prefix: str      # "layer2.0"
    cin: int
    width: int
    stride: int
    downsample: bool

    @property
    def cout(self) -> int:
        return self.width * EXPANSION


def blocks() -> list[Bottleneck]:
    out, cin = [], 64
    for si, (w, n, s) in enumerate(STAGES, start=1):
        for bi in range(n):
            stride = s if bi == 0 else 1
            out.append(Bottleneck(f"layer{si}.{bi}", cin, w, stride, bi == 0))
            cin = w * EXPANSION
    return out


def _bn_shapes(name: str, c: int) -> dict:
    return {f"{name}.weight": (c,), f"{name}.bias": (c,), f"{name}.running_mean": (c,),
            f"{name}.running_var": (c,)}


def param_shapes(num_classes: int = NUM_CLASSES) -> dict[str, tuple]:
    s = {"conv1.weight": (64, 3, 7, 7), **_bn_shapes("bn1", 64)}
    for b in blocks():
        s[f"{b.prefix}.conv1.weight"] = (b.width, b.cin, 1, 1)
        s.update(_bn_shapes(f"{b.prefix}.bn1", b.width))
        s[f"{b.prefix}.conv2.weight"] = (b.width, b.width, 3, 3)
        s.update(_bn_shapes(f"{b.prefix}.bn2", b.width))
        s[f"{b.prefix}.conv3.weight"] = (b.cout, b.width, 1, 1)
        s.update(_bn_shapes(f"{b.prefix}.bn3", b.cout))
        if b.downsample:
            s[f"{b.prefix}.downsample.0.weight"] = (b.cout, b.cin, 1, 1)
            s.update(_bn_shapes(f"{b.prefix}.downsample.1", b.cout))
    s["fc.weight"] = (num_classes, 2048)
    s["fc.bias"] = (num_classes,)
    return s


def count_params(num_classes: int = NUM_CLASSES) -> int:
    n = 0
    for k, shp in param_shapes(num_classes).items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            continue
        p = 1
        for d in shp:
            p *= d
        n += p
    return n


def init_params(seed: int = 0, num_classes: int = NUM_CLASSES, calibrate: bool = True,
                calib_batch: int = 2) -> dict[str, torch.Tensor]:
    """Random-init weights of the exact architecture; BN statistics calibrated on a
    random batch so activations keep a trained-like scale (see xception.init_params)."""
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
        elif k == "fc.weight":
            t = torch.randn(shp, generator=g) * (1.0 / shp[1]) ** 0.5
        elif k == "fc.bias":
            t = torch.randn(shp, generator=g) * 0.01
        elif k.endswith(".weight"):      # BN gamma
            t = 0.6 + 0.4 * torch.rand(shp, generator=g)
        else:                            # BN beta
            t = torch.randn(shp, generator=g) * 0.1
        p[k] = t.float()
    if calibrate:
        x = torch.randint(0, 256, (calib_batch, INPUT_SIZE, INPUT_SIZE, 3), generator=g, dtype=torch.uint8)
        resnet_forward(p, x, calibrate_bn=True)
    return p


def preprocess(x_u8_nhwc: torch.Tensor) -> torch.Tensor:
    """uint8 NHWC -> normalised fp32 NCHW (torchvision transforms.Normalize)."""
    x = x_u8_nhwc.float().permute(0, 3, 1, 2) / 255.0
    mean = torch.tensor(MEAN, device=x_u8_nhwc.device).view(1, 3, 1, 1)
    std = torch.tensor(STD, device=x_u8_nhwc.device).view(1, 3, 1, 1)
    return (x - mean) / std


def _bn(x, p, name, calibrate):
    if calibrate:
        p[f"{name}.running_mean"] = x.mean(dim=(0, 2, 3)).detach().clone()
        p[f"{name}.running_var"] = x.var(dim=(0, 2, 3), unbiased=False).detach().clone()
    return F.batch_norm(x, p[f"{name}.running_mean"], p[f"{name}.running_var"], p[f"{name}.weight"],
                        p[f"{name}.bias"], False, 0.0, BN_EPS)


@torch.no_grad()
def features(p, x_nchw, calibrate_bn: bool = False) -> torch.Tensor:
    x = F.conv2d(x_nchw, p["conv1.weight"], stride=2, padding=3)
    x = torch.relu(_bn(x, p, "bn1", calibrate_bn))
    x = F.max_pool2d(x, 3, 2, 1)
    for b in blocks():
        y = torch.relu(_bn(F.conv2d(x, p[f"{b.prefix}.conv1.weight"]), p, f"{b.prefix}.bn1", calibrate_bn))
        y = torch.relu(_bn(F.conv2d(y, p[f"{b.prefix}.conv2.weight"], stride=b.stride, padding=1), p,
                           f"{b.prefix}.bn2", calibrate_bn))
        y = _bn(F.conv2d(y, p[f"{b.prefix}.conv3.weight"]), p, f"{b.prefix}.bn3", calibrate_bn)
        if b.downsample:
            sc = _bn(F.conv2d(x, p[f"{b.prefix}.downsample.0.weight"], stride=b.stride), p,
                     f"{b.prefix}.downsample.1", calibrate_bn)
        else:
            sc = x
        x = torch.relu(y + sc)
    return x


@torch.no_grad()
def resnet_forward(p, x_u8_nhwc: torch.Tensor, calibrate_bn: bool = False) -> torch.Tensor:
    """fp32 oracle: uint8 NHWC [B,224,224,3] -> logits [B,1000]."""
    f = features(p, preprocess(x_u8_nhwc), calibrate_bn)
    return f.mean(dim=(2, 3)) @ p["fc.weight"].t() + p["fc.bias"]


def macs_per_image() -> int:
    """Multiply-accumulates of one 224x224 forward (convs + fc)."""
    total = 112 * 112 * 64 * 3 * 49
    h = 56
    for b in blocks():
        oh = h // b.stride
        total += h * h * b.width * b.cin
        total += oh * oh * b.width * b.width * 9
        total += oh * oh * b.cout * b.width
        if b.downsample:
            total += oh * oh * b.cout * b.cin
        h = oh
    return total + 2048 * NUM_CLASSES
