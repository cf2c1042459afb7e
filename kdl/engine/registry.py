"""Model-family registry: oracle params + MI355X engine + benchmark metadata.

One entry per BASELINE.json config family the stack serves.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable


@dataclass(frozen=True)
class ModelInfo:
    name: str
    input_size: int
    classes: int
    params_total: int
    description: str
    init_params: Callable
    engine: Callable          # (params, max_batch, device, **kw) -> EngineBase
    oracle: Callable          # (params, uint8 NHWC) -> fp32 logits
    dtype: str = "bf16"       # compute dtype of the engine (bench.py's "dtype" field)
    tuning: str = ""          # tuning-table family name when it differs from ``name``
    stage_cut: str = ""       # default stage-pipeline cut (stages.py) for bench / serving; "" = lanes


def _xception():
    from ..models import xception as X
    from .xception import XceptionEngine
    return ModelInfo("xception", X.INPUT_SIZE, 10, 21_067_390,
                     "Keras Xception 299x299 + clothing head (21,067,390 params)",
                     lambda seed=0: X.init_params(seed=seed),
                     lambda p, max_batch, device, **kw: XceptionEngine(p, max_batch=max_batch, device=device,
                                                                       in_kind="u8", **kw),
                     lambda p, x: X.xception_forward(p, x.float() / 127.5 - 1.0),
                     stage_cut="block8_sepconv3")


def _resnet50(dtype: str = "fp16"):
    """BASELINE.json config 3 is "ResNet-50 224x224 fp16": fp16 by default,
    ``resnet50_bf16`` for the bf16 variant (same kernels, v_mfma_*_bf16)."""
    from ..models import resnet as R
    from .resnet import ResNetEngine
    return ModelInfo("resnet50" if dtype == "fp16" else "resnet50_bf16", R.INPUT_SIZE, 1000, R.TOTAL_PARAMS,
                     f"ResNet-50 v1.5 224x224 (torchvision layout, 25,557,032 params), {dtype}",
                     lambda seed=0: R.init_params(seed=seed),
                     lambda p, max_batch, device, **kw: ResNetEngine(p, max_batch=max_batch, device=device,
                                                                     dtype=dtype, **kw),
                     # three stages (3 compute streams): +1.3-1.9 % over the round-2 cut after layer3.1
                     # (profiles/stages3_ab_r3.txt)
                     R.resnet_forward, dtype=dtype, tuning="resnet50", stage_cut="layer2.1.conv3,layer3.3.conv3")


def _vit_b16():
    from ..models import vit as V
    from .vit import ViTEngine
    return ModelInfo("vit_b16", V.INPUT_SIZE, 1000, V.TOTAL_PARAMS,
                     "ViT-B/16 224x224 (torchvision layout, 86,567,656 params)",
                     lambda seed=0: V.init_params(seed=seed),
                     lambda p, max_batch, device, **kw: ViTEngine(p, max_batch=max_batch, device=device, **kw),
                     V.vit_forward, stage_cut="encoder.layers.encoder_layer_5.mlp.3")


def _efficientnet_b7():
    from ..models import efficientnet as E
    from .efficientnet import EfficientNetEngine
    return ModelInfo("efficientnet_b7", E.INPUT_SIZE, 1000, E.TOTAL_PARAMS,
                     "EfficientNet-B7 600x600 (torchvision layout, 66,347,960 params)",
                     lambda seed=0: E.init_params(seed=seed),
                     lambda p, max_batch, device, **kw: EfficientNetEngine(p, max_batch=max_batch, device=device,
                                                                           **kw),
                     E.efficientnet_forward, stage_cut="features.4.9.block.3")


def _vit_b16_fp8():
    from ..models import vit as V
    from .vit import ViTEngine
    return ModelInfo("vit_b16_fp8", V.INPUT_SIZE, 1000, V.TOTAL_PARAMS,
                     "ViT-B/16 224x224, e4m3 linears (static per-tensor activation / per-channel weight scales)",
                     lambda seed=0: V.init_params(seed=seed),
                     lambda p, max_batch, device, **kw: ViTEngine(p, max_batch=max_batch, device=device, fp8=True,
                                                                  **kw),
                     V.vit_forward, dtype="fp8-e4m3 linears / bf16 rest",
                     stage_cut="encoder.layers.encoder_layer_5.mlp.3")


_FACTORIES = {"xception": _xception, "resnet50": _resnet50, "resnet50_bf16": lambda: _resnet50("bf16"),
              "vit_b16": _vit_b16, "vit_b16_fp8": _vit_b16_fp8, "efficientnet_b7": _efficientnet_b7}


# (family, --dtype) -> engine variant; "auto" keeps the family's own default
_VARIANTS = {("resnet50", "bf16"): "resnet50_bf16", ("resnet50_bf16", "fp16"): "resnet50",
             ("vit_b16", "fp8"): "vit_b16_fp8", ("vit_b16_fp8", "bf16"): "vit_b16"}
_DTYPES = {"xception": {"bf16"}, "resnet50": {"fp16"}, "resnet50_bf16": {"bf16"}, "vit_b16": {"bf16"},
           "vit_b16_fp8": {"fp8"}, "efficientnet_b7": {"bf16"}}


def variant(family: str, dtype: str = "auto") -> str:
    """The engine variant of `family` computing in `dtype` (server ``--dtype``)."""
    if dtype in ("auto", "") or dtype in _DTYPES.get(family, set()):
        return family
    v = _VARIANTS.get((family, dtype))
    if v is None:
        raise ValueError(f"{family} has no {dtype} engine (available: "
                         f"{sorted(_DTYPES.get(family, set()) | {d for (f, d) in _VARIANTS if f == family})})")
    return v


def models() -> list[str]:
    return sorted(_FACTORIES)


def get(name: str) -> ModelInfo:
    if name not in _FACTORIES:
        raise KeyError(f"unknown model {name!r}; known: {', '.join(models())}")
    return _FACTORIES[name]()
