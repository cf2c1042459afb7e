"""Map Keras variable names from a SavedModel onto the Xception parameter dict.

Named layers (``block*_conv*``, ``block*_sepconv*``, their ``_bn``) map 1:1.
The residual 1x1 convs, their BatchNorms and the head Dense layers are Keras
*auto-named* (``conv2d``, ``batch_normalization_3``, ``dense_7``...) with suffixes
that depend on the training session (`guide.md:234-235`), so they are matched
by creation order (numeric suffix) and checked by shape.
"""
from __future__ import annotations

import re

import numpy as np
import torch

from ..models import xception as X

_AUTO = re.compile(r"^(conv2d|batch_normalization|dense)(?:_(\d+))?$")


def _suffix_order(names: list[str]) -> list[str]:
    def key(n):
        m = _AUTO.match(n)
        return -1 if m.group(2) is None else int(m.group(2))
    return sorted(names, key=key)


def to_xception_params(variables: dict[str, np.ndarray]) -> tuple[dict[str, torch.Tensor], X.Head]:
    """Returns (params in the framework's naming, head names actually used)."""
    by_layer: dict[str, dict[str, np.ndarray]] = {}
    for full, arr in variables.items():
        if "/" not in full:
            continue
        layer, var = full.rsplit("/", 1)
        layer = layer.split("/")[-1]  # drop any enclosing model scope
        by_layer.setdefault(layer, {})[var] = arr
    auto = {"conv2d": [], "batch_normalization": [], "dense": []}
    for layer in by_layer:
        m = _AUTO.match(layer)
        if m:
            auto[m.group(1)].append(layer)
    want = X.param_shapes(include_head=False)
    res_convs = [b.res_conv for b in X.SPEC if b.res_conv is not None]
    rename: dict[str, str] = {}
    convs = _suffix_order(auto["conv2d"])
    bns = _suffix_order(auto["batch_normalization"])
    if len(convs) < len(res_convs) or len(bns) < len(res_convs):
        raise ValueError(f"expected {len(res_convs)} auto-named residual convs/BNs, found {convs} / {bns}")
    for rc, src_c, src_b in zip(res_convs, convs[-len(res_convs):], bns[-len(res_convs):]):
        rename[src_c] = rc.name
        rename[src_b] = rc.bn
    params: dict[str, torch.Tensor] = {}
    for layer, vars_ in by_layer.items():
        tgt = rename.get(layer, layer)
        for var, arr in vars_.items():
            key = f"{tgt}/{var}"
            if key in want:
                if tuple(arr.shape) != tuple(want[key]):
                    raise ValueError(f"{key}: shape {arr.shape} != expected {want[key]}")
                params[key] = torch.from_numpy(np.array(arr, dtype=np.float32))
    missing = sorted(set(want) - set(params))
    if missing:
        raise ValueError(f"SavedModel is missing {len(missing)} Xception variables, e.g. {missing[:5]}")
    dense = _suffix_order(auto["dense"])
    if len(dense) < 2:
        raise ValueError(f"expected the 2 Dense layers of the clothing head, found {dense}")
    hidden, out = dense[-2], dense[-1]
    k1, k2 = by_layer[hidden]["kernel"], by_layer[out]["kernel"]
    if k1.shape[0] != 2048 or k2.shape[0] != k1.shape[1]:
        raise ValueError(f"unexpected head shapes {hidden}:{k1.shape} {out}:{k2.shape}")
    head = X.Head(hidden=hidden, out=out, hidden_units=int(k1.shape[1]), classes=int(k2.shape[1]))
    for name in (hidden, out):
        for var in ("kernel", "bias"):
            params[f"{name}/{var}"] = torch.from_numpy(np.array(by_layer[name][var], dtype=np.float32))
    return params, head


def to_keras_variables(params: dict[str, torch.Tensor], residual_offset: int = 0,
                       head: X.Head = X.DEFAULT_HEAD) -> dict[str, np.ndarray]:
    """Inverse mapping (used to synthesise SavedModel fixtures): rename the
    residual convs/BNs with a session-dependent suffix offset."""
    out = {}
    ren = {}
    for i, b in enumerate([b for b in X.SPEC if b.res_conv is not None]):
        k = i + residual_offset
        ren[b.res_conv.name] = "conv2d" if k == 0 else f"conv2d_{k}"
        ren[b.res_conv.bn] = "batch_normalization" if k == 0 else f"batch_normalization_{k}"
    for key, t in params.items():
        layer, var = key.rsplit("/", 1)
        out[f"{ren.get(layer, layer)}/{var}"] = t.detach().cpu().numpy().astype(np.float32)
    return out
