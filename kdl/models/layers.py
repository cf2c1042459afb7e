"""Keras-exact building blocks for the fp32 torch oracle.

The reference serves a Keras model through TF-Serving (`tf-serving.dockerfile:2`,
`convert.py:4-6`), so every numeric convention here follows TensorFlow/Keras, not
PyTorch defaults:

* TF ``'same'`` padding puts the odd pad element at the bottom/right
  (the 74->37 max-pool is padded (0, 1), which
  ``nn.MaxPool2d(padding=1)`` gets wrong).
* Keras ``BatchNormalization`` uses ``epsilon=1e-3`` (PyTorch defaults to 1e-5).
* Max-pool padding never wins (it is -inf, TF ignores the pad).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

KERAS_BN_EPS = 1e-3


def tf_same_pad(in_size: int, kernel: int, stride: int) -> tuple[int, int, int]:
    """Return (out_size, pad_before, pad_after) of TF 'same' padding on one axis."""
    out = math.ceil(in_size / stride)
    total = max((out - 1) * stride + kernel - in_size, 0)
    before = total // 2
    return out, before, total - before


def tf_valid_out(in_size: int, kernel: int, stride: int) -> int:
    return (in_size - kernel) // stride + 1


def pad_same_nchw(x: torch.Tensor, kernel: int, stride: int, value: float = 0.0) -> torch.Tensor:
    _, _, h, w = x.shape
    _, t, b = tf_same_pad(h, kernel, stride)
    _, l, r = tf_same_pad(w, kernel, stride)
    if t == b == l == r == 0:
        return x
    return F.pad(x, (l, r, t, b), value=value)


def maxpool_same(x: torch.Tensor, kernel: int = 3, stride: int = 2) -> torch.Tensor:
    """TF MaxPool2D(padding='same') on NCHW."""
    return F.max_pool2d(pad_same_nchw(x, kernel, stride, value=float("-inf")), kernel, stride)


def bn_eval(x: torch.Tensor, gamma, beta, mean, var, eps: float = KERAS_BN_EPS) -> torch.Tensor:
    """Inference-mode BatchNormalization over channel axis 1."""
    scale = gamma / torch.sqrt(var + eps)
    shift = beta - mean * scale
    return x * scale[None, :, None, None] + shift[None, :, None, None]


def fold_bn(gamma, beta, mean, var, eps: float = KERAS_BN_EPS):
    """Return (scale, shift) so that BN(x) == x*scale + shift."""
    scale = gamma / torch.sqrt(var + eps)
    return scale, beta - mean * scale
