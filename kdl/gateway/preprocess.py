"""Xception image preprocessing, bit-compatible with keras_image_helper 0.0.1.

The reference gateway calls ``create_preprocessor('xception', target_size=(299,
299)).from_url(url)`` (`model_server.py:8,18,53`): download -> PIL open ->
convert('RGB') -> resize(target, Image.NEAREST) -> float32 -> x/127.5 - 1
(SURVEY.md §2.3 X5, §2.9.4). ``nearest_indices`` reproduces PIL's NEAREST
source-index rule (double-precision accumulation, *not* floor((i+0.5)*s)); the
same tables drive the GPU resize kernel (``resize_nearest_u8``).
"""
from __future__ import annotations

import io
import urllib.request

import numpy as np
from PIL import Image

TARGET = (299, 299)


def nearest_indices(src: int, dst: int) -> np.ndarray:
    """PIL Image.NEAREST source index for each destination pixel on one axis."""
    scale = src / dst
    xx = 0.5 * scale
    out = np.empty(dst, dtype=np.int32)
    for i in range(dst):
        out[i] = min(int(xx), src - 1)
        xx += scale
    return out


def load_image(data: bytes) -> Image.Image:
    img = Image.open(io.BytesIO(data))
    if img.mode != "RGB":
        img = img.convert("RGB")
    return img


def to_uint8(img: Image.Image, target=TARGET) -> np.ndarray:
    """uint8 HWC after NEAREST resize (the native serving_uint8 payload)."""
    return np.asarray(img.resize(target, Image.NEAREST), dtype=np.uint8)


def resize_nearest_np(arr: np.ndarray, target=TARGET) -> np.ndarray:
    """Same as PIL NEAREST via the index tables (used to validate the tables)."""
    h, w = arr.shape[:2]
    ys, xs = nearest_indices(h, target[1]), nearest_indices(w, target[0])
    return arr[ys][:, xs]


def xception_preprocess(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32)
    x /= 127.5
    x -= 1.0
    return x


def image_to_tensor(img: Image.Image, target=TARGET) -> np.ndarray:
    """float32 [1, 299, 299, 3] in [-1, 1] (the reference's input_8 payload)."""
    x = np.array(img.resize(target, Image.NEAREST), dtype="float32")
    return xception_preprocess(np.array([x]))


def fetch(url: str, timeout: float = 10.0) -> bytes:
    with urllib.request.urlopen(url, timeout=timeout) as resp:
        return resp.read()


class XceptionPreprocessor:
    """Drop-in for keras_image_helper's ``create_preprocessor('xception', ...)``."""

    def __init__(self, target_size=TARGET):
        self.target_size = target_size

    def from_url(self, url: str) -> np.ndarray:
        return self.convert_to_tensor(load_image(fetch(url)))

    def from_bytes(self, data: bytes) -> np.ndarray:
        return self.convert_to_tensor(load_image(data))

    def convert_to_tensor(self, img: Image.Image) -> np.ndarray:
        if img.mode != "RGB":
            img = img.convert("RGB")
        return image_to_tensor(img, self.target_size)


def create_preprocessor(name: str, target_size=TARGET) -> XceptionPreprocessor:
    if name != "xception":
        raise ValueError(f"unsupported preprocessor {name!r} (this framework serves Xception)")
    return XceptionPreprocessor(target_size)
