"""``serving_image``: uint8 images of ANY size, resized to the model input on the GPU.

The reference resizes in the gateway, on the CPU: keras_image_helper's PIL
``Image.NEAREST`` to 299x299 (`model_server.py:18,53`), then ships
f32 pixels. Here the gateway may ship the decoded pixels as they are
(``GATEWAY_MODE=raw``) and the model server resizes them with the table-driven
``resize_nearest_u8`` kernel (kdl/csrc/kernels/preprocess.hip; the row / column
tables are PIL's own double-precision rule, ``gateway.preprocess.nearest_indices``,
so the result is bit-identical to PIL) before the resized batch joins the
``serving_uint8`` batcher. Without a GPU the same tables drive a numpy gather.
"""
from __future__ import annotations

import os
import threading
from collections import OrderedDict

import numpy as np
import torch

from ..gateway.preprocess import nearest_indices
from ..ops import _lib

IMAGE_SIGNATURE = "serving_image"
MAX_PIXELS = int(os.environ.get("KDL_MAX_IMAGE_PIXELS", str(64 << 20)))   # per request, all images


class Resizer:
    """[n, H, W, 3] uint8 -> [n, S, S, 3] uint8, PIL-NEAREST exact. ``device``: a GPU index
    (HIP kernel on a stream of its own) or None (numpy)."""

    def __init__(self, size: int, device: int | None):
        self.S = size
        self.device = device
        self._lock = threading.Lock()
        self._tabs: OrderedDict[tuple[int, int], tuple] = OrderedDict()
        if device is not None:
            self._dev = torch.device("cuda", device)
            self.stream = torch.cuda.Stream(device=self._dev)
            self._cap_in = self._cap_out = 0

    def _tables(self, H: int, W: int):
        key = (H, W)
        t = self._tabs.get(key)
        if t is None:
            ys, xs = nearest_indices(H, self.S), nearest_indices(W, self.S)
            if self.device is not None:
                ys = torch.from_numpy(ys).to(self._dev)
                xs = torch.from_numpy(xs).to(self._dev)
            t = self._tabs[key] = (ys, xs)
            if len(self._tabs) > 256:
                self._tabs.popitem(last=False)
        else:
            self._tabs.move_to_end(key)
        return t

    def _grow(self, n_in: int, n_out: int) -> None:
        if n_in > self._cap_in:
            self._cap_in = max(n_in, 2 * self._cap_in)
            self._h_in = torch.empty(self._cap_in, dtype=torch.uint8).pin_memory()
            self._d_in = torch.empty(self._cap_in, dtype=torch.uint8, device=self._dev)
        if n_out > self._cap_out:
            self._cap_out = max(n_out, 2 * self._cap_out)
            self._h_out = torch.empty(self._cap_out, dtype=torch.uint8).pin_memory()
            self._d_out = torch.empty(self._cap_out, dtype=torch.uint8, device=self._dev)

    def __call__(self, x: np.ndarray) -> np.ndarray:
        assert x.dtype == np.uint8 and x.ndim == 4 and x.shape[3] == 3, (x.dtype, x.shape)
        n, H, W, _ = x.shape
        S = self.S
        if n * H * W > MAX_PIXELS:
            raise ValueError(f"{n} images of {H}x{W} exceed the {MAX_PIXELS}-pixel request limit")
        if self.device is None:
            ys, xs = self._tables(H, W)
            return np.ascontiguousarray(x[:, ys][:, :, xs])
        n_in, n_out = x.size, n * S * S * 3
        with self._lock:
            self._grow(n_in, n_out)
            ys, xs = self._tables(H, W)
            self._h_in[:n_in].numpy()[:] = x.reshape(-1)
            with torch.cuda.stream(self.stream):
                self._d_in[:n_in].copy_(self._h_in[:n_in], non_blocking=True)
                _lib.lib().resize_nearest_u8(
                    dict(src=_lib.ptr(self._d_in), dst=_lib.ptr(self._d_out), ytab=_lib.ptr(ys), xtab=_lib.ptr(xs),
                         SH=H, SW=W, OH=S, OW=S, n=n), int(self.stream.cuda_stream))
                self._h_out[:n_out].copy_(self._d_out[:n_out], non_blocking=True)
            self.stream.synchronize()
            return self._h_out[:n_out].numpy().reshape(n, S, S, 3).copy()


class ImageRunner:
    """The ``serving_image`` signature: resize (GPU when the servable has one), then the
    ``serving_uint8`` runner's batcher and executors; images already at the model size
    skip the resize."""

    def __init__(self, sig, inner, devices: list[int]):
        self.sig, self.inner = sig, inner
        self.source = inner.source
        self.resizer = Resizer(inner.source.input_size, devices[0] if devices else None)

    def predict(self, x, n: int, deadline_us: int) -> np.ndarray:
        x = np.asarray(x)
        S = self.source.input_size
        y = x if x.shape[1:3] == (S, S) else self.resizer(x)
        return self.inner.predict(np.ascontiguousarray(y), n, deadline_us)

    def healthy(self) -> bool:
        return self.inner.healthy()

    def close(self) -> None:       # the inner runner belongs to the servable
        pass
