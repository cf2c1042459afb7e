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


class _Ctx:
    """One in-flight resize: its own stream and pinned / device buffers (grown on demand)."""

    def __init__(self, dev: torch.device):
        self.dev = dev
        self.stream = torch.cuda.Stream(device=dev)
        self.cap_in = self.cap_out = 0

    def grow(self, n_in: int, n_out: int) -> None:
        if n_in > self.cap_in:
            self.cap_in = max(n_in, 2 * self.cap_in)
            self.h_in = torch.empty(self.cap_in, dtype=torch.uint8).pin_memory()
            self.d_in = torch.empty(self.cap_in, dtype=torch.uint8, device=self.dev)
        if n_out > self.cap_out:
            self.cap_out = max(n_out, 2 * self.cap_out)
            self.h_out = torch.empty(self.cap_out, dtype=torch.uint8).pin_memory()
            self.d_out = torch.empty(self.cap_out, dtype=torch.uint8, device=self.dev)


class Resizer:
    """[n, H, W, 3] uint8 -> [n, S, S, 3] uint8, PIL-NEAREST exact. ``device``: a GPU index
    (HIP kernel) or None (numpy). Concurrent requests do not serialise: each call takes one of
    up to ``KDL_RESIZE_CTX`` (default 4) contexts -- stream + pinned staging -- from a free list,
    so the H2D, kernel and D2H of different requests overlap on the GPU."""

    def __init__(self, size: int, device: int | None, contexts: int | None = None):
        self.S = size
        self.device = device
        self._tab_lock = threading.Lock()
        self._tabs: OrderedDict[tuple[int, int], tuple] = OrderedDict()
        if device is not None:
            import queue
            self._dev = torch.device("cuda", device)
            n = contexts or int(os.environ.get("KDL_RESIZE_CTX", "4"))
            self._free: queue.SimpleQueue = queue.SimpleQueue()
            for _ in range(max(1, n)):
                self._free.put(_Ctx(self._dev))

    def _tables(self, H: int, W: int):
        key = (H, W)
        with self._tab_lock:
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
        ys, xs = self._tables(H, W)
        c = self._free.get()
        try:
            c.grow(n_in, n_out)
            c.h_in[:n_in].numpy()[:] = x.reshape(-1)
            with torch.cuda.device(self._dev), torch.cuda.stream(c.stream):
                c.d_in[:n_in].copy_(c.h_in[:n_in], non_blocking=True)
                _lib.lib().resize_nearest_u8(
                    dict(src=_lib.ptr(c.d_in), dst=_lib.ptr(c.d_out), ytab=_lib.ptr(ys), xtab=_lib.ptr(xs),
                         SH=H, SW=W, OH=S, OW=S, n=n), int(c.stream.cuda_stream))
                c.h_out[:n_out].copy_(c.d_out[:n_out], non_blocking=True)
            c.stream.synchronize()
            return c.h_out[:n_out].numpy().reshape(n, S, S, 3).copy()
        finally:
            self._free.put(c)


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
