"""``serving_image``: uint8 images of ANY size, resized to the model input on the GPU.

The reference resizes in the gateway, on the CPU: keras_image_helper's PIL
``Image.NEAREST`` to 299x299 (`model_server.py:18,53`), then ships
f32 pixels. Here the gateway may ship the decoded pixels as they are
(``GATEWAY_MODE=raw``) and the model server resizes them with the table-driven
``resize_nearest_u8`` kernel (kdl/csrc/kernels/preprocess.hip; the row / column
tables are PIL's own double-precision rule, ``gateway.preprocess.nearest_indices``,
so the result is bit-identical to PIL) before the resized batch joins the
``serving_uint8`` batcher. Without a GPU the same tables drive a numpy gather.

With native GPU executors behind the batcher the resized images never come back to the
host: the kernel writes them into a device buffer, the request is queued as a
device-resident batcher item (``DynamicBatcher.submit_device``) and the executor's backend
copies its rows device-to-device into the engine's input slot (``HipExecBackend::issue_dev``,
kdl/csrc/runtime/hip_backend.cpp) while the other rows of the batch come from the pinned
staging as usual.
"""
from __future__ import annotations

import contextlib
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
    """One in-flight resize: its own stream and pinned / device buffers (grown on demand).
    Outgrown device output buffers are kept, not freed: a device-resident batcher item whose
    request hit its deadline returns before the executor's device-to-device copy of it ran,
    so its buffer must stay valid (a later request may overwrite it: only the abandoned row
    reads garbage)."""

    def __init__(self, dev: torch.device):
        self.dev = dev
        self.stream = torch.cuda.Stream(device=dev)
        self.cap_in = self.cap_out = 0
        self._retired: list[torch.Tensor] = []

    def grow(self, n_in: int, n_out: int) -> None:
        if n_in > self.cap_in:
            self.cap_in = max(n_in, 2 * self.cap_in)
            self.h_in = torch.empty(self.cap_in, dtype=torch.uint8).pin_memory()
            self.d_in = torch.empty(self.cap_in, dtype=torch.uint8, device=self.dev)
        if n_out > self.cap_out:
            if self.cap_out:
                self._retired.append(self.d_out)
            self.cap_out = max(n_out, 2 * self.cap_out)
            self.h_out = torch.empty(self.cap_out, dtype=torch.uint8).pin_memory()
            self.d_out = torch.empty(self.cap_out, dtype=torch.uint8, device=self.dev)


class Resizer:
    """[n, H, W, 3] uint8 -> [n, S, S, 3] uint8, PIL-NEAREST exact. ``device``: a GPU index
    (HIP kernel), a list of them (contexts spread over the GPUs), or None (numpy). Concurrent
    requests do not serialise: each call takes one of up to ``KDL_RESIZE_CTX`` (default 4) per
    GPU contexts -- stream + pinned staging -- from a free list, so the H2D, kernel and D2H of
    different requests overlap on the GPU."""

    def __init__(self, size: int, device: int | list[int] | None, contexts: int | None = None):
        self.S = size
        devs = [] if device is None else [device] if isinstance(device, int) else list(device)
        self.device = devs[0] if devs else None
        self._tab_lock = threading.Lock()
        self._tabs: OrderedDict[tuple[int, int, int], tuple] = OrderedDict()
        if devs:
            import queue
            n = contexts or int(os.environ.get("KDL_RESIZE_CTX", "4"))
            self._free: queue.SimpleQueue = queue.SimpleQueue()
            for _ in range(max(1, n)):
                for d in devs:
                    self._free.put(_Ctx(torch.device("cuda", d)))

    def _tables(self, H: int, W: int, dev: torch.device | None):
        key = (H, W, -1 if dev is None else dev.index)
        with self._tab_lock:
            t = self._tabs.get(key)
            if t is None:
                ys, xs = nearest_indices(H, self.S), nearest_indices(W, self.S)
                if dev is not None:
                    ys = torch.from_numpy(ys).to(dev)
                    xs = torch.from_numpy(xs).to(dev)
                t = self._tabs[key] = (ys, xs)
                if len(self._tabs) > 256:
                    self._tabs.popitem(last=False)
            else:
                self._tabs.move_to_end(key)
            return t

    def _check(self, x: np.ndarray) -> None:
        assert x.dtype == np.uint8 and x.ndim == 4 and x.shape[3] == 3, (x.dtype, x.shape)
        n, H, W, _ = x.shape
        if n * H * W > MAX_PIXELS:
            raise ValueError(f"{n} images of {H}x{W} exceed the {MAX_PIXELS}-pixel request limit")

    def _resize_on(self, c: _Ctx, x: np.ndarray) -> int:
        """H2D + resize kernel on context ``c``'s stream; returns the output's element count."""
        n, H, W, _ = x.shape
        S = self.S
        n_in, n_out = x.size, n * S * S * 3
        ys, xs = self._tables(H, W, c.dev)
        c.grow(n_in, n_out)
        c.h_in[:n_in].numpy()[:] = x.reshape(-1)
        with torch.cuda.device(c.dev), torch.cuda.stream(c.stream):
            c.d_in[:n_in].copy_(c.h_in[:n_in], non_blocking=True)
            _lib.lib().resize_nearest_u8(
                dict(src=_lib.ptr(c.d_in), dst=_lib.ptr(c.d_out), ytab=_lib.ptr(ys), xtab=_lib.ptr(xs),
                     SH=H, SW=W, OH=S, OW=S, n=n), int(c.stream.cuda_stream))
        return n_out

    def __call__(self, x: np.ndarray) -> np.ndarray:
        self._check(x)
        n, H, W, _ = x.shape
        S = self.S
        if self.device is None:
            ys, xs = self._tables(H, W, None)
            return np.ascontiguousarray(x[:, ys][:, :, xs])
        c = self._free.get()
        try:
            n_out = self._resize_on(c, x)
            with torch.cuda.device(c.dev), torch.cuda.stream(c.stream):
                c.h_out[:n_out].copy_(c.d_out[:n_out], non_blocking=True)
            c.stream.synchronize()
            return c.h_out[:n_out].numpy().reshape(n, S, S, 3).copy()
        finally:
            self._free.put(c)

    @contextlib.contextmanager
    def on_device(self, x: np.ndarray):
        """Resize into a device buffer and yield its address ([n, S, S, 3] uint8, valid inside
        the block; the kernel has finished when the block starts)."""
        assert self.device is not None
        self._check(x)
        c = self._free.get()
        try:
            self._resize_on(c, x)
            c.stream.synchronize()
            yield _lib.ptr(c.d_out)
        finally:
            self._free.put(c)


class ImageRunner:
    """The ``serving_image`` signature: resize (GPU when the servable has one), then the
    ``serving_uint8`` runner's batcher and executors; images already at the model size
    skip the resize."""

    def __init__(self, sig, inner, devices: list[int]):
        self.sig, self.inner = sig, inner
        self.source = inner.source
        self.resizer = Resizer(inner.source.input_size, devices or None)
        self.device_path = bool(devices) and inner.takes_device_items()

    def predict(self, x, n: int, deadline_us: int) -> np.ndarray:
        x = np.asarray(x)
        S = self.source.input_size
        if x.shape[1:3] == (S, S):
            return self.inner.predict(np.ascontiguousarray(x), n, deadline_us)
        if self.device_path:           # resized straight into device memory: no host round trip
            with self.resizer.on_device(x) as ptr:
                return self.inner.predict_device(ptr, n, deadline_us)
        return self.inner.predict(self.resizer(x), n, deadline_us)

    def healthy(self) -> bool:
        return self.inner.healthy()

    def close(self) -> None:       # the inner runner belongs to the servable
        pass
