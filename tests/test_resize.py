"""PIL-NEAREST-exact resize of any-size uint8 images (kdl/serving/resize.py).

The reference resizes with PIL ``Image.NEAREST`` in its gateway (keras_image_helper,
`model_server.py:18,53`). The numpy path (CPU servers) and the HIP kernel
``resize_nearest_u8`` (GPU servers, the ``serving_image`` signature) must both equal
PIL exactly, for down-, up- and extreme scales.
"""
import numpy as np
import pytest
import torch
from PIL import Image

from kdl.serving.resize import Resizer

SHAPES = [(1, 534, 400), (1, 1, 1), (1, 2200, 2200), (3, 300, 1200), (2, 17, 299)]


def _pil(x):
    return np.stack([np.asarray(Image.fromarray(im).resize((299, 299), Image.NEAREST)) for im in x])


@pytest.mark.parametrize("shape", SHAPES)
def test_numpy_resize_equals_pil(shape):
    n, H, W = shape
    x = np.random.default_rng(H + W).integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    assert np.array_equal(Resizer(299, None)(x), _pil(x))


@pytest.mark.gpu
def test_gpu_resize_kernel_equals_pil():
    from kdl.ops import _lib
    assert _lib.available(), "kdl._C must be built for the GPU resize"
    r = Resizer(299, torch.cuda.current_device())
    for n, H, W in SHAPES + [(1, 534, 400)]:     # repeated size: cached tables, reused buffers
        x = np.random.default_rng(H * 3 + W).integers(0, 256, (n, H, W, 3), dtype=np.uint8)
        assert np.array_equal(r(x), _pil(x)), (n, H, W)


@pytest.mark.gpu
def test_gpu_resize_concurrent_requests_stay_exact():
    """No global lock: 8 threads x 6 requests of mixed sizes on 3 contexts (each its own stream
    and pinned staging) all equal PIL."""
    import threading
    r = Resizer(299, torch.cuda.current_device(), contexts=3)
    errs = []

    def worker(i):
        rng = np.random.default_rng(100 + i)
        for k in range(6):
            H, W = [(534, 400), (299, 299), (1200, 300), (64, 77)][(i + k) % 4]
            x = rng.integers(0, 256, (1 + k % 2, H, W, 3), dtype=np.uint8)
            if not np.array_equal(r(x), _pil(x)):
                errs.append((i, k, H, W))
    ths = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
