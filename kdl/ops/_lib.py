"""Loader for the in-tree native extensions.

``import torch`` MUST precede loading ``kdl._C``: torch ships its own HIP runtime
(soname ``libamdhip64.so.7``) and the dynamic loader then binds our extension to
that same instance, so streams and device pointers are shared. There is no
silent fallback: on a GPU box a missing or broken ``_C`` raises.
"""
from __future__ import annotations

import importlib

import torch  # noqa: F401  (load order matters, see module doc)

_C = None
_RT = None
_ERR: Exception | None = None
_RT_ERR: Exception | None = None


def _try_load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    try:
        _C = importlib.import_module("kdl._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e


def lib():
    """The HIP kernel/executor module; raises if it is not built."""
    _try_load()
    if _C is None:
        raise RuntimeError(
            f"kdl._C (HIP kernels for gfx950) is not available: {_ERR!r}. "
            "Build it with `python -m kdl.csrc.build`.")
    return _C


def available() -> bool:
    _try_load()
    return _C is not None


def rt():
    """The CPU-only native runtime module (batcher, tfproto, sstable)."""
    global _RT, _RT_ERR
    if _RT is None and _RT_ERR is None:
        try:
            _RT = importlib.import_module("kdl._rt")
        except Exception as e:  # pragma: no cover
            _RT_ERR = e
    if _RT is None:
        raise RuntimeError(f"kdl._rt is not available: {_RT_ERR!r}. Build with `python -m kdl.csrc.build`.")
    return _RT


def rt_available() -> bool:
    try:
        rt()
        return True
    except RuntimeError:
        return False


def stream_ptr(stream: torch.cuda.Stream | None = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else int(t.data_ptr())


def num_cus(device: torch.device | str | None = None) -> int:
    """Compute units of a GPU (persistent kernels launch one workgroup per CU); 256 on MI355X."""
    d = torch.device(device) if device is not None else torch.device("cuda")
    if d.type != "cuda" or not torch.cuda.is_available():
        return 256
    return torch.cuda.get_device_properties(d).multi_processor_count
