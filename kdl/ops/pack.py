"""Host-side weight preparation: BN folding and MFMA fragment packing.

SURVEY.md §2.5 K8: BatchNorm is folded at load time (W' = W*gamma/sqrt(var+eps),
b' = beta - mean*gamma/sqrt(var+eps), Keras eps = 1e-3). The folded pointwise /
conv weights are then re-laid out into the exact order the MFMA B-operand
fragments are consumed by ``conv_gemm.hip``: ``[n_frag][k_step][lane][8]`` with
lane l holding W[16*n_frag + (l & 15)][32*k_step + 8*(l >> 4) + j].
"""
from __future__ import annotations

import torch

from ..models.layers import KERAS_BN_EPS


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def bn_scale_shift(p: dict, bn: str, eps: float = KERAS_BN_EPS):
    if f"{bn}/gamma" not in p:          # BN already folded into the kernel (kdl.ingest.fold)
        b = p[f"{bn}/beta"].double()
        return torch.ones_like(b), b
    g, b = p[f"{bn}/gamma"].double(), p[f"{bn}/beta"].double()
    m, v = p[f"{bn}/moving_mean"].double(), p[f"{bn}/moving_variance"].double()
    s = g / torch.sqrt(v + eps)
    return s, b - m * s


def pack_fragments(w_nk: torch.Tensor, nf: int, kt: int, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """W[N][K] (any float dtype) -> ``dtype`` (bf16 or fp16) [nf][kt][64][8] zero padded."""
    n, k = w_nk.shape
    assert n <= nf * 16 and k <= kt * 32, (w_nk.shape, nf, kt)
    full = torch.zeros(nf * 16, kt * 32, dtype=torch.float32)
    full[:n, :k] = w_nk.float()
    # [nf, 16(r), kt, 4(q), 8(j)] -> [nf, kt, q, r, j] ; lane = q*16 + r
    t = full.view(nf, 16, kt, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
    return t.view(nf, kt, 64, 8).to(dtype)


def unpack_fragments(packed: torch.Tensor, n: int, k: int) -> torch.Tensor:
    nf, kt = packed.shape[0], packed.shape[1]
    t = packed.float().view(nf, kt, 4, 16, 8).permute(0, 3, 1, 2, 4).contiguous()
    return t.view(nf * 16, kt * 32)[:n, :k]


def pad_vec(v: torch.Tensor, n: int) -> torch.Tensor:
    out = torch.zeros(n, dtype=torch.float32)
    out[: v.numel()] = v.float()
    return out


def rowrun_weights(w_nk: torch.Tensor, kh: int, run: int, rp: int) -> torch.Tensor:
    """Stem weights W[N][kh*run] (k = ky*run + kx*3 + c) -> W[N][kh*rp]: every kernel row's
    run of kx*3 + c slots zero-padded to rp (the K layout of stem_rows_kernel, stem.hip)."""
    n = w_nk.shape[0]
    out = torch.zeros(n, kh, rp, dtype=w_nk.dtype)
    out[:, :, :run] = w_nk.reshape(n, kh, run)
    return out.reshape(n, kh * rp)
