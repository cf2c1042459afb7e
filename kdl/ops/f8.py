"""FP8 (OCP e4m3) linear layers on ``gemm_f8.hip`` (BASELINE.json ViT-B/16 fp8 config).

Static quantisation: weights per output channel (s_w[n] = amax_n / 448), activations
per tensor with a calibrated scale s_a; the kernel computes in e4m3 x e4m3 -> fp32
on the block-scaled MFMA and applies colscale[n] = s_a * s_w[n] and the bias in the
fp32 epilogue. Producers of fp8 activations (LayerNorm, attention, the GELU GEMM)
write e4m3 = value / s_a directly, so no separate quantise pass exists.
"""
from __future__ import annotations

import torch

from . import _lib

E4M3_MAX = 448.0
# (FM, FN, WGM, WGN, STAGES) of KDL_F8_CONFIGS in gemm_f8.hip
F8_CONFIGS = {0: (4, 4, 2, 2, 2), 1: (4, 4, 2, 2, 3), 2: (2, 4, 2, 2, 3), 3: (4, 2, 2, 4, 2),
              4: (3, 3, 2, 4, 2), 5: (6, 3, 2, 4, 2), 6: (3, 6, 2, 4, 2), 7: (4, 4, 2, 4, 2),
              8: (5, 2, 2, 4, 2), 9: (5, 3, 2, 4, 2), 10: (5, 4, 2, 4, 2),
              11: (4, 4, 2, 4, 3), 12: (5, 2, 2, 4, 3), 13: (4, 2, 2, 4, 3), 14: (5, 2, 2, 4, 4),
              15: (4, 2, 2, 4, 4), 16: (8, 4, 2, 4, 2), 17: (6, 4, 2, 4, 2)}


def f8_tile(cfg: int) -> tuple[int, int]:
    fm, fn, wgm, wgn, _ = F8_CONFIGS[cfg]
    return 16 * fm * wgm, 16 * fn * wgn


def to_e4m3(x: torch.Tensor) -> torch.Tensor:
    """Saturating float -> OCP e4m3 bytes (uint8)."""
    return x.float().clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).view(torch.uint8)


def from_e4m3(b: torch.Tensor) -> torch.Tensor:
    return b.view(torch.float8_e4m3fn).float()


def pack_f8_weights(w8: torch.Tensor, nf: int) -> torch.Tensor:
    """e4m3 bytes W8[N][K] -> [nf][K/128][2][64][16]: lane l = 16g + r holds row 16nf + r,
    k = 128kt + 32g + 16h + j in half h byte j (the 'contig32' operand order)."""
    n, k = w8.shape
    assert k % 128 == 0 and n <= nf * 16
    full = torch.zeros(nf * 16, k, dtype=torch.uint8)
    full[:n] = w8
    kt = k // 128
    t = full.view(nf, 16, kt, 4, 2, 16).permute(0, 2, 4, 3, 1, 5).contiguous()  # nf, kt, h, g, r, j
    return t.view(nf, kt, 2, 64, 16)


class F8Linear:
    """y = act(x @ W^T + b) (+res) with x given as e4m3 bytes scaled by ``in_scale``."""

    mode = -1
    split = False

    def __init__(self, name: str, w: torch.Tensor, b: torch.Tensor, in_scale: float, relu_out: int = 0,
                 device="cuda", candidates: list[int] | None = None):
        self.name = name
        self.n, self.k = w.shape
        assert self.k % 128 == 0, (name, w.shape)
        self.candidates = candidates or [c for c in F8_CONFIGS if self.n % f8_tile(c)[1] == 0]
        self.cfg = self.candidates[0]
        bn_max = max(f8_tile(c)[1] for c in self.candidates)
        self.nf = (self.n + bn_max - 1) // bn_max * bn_max // 16
        w = w.float()
        sw = (w.abs().amax(dim=1) / E4M3_MAX).clamp_min(1e-12)
        w8 = to_e4m3(w / sw[:, None])
        self.w_ref = from_e4m3(w8) * sw[:, None]          # exactly what the kernel multiplies
        self.wp = pack_f8_weights(w8, self.nf).to(device).contiguous()
        pad = self.nf * 16
        self.bias = torch.zeros(pad, device=device)
        self.bias[: self.n] = b.float().to(device)
        self.in_scale = float(in_scale)
        self.colscale = torch.zeros(pad, device=device)
        self.colscale[: self.n] = (sw * self.in_scale).to(device)
        self.relu_out = relu_out

    def variants(self, W=None):
        return [(False, c) for c in self.candidates]

    def args(self, x8: int, M: int, y: int | None = None, y8: int | None = None, out_scale: float = 1.0,
             res: int | None = None, ldy: int | None = None) -> dict:
        return dict(x=x8, wp=_lib.ptr(self.wp), bias=_lib.ptr(self.bias), colscale=_lib.ptr(self.colscale),
                    res=res, y=y, y8=y8, out_inv_scale=1.0 / out_scale, M=M, K=self.k, ldx=self.k,
                    ldy=ldy or self.n, ldr=ldy or self.n, NF=self.nf, nstore=self.n, relu_out=self.relu_out)

    def emit(self, prog, cfg: int | None = None, **kw) -> None:
        cfg = self.cfg if cfg is None else cfg
        a = self.args(**kw)
        if prog is None:
            _lib.lib().gemm_f8(cfg, a, _lib.stream_ptr())
        else:
            prog.add_gemm_f8(self.name, cfg, a)
