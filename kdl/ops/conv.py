"""Layer objects for the fused conv-GEMM kernel family (``conv_gemm.hip``).

Each ``ConvGemmLayer`` owns device-resident, BN-folded, fragment-packed weights
and knows how to emit its launch (eagerly, for tests, or into a native
``Program`` for hipGraph capture). The tile config is a free choice among
``CONFIGS`` (same table as ``KDL_CONFIGS`` in the HIP source); the engine's
autotuner picks one per layer by timing on the device.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib
from .pack import pack_fragments, pad_vec, round_up

MODE_PW, MODE_CONV, MODE_DW = 0, 1, 2

# (FM, FN, WGM, WGN): block tile = (16*FM*WGM) x (16*FN*WGN).
# ids < PIPE_BASE: KDL_CONFIGS in conv_gemm.hip (register-B kernel, supports the
# fused depthwise producer); ids >= PIPE_BASE: KDL_PIPE_CONFIGS in gemm_pipe.hip
# (LDS-DMA ring, pointwise / 3x3 only); ids >= SEP_BASE: fused separable convs
# (MODE_DW). Ids 64-119 belonged to the round-1/2 sepconv_fused / sepconv_pipe kernels,
# retired in round 3 (slower than sepconv_ws / sepconv_2d on every Xception shape).
PIPE_BASE = 16
CONFIGS = {0: (2, 2, 2, 2), 1: (4, 2, 2, 2), 2: (2, 4, 2, 2), 3: (4, 4, 2, 2), 4: (4, 6, 1, 8),
           5: (2, 12, 1, 4), 6: (4, 4, 1, 4), 7: (2, 6, 1, 8), 8: (8, 2, 1, 4), 9: (4, 2, 1, 4),
           16: (4, 4, 2, 2), 17: (2, 4, 2, 2), 18: (4, 2, 2, 2), 19: (2, 2, 2, 2),
           20: (8, 2, 1, 4), 21: (4, 4, 1, 4), 22: (4, 8, 2, 2), 23: (8, 4, 1, 4),
           24: (3, 6, 2, 4), 25: (6, 3, 2, 4), 26: (3, 3, 2, 4), 27: (4, 4, 2, 2),
           28: (2, 6, 2, 4), 29: (4, 2, 2, 4), 30: (3, 3, 2, 4), 31: (6, 3, 2, 4),
           32: (4, 2, 2, 4), 33: (4, 4, 2, 2), 34: (3, 3, 2, 4), 35: (4, 4, 2, 2),
           36: (2, 4, 2, 2), 37: (4, 2, 2, 2), 38: (6, 3, 2, 4), 39: (3, 6, 2, 4),
           40: (3, 3, 2, 4), 41: (4, 2, 2, 4), 42: (6, 3, 2, 4),
           # 160-row LDS-DMA tiles (gemm_pipe.hip ids 45-47): whole waves at the ViT token counts;
           # 43-45: the same with 64-deep stages (half the barriers over ViT's K = 3072), 46: 4-stage ring
           43: (5, 2, 2, 4), 44: (5, 3, 2, 4), 45: (5, 4, 2, 4), 46: (5, 2, 2, 4),
           61: (5, 2, 2, 4), 62: (5, 3, 2, 4), 63: (5, 4, 2, 4),
           # warp-specialized fused separable conv (sepconv_ws.hip, KDL_SEPW_CONFIGS): (FM, FN, 1, 4);
           # 127 = s_memtime stamping build of 121 (tools/stamps.py, never a candidate)
           120: (6, 6, 1, 4), 121: (6, 6, 1, 4), 122: (6, 6, 1, 4), 123: (6, 6, 1, 4), 124: (6, 3, 1, 4),
           125: (4, 6, 1, 4), 126: (6, 6, 1, 4), 127: (6, 6, 1, 4),
           135: (12, 3, 1, 4), 136: (8, 3, 1, 4), 137: (12, 3, 1, 4),
           140: (4, 3, 1, 4), 141: (4, 3, 1, 4), 142: (2, 6, 1, 4),
           # 143-146 = 120, 122, 123, 125 walking K from a per-M-tile rotated start
           143: (6, 6, 1, 4), 144: (6, 6, 1, 4), 145: (6, 6, 1, 4), 146: (4, 6, 1, 4),
           # timing ablation of 143 (sepconv_ws.hip ABL; wrong values): full-line band reads
           147: (6, 6, 1, 4),
           # round 6 (sepconv_ws.hip): 128-131 stamped producer ablations of 143 (ABL 2 / 4 / 8 / 14,
           # wrong values), 132 stamped 143 with per-stage zero blocks (ZF), 133 stamped 143;
           # 148, 149, 156, 157 = 143-146 with ZF, 158 = 120 with ZF
           128: (6, 6, 1, 4), 129: (6, 6, 1, 4), 130: (6, 6, 1, 4), 131: (6, 6, 1, 4), 132: (6, 6, 1, 4),
           133: (6, 6, 1, 4), 148: (6, 6, 1, 4), 149: (6, 6, 1, 4), 156: (6, 6, 1, 4), 157: (4, 6, 1, 4),
           158: (6, 6, 1, 4),
           # 150-155: round 4's wide-tile variant and round 6's producer read-ahead, both measured slower and
           # removed (profiles/sepconv_wide_r4.txt, profiles/middle_flow_r6.txt)
           # fused separable conv over 2-D TH x TW pixel tiles (sepconv_2d.hip, KDL_S2D_CONFIGS)
           160: (3, 2, 2, 4), 161: (4, 2, 2, 4), 162: (2, 2, 2, 4), 163: (3, 4, 2, 4), 164: (4, 4, 2, 4),
           165: (4, 2, 2, 4), 166: (2, 4, 2, 4), 167: (3, 2, 2, 4), 168: (4, 1, 2, 4), 169: (2, 1, 4, 2),
           170: (3, 2, 2, 4), 171: (2, 2, 2, 4), 172: (2, 2, 2, 4), 173: (3, 4, 2, 4),
           # persistent 2-D tiled variant (sepconv_2dp_kernel, KDL_S2DP_CONFIGS): weights LDS-resident
           184: (3, 2, 2, 4), 185: (2, 2, 2, 4), 186: (2, 4, 2, 4), 187: (4, 2, 2, 4), 188: (3, 2, 2, 4),
           189: (2, 4, 2, 4), 190: (2, 2, 2, 4), 191: (2, 2, 2, 4), 192: (3, 2, 2, 4),
           # persistent 2-D sepconv with a dedicated DMA wave, direct stores (KDL_S2DW_CONFIGS)
           200: (2, 2, 2, 4), 201: (4, 2, 2, 4), 202: (3, 2, 2, 4), 203: (2, 4, 2, 4), 204: (4, 2, 2, 4),
           # 205-207 retired (round 3's pooled variant, measured slower)
           # 3x3 'valid' conv over 2-D tiles, LDS halo patch, cin 32 (conv3x3_2d.hip, KDL_C3_CONFIGS)
           208: (2, 2, 4, 2), 209: (1, 2, 4, 2), 210: (2, 2, 4, 2), 211: (3, 2, 4, 2),
           # ... with a dedicated DMA wave, accumulators stored directly (conv3x3_2dw_kernel)
           212: (2, 2, 4, 2), 213: (1, 2, 4, 2), 214: (2, 2, 4, 2), 215: (2, 4, 4, 1)}
# persistent 2-D variant: (STAGES, TH, TW) per id, mirror of KDL_S2DP_CONFIGS (LDS sizing)
S2DP = {184: (4, 6, 16), 185: (4, 4, 16), 186: (3, 4, 16), 187: (4, 8, 16), 188: (6, 6, 16), 189: (4, 4, 16),
        190: (8, 4, 16), 191: (11, 4, 16), 192: (7, 6, 16)}
# DMA-wave variant (sepconv_2dw_kernel): no C tile / bias in LDS
S2DW = {200: (4, 4, 16), 201: (4, 8, 16), 202: (4, 6, 16), 203: (4, 4, 16), 204: (6, 8, 16)}
SEP_BASE = 64
SEPW_BASE = 120   # warp-specialized variant (sepconv_ws.hip)
S2D_BASE = 160    # 2-D spatial tiles (sepconv_2d.hip): the early flow's 147x147 / 74x74 maps
C3_BASE = 208     # 2-D tiled 3x3 conv, cin 32 (conv3x3_2d.hip): block1_conv2
S2D_MIN_W = 64    # 16-pixel tile rows waste too much of a narrower map (37 -> 48, 19 -> 32)
# x-band KiB per stage of each KDL_SEPW_CONFIGS entry (mirror of sepconv_ws_fits)
SEPW_XB = {120: 9, 121: 9, 122: 11, 123: 16, 124: 9, 125: 8, 126: 9, 127: 9,
           135: 15, 136: 11, 137: 15, 140: 8, 141: 8, 142: 8,
           143: 9, 144: 11, 145: 16, 146: 8, 147: 9,
           128: 9, 129: 9, 130: 9, 131: 9, 132: 9, 133: 9, 148: 9, 149: 11, 156: 16, 157: 8, 158: 9}
# ids 1000..1999 were the hipBLASLt node (rounds 3-4); retired in round 5 -- every GEMM of the
# product is hand-written (the vendor library stays a measuring stick: tools/gemm_vs_vendor.py)
# ids >= SPLITK_BASE: an LDS-DMA GEMM config (16..63) with K split over ksplit workgroups per tile
# (gemm_pipe.hip ConvGemmArgs.ksplit): SPLITK_BASE + 100 * ksplit + base id
SPLITK_BASE = 2000
# STREAM_BASE: persistent streaming pointwise GEMM with the weights resident in LDS (gemm_stream.hip;
# MODE_PW stride 1; only the (K/32, ldy/16) instances in STREAM_SHAPES (bf16: EfficientNet-B7's
# large-map expand / project convs) and STREAM_SHAPES_F16 (fp16: ResNet-50's 56x56 1x1 convs)). Stores all ldy channels, so its nominal tile is 16 x 32.
# STREAM_NT: the same with nontemporal output stores (outputs far past the 256 MB MALL).
STREAM_BASE = 3000
STREAM_NT = 3001
STREAM_IDS = (STREAM_BASE, STREAM_NT)
STREAM_SHAPES = frozenset([(1, 2), (2, 2), (1, 12), (6, 4), (2, 18), (9, 4), (9, 6), (3, 30), (15, 6)])
# fp16 instances (dt 1): ResNet-50's layer1 / layer2.0 1x1 convs at 56x56 (gemm_stream.hip KDL_STREAM_SHAPES_F16)
STREAM_SHAPES_F16 = frozenset([(2, 4), (2, 16), (8, 4), (8, 8)])
# never autotune candidates: the ws stamping build and band ablation
ABLATION_IDS = frozenset([127, 147, 128, 129, 130, 131, 132, 133])


def s2dp_smem(cfg: int, K: int) -> int:
    """LDS bytes of a persistent 2-D sepconv config (mirror of s2dp_smem / launch_s2dw in sepconv_2d.hip)."""
    st, th, tw = S2DP[cfg] if cfg in S2DP else S2DW[cfg]
    bm, bn = cfg_tile(cfg)
    ipp = ((th + 2) * (tw + 2) + 1 + 63) // 64
    kt = K // 32
    if cfg in S2DW:
        return kt * (bn // 16) * 1024 + kt * 1024 + st * 4 * ipp * 1024 + 2 * (bm // 16) * 1024
    return kt * (bn // 16) * 1024 + kt * 1024 + st * 4 * ipp * 1024 + 2 * (bm // 16) * 1024 + bm * (bn * 2 + 16) + 1024


def config_applicable(cfg: int, W: int | None, K: int | None = None, n: int | None = None) -> bool:
    """Mirror of the host-side launch checks in sepconv_ws.hip / sepconv_2d.hip / conv3x3_2d.hip."""
    if cfg >= C3_BASE:    # one N tile of all outputs, 32 input channels (K = 288)
        return (K is None or K == 288) and (n is None or round_up(n, cfg_tile(cfg)[1]) == cfg_tile(cfg)[1])
    if cfg < SEP_BASE or W is None:
        return True
    if cfg in S2DP or cfg in S2DW:   # one N tile (all of N) with the whole K x N weight block resident in LDS
        return (W >= S2D_MIN_W and (K is None or s2dp_smem(cfg, K) <= 160 * 1024)
                and (n is None or round_up(n, cfg_tile(cfg)[1]) == cfg_tile(cfg)[1]))
    if cfg >= S2D_BASE:
        return W >= S2D_MIN_W
    if cfg >= SEPW_BASE:
        return cfg_tile(cfg)[0] + 2 * W + 3 <= SEPW_XB[cfg] * 16
    return False


def is_splitk(cfg: int) -> bool:
    return SPLITK_BASE <= cfg < STREAM_BASE


def splitk_parts(cfg: int) -> tuple[int, int]:
    """split-K id -> (ksplit, base LDS-DMA GEMM config)."""
    return (cfg - SPLITK_BASE) // 100, (cfg - SPLITK_BASE) % 100


def splitk_id(ksplit: int, base: int) -> int:
    assert 2 <= ksplit <= 16 and PIPE_BASE <= base < SEP_BASE, (ksplit, base)
    return SPLITK_BASE + 100 * ksplit + base


def cfg_tile(cfg: int) -> tuple[int, int]:
    if cfg in STREAM_IDS:
        return 16, 32
    if is_splitk(cfg):
        cfg = splitk_parts(cfg)[1]
    fm, fn, wgm, wgn = CONFIGS[cfg]
    return 16 * fm * wgm, 16 * fn * wgn


def candidate_configs(n: int, m: int | None = None, mode: int | None = None) -> list[int]:
    """Configs whose N tile does not waste more than ~35% of the channels (the fused
    separable ids >= SEP_BASE only for MODE_DW layers)."""
    ids = sorted(c for c in CONFIGS if c not in ABLATION_IDS
                 and (mode is None or (c < SEP_BASE) or (mode == MODE_DW and c < C3_BASE)
                      or (mode == MODE_CONV and c >= C3_BASE)))
    out = [c for c in ids if round_up(n, cfg_tile(c)[1]) <= 1.35 * round_up(n, 16)]
    if not any(c < SEP_BASE for c in out):   # tiny N: always keep the plain GEMMs with the smallest N tile
        plain = [c for c in ids if c < SEP_BASE]
        bn_min = min(cfg_tile(c)[1] for c in plain)
        out = sorted(out + [c for c in plain if cfg_tile(c)[1] == bn_min])
    return out


def default_config(mode: int, n: int, m: int) -> int:
    cands = candidate_configs(n, m, mode)
    pref = [4, 6, 3, 2, 1, 0] if mode == MODE_DW else [16, 21, 18, 17, 19, 3, 6, 1, 2, 0]
    # (fused-separable ids are picked by the autotuner, which knows the image width)
    for c in pref:
        if c in cands:
            return c
    return cands[0]


@dataclass
class Geometry:
    B: int
    H: int
    W: int
    OH: int
    OW: int

    @property
    def M(self) -> int:
        return self.B * self.OH * self.OW


class ConvGemmLayer:
    """A 1x1 / strided 1x1 / 3x3-valid / separable conv with fused BN(+ReLU)(+add).

    ``w_nk``: folded weights [N][K] in the kernel's K order (K = padded cin for
    pointwise, 9*padded cin for 3x3 with k = tap*cin + c). ``bias``: [N].
    ``dww``: MODE_DW depthwise weights [9][padded cin] fp32.
    """

    def __init__(self, name: str, mode: int, w_nk: torch.Tensor, bias: torch.Tensor, *,
                 cin_pad: int, n: int, stride: int = 1, dww: torch.Tensor | None = None,
                 relu_in: bool = False, relu_out: bool | int = False, device="cuda",
                 candidates: list[int] | None = None, dtype: torch.dtype = torch.bfloat16,
                 ksplit: tuple = ()):
        """``dtype``: element type of the activations and packed weights, bf16 (default)
        or fp16 (MODE_PW / MODE_CONV only; ``dt`` = 1 in the launch args).
        ``ksplit``: split-K factors to offer with the LDS-DMA GEMM tiles of at most 160 rows
        (ids >= SPLITK_BASE; for layers whose M fills few CUs: ResNet-50 layer3/4)."""
        assert dtype in (torch.bfloat16, torch.float16), dtype
        assert dtype == torch.bfloat16 or mode != MODE_DW, "fused separable convs are bf16-only"
        self.dtype, self.dt = dtype, int(dtype == torch.float16)
        self.name, self.mode, self.n = name, mode, n
        self.cin_pad, self.stride = cin_pad, stride
        # relu_out: 0/False none, 1/True ReLU before the residual add, 2 ReLU after it
        self.relu_in, self.relu_out = relu_in, int(relu_out)
        self.K = w_nk.shape[1]
        assert self.K % 32 == 0, (name, self.K)
        self.ldy = round_up(n, 32)
        self.candidates = candidates if candidates is not None else candidate_configs(n, mode=mode)
        self.nf_max = max(round_up(n, cfg_tile(c)[1]) // 16 for c in self.candidates)
        self.cfg = default_config(mode, n, 0) if candidates is None else self.candidates[0]
        if self.cfg not in self.candidates:
            self.cfg = self.candidates[0]
        self.wp = pack_fragments(w_nk, self.nf_max, self.K // 32, dtype).to(device).contiguous()
        self.bias = pad_vec(bias, self.nf_max * 16).to(device)
        self.dww = None
        self.dwk = None
        # LDS-DMA pipelined GEMM configs: every M tile walks K from its own start step
        # (ConvGemmArgs.krot); engines enable it where measured (ResNet-50: +3 %)
        self.krot = 0
        if mode == MODE_DW:
            assert dww is not None and dww.shape == (9, cin_pad)
            self.dww = dww.float().contiguous().to(device)
            self.dwk = pack_dw_entries(dww).to(device)
        # keep an fp32 copy of the exact (bf16-rounded) weights for reference checks
        self.w_ref = w_nk.to(dtype).float()
        self.ksplit = tuple(ksplit)
        assert not self.ksplit or mode in (MODE_PW, MODE_CONV, MODE_DW), (name, "split-K: LDS-DMA GEMM lowerings only")
        self._splitk_bufs: tuple | None = None     # (fp32 partials, per-tile counters), grown on demand
        # MODE_DW lowering: fused (dw in the GEMM's A producer) or split (dw3x3
        # kernel into a scratch buffer, then the MODE_PW GEMM). Autotuned.
        self.split = False

    def variants(self, W: int | None = None) -> list[tuple[bool, int]]:
        """(split, cfg) pairs valid for this layer (``W``: image width, filters the
        fused separable configs whose LDS row band would not fit)."""
        skv = [(False, splitk_id(sk, c)) for sk in self.ksplit for c in self.candidates
               if PIPE_BASE <= c < SEP_BASE and cfg_tile(c)[0] <= 160 and (self.K // 32) % sk == 0]
        if self.mode == MODE_CONV:
            return [(False, c) for c in self.candidates
                    if c < SEP_BASE or (c >= C3_BASE and self.stride == 1 and config_applicable(c, W, self.K, self.n))] + skv
        if self.mode != MODE_DW:
            return ([(False, c) for c in self.candidates if c < SEP_BASE] + skv
                    + ([(False, c) for c in STREAM_IDS] if self.stream_ok() else []))
        # separable conv: fused configs, or the split lowering (depthwise, then a plain GEMM -- split-K too)
        return ([(False, c) for c in self.candidates
                 if (c < PIPE_BASE or c >= SEP_BASE) and config_applicable(c, W, self.K, self.n)]
                + [(True, c) for c in self.candidates if c < SEP_BASE] + [(True, c) for _, c in skv])

    def stream_ok(self, res: bool = False) -> bool:
        """The streaming GEMM has an instance for this layer (host mirror of gemm_stream's checks;
        the packed weights must hold all ldy / 16 fragments; residual instances up to ldy 288)."""
        if res and self.ldy > 288:
            return False
        shapes = STREAM_SHAPES if self.dt == 0 else STREAM_SHAPES_F16
        return (self.mode == MODE_PW and self.stride == 1 and not self.relu_in
                and self.relu_out != 3 and (self.K // 32, self.ldy // 16) in shapes
                and self.nf_max * 16 >= self.ldy)

    def dw_args(self, x: int, tmp: int, g: Geometry, ldx: int | None = None) -> dict:
        assert (ldx or self.cin_pad) == self.cin_pad
        return dict(x=x, w=_lib.ptr(self.dww), y=tmp, B=g.B, H=g.H, W=g.W, C=self.cin_pad,
                    relu_in=int(self.relu_in))

    def emit(self, prog, x: int, y: int, g: Geometry, res: int | None = None, ldx: int | None = None,
             ldr: int | None = None, tmp: int | None = None, split: bool | None = None,
             cfg: int | None = None, opad: int = 0,
             ascale: tuple[int, int] | None = None) -> None:
        """Append this layer's launches to a native Program (or launch now if prog is None).
        ``ascale``: (pointer, per-image stride) of fp32 per-image channel scales applied to the A
        operand (ConvGemmArgs.ascale; LDS-DMA / streaming GEMM configs, bf16 pointwise only)."""
        split = self.split if split is None else split
        cfg = self.cfg if cfg is None else cfg
        C = _lib.lib()
        if self.mode == MODE_DW and split:
            assert tmp is not None, "split separable conv needs a scratch buffer"
            da = self.dw_args(x, tmp, g, ldx)
            if is_splitk(cfg):
                sk, cfg = splitk_parts(cfg)
                ga = self.args(tmp, y, g, res, ldx=self.cin_pad, ldr=ldr, cfg=cfg, opad=opad)
                ws, cnt = self._splitk_workspace(sk, cfg, g.M)
                ga.update(ksplit=sk, ws=_lib.ptr(ws), cnt=_lib.ptr(cnt))
            else:
                ga = self.args(tmp, y, g, res, ldx=self.cin_pad, ldr=ldr, cfg=cfg, opad=opad)
            if prog is None:
                s = _lib.stream_ptr()
                C.dw3x3(da, s)
                C.conv_gemm(MODE_PW, cfg, ga, s)
            else:
                prog.add_dw(self.name + "/dw", da)
                prog.add_conv_gemm(self.name, MODE_PW, cfg, ga)
            return
        if is_splitk(cfg):
            sk, cfg = splitk_parts(cfg)
            assert ascale is None and (self.K // 32) % sk == 0, (self.name, sk)
            ga = self.args(x, y, g, res, ldx=ldx, ldr=ldr, cfg=cfg, opad=opad)
            ws, cnt = self._splitk_workspace(sk, cfg, g.M)
            ga.update(ksplit=sk, ws=_lib.ptr(ws), cnt=_lib.ptr(cnt))
            if prog is None:
                C.conv_gemm(self.mode, cfg, ga, _lib.stream_ptr())
            else:
                prog.add_conv_gemm(self.name, self.mode, cfg, ga)
            return
        ga = self.args(x, y, g, res, ldx=ldx, ldr=ldr, cfg=cfg, opad=opad)
        if ascale:
            assert (PIPE_BASE <= cfg < SEP_BASE or cfg in STREAM_IDS) and self.mode == MODE_PW and \
                self.dt == 0, \
                "A-operand channel scales ride the bf16 pointwise LDS-DMA pipelined or streaming GEMM"
            ga.update(ascale=ascale[0], ascale_ld=ascale[1])
        if prog is None:
            C.conv_gemm(self.mode, cfg, ga, _lib.stream_ptr())
        else:
            prog.add_conv_gemm(self.name, self.mode, cfg, ga)

    def _splitk_workspace(self, ksplit: int, cfg: int, M: int):
        """fp32 partials [ksplit][tiles][BM*BN] and zeroed per-tile counters (the last split of a tile
        resets its counter, so graph replays need no memset). One pair per layer, grown to the largest
        request: a layer's launches never overlap (one stream per engine / pipeline stage)."""
        bm, bn = cfg_tile(cfg)
        tiles = -(-M // bm) * (self.nf(cfg) * 16 // bn)
        need_ws, need_cnt = ksplit * tiles * bm * bn, tiles
        cur = self._splitk_bufs
        if cur is None or cur[0].numel() < need_ws or cur[1].numel() < need_cnt:
            dev = self.wp.device
            n_ws = max(need_ws, cur[0].numel() if cur else 0)
            n_cnt = max(need_cnt, cur[1].numel() if cur else 0)
            self._splitk_bufs = (torch.zeros(n_ws, dtype=torch.float32, device=dev),
                                 torch.zeros(n_cnt, dtype=torch.int32, device=dev))
            self._splitk_old = getattr(self, "_splitk_old", []) + ([cur] if cur else [])   # captured graphs may hold them
        return self._splitk_bufs

    def nf(self, cfg: int | None = None) -> int:
        cfg = self.cfg if cfg is None else cfg
        return round_up(self.n, cfg_tile(cfg)[1]) // 16

    def args(self, x: int, y: int, g: Geometry, res: int | None = None, ldx: int | None = None,
             ldr: int | None = None, cfg: int | None = None, opad: int = 0) -> dict:
        return dict(x=x, wp=_lib.ptr(self.wp), bias=_lib.ptr(self.bias),
                    dww=_lib.ptr(self.dww), dwk=_lib.ptr(self.dwk), res=res, y=y,
                    B=g.B, H=g.H, W=g.W, OH=g.OH, OW=g.OW, M=g.M,
                    ldx=ldx if ldx is not None else self.cin_pad, ldy=self.ldy,
                    ldr=ldr if ldr is not None else self.ldy,
                    K=self.K, cin=self.cin_pad, NF=self.nf(cfg), nstore=self.ldy,
                    stride=self.stride, relu_in=int(self.relu_in), relu_out=int(self.relu_out),
                    opad=int(opad), dt=self.dt, krot=int(self.krot))

    def launch(self, x: torch.Tensor, y: torch.Tensor, g: Geometry, res: torch.Tensor | None = None,
               cfg: int | None = None, split: bool = False, tmp: torch.Tensor | None = None,
               opad: int = 0) -> None:
        """Eager launch on torch tensors (shape-checked on the host first)."""
        self.check(x, y, g, res, opad)
        if split:
            if tmp is None:
                tmp = torch.empty(g.M * self.cin_pad, dtype=torch.bfloat16, device=x.device)
            assert tmp.numel() >= g.M * self.cin_pad
        self.emit(None, _lib.ptr(x), _lib.ptr(y), g, _lib.ptr(res), tmp=_lib.ptr(tmp), split=split, cfg=cfg,
                  opad=opad)

    def check(self, x, y, g: Geometry, res=None, opad: int = 0) -> None:
        assert x.dtype == self.dtype and y.dtype == self.dtype, (x.dtype, y.dtype, self.dtype)
        assert x.is_contiguous() and y.is_contiguous()
        assert x.numel() >= g.B * g.H * g.W * self.cin_pad, (self.name, x.shape)
        assert y.numel() >= g.B * (g.OH + 2 * opad) * (g.OW + 2 * opad) * self.ldy, (self.name, y.shape)
        if self.mode == MODE_DW:
            assert g.OH == g.H and g.OW == g.W
        elif self.mode == MODE_CONV:
            assert g.OH == (g.H - 3) // self.stride + 1 and g.OW == (g.W - 3) // self.stride + 1
        else:
            assert g.OH == (g.H - 1) // self.stride + 1 and g.OW == (g.W - 1) // self.stride + 1
        if res is not None:
            assert res.dtype == self.dtype and res.numel() >= g.M * self.ldy


def pack_dw_entries(dww: torch.Tensor) -> torch.Tensor:
    """Depthwise weights [9][C] -> the per-k-step weight entries of the fused separable
    kernels, bf16 [C/32][g 2][n 16][parity 2][8]: entry (g, n, p) holds w[p + 2j][32t + 16g + n]
    for j = 0..4 (0 past tap 8), one 16-byte LDS read per lane (sepconv_ws.hip: the depthwise
    3x3 as a block-diagonal 16x16x32 MFMA B operand)."""
    C = dww.shape[1]
    w = torch.cat([dww.float(), torch.zeros(1, C)], 0)          # taps 0..9
    w = w.view(5, 2, C // 32, 2, 16)                           # [j][parity][t][g][n]
    e = w.permute(2, 3, 4, 1, 0)                               # [t][g][n][parity][j]
    e = torch.cat([e, torch.zeros(*e.shape[:-1], 3)], -1)      # j padded to 8
    return e.to(torch.bfloat16).contiguous()


def conv_weights_nk(kernel_hwio: torch.Tensor, cin_pad: int) -> torch.Tensor:
    """Keras HWIO kernel -> [N][K] with k = (dy*kw+dx)*cin_pad + c."""
    kh, kw, cin, cout = kernel_hwio.shape
    w = torch.zeros(kh * kw, cin_pad, cout, dtype=torch.float64)
    w[:, :cin, :] = kernel_hwio.double().reshape(kh * kw, cin, cout)
    return w.reshape(kh * kw * cin_pad, cout).t().contiguous()
