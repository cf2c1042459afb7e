"""MI355X executor for ResNet-50 v1.5 (BASELINE.json config 3).

Lowering (one launch per box, all captured into one hipGraph per batch bucket):

    stem_conv   conv1 7x7/2 pad 3 + BN + ReLU; torchvision mean/std applied on load
    pool_add    3x3/2 max-pool, pad 1 (no residual)
    per bottleneck (16):
      conv_gemm MODE_PW   conv1 1x1 + BN + ReLU, written with opad=1 into a
                          zero-bordered buffer (the 3x3 needs no bounds checks)
      conv_gemm MODE_CONV conv2 3x3 (stride 1 or 2, v1.5) + BN + ReLU, implicit GEMM
      conv_gemm MODE_PW   downsample 1x1/s + BN            (first block of a stage)
      conv_gemm MODE_PW   conv3 1x1 + BN, + shortcut, ReLU after the add (relu_out=2)
    gap + fc    global average pool (bf16 features), Dense 2048 -> 1000 on MFMA

= 2 + 16*3 + 4 + 2 = 56 launches. Buffers: block outputs ping-pong between two
slabs and each stage owns its padded / mid / shortcut scratch (a few hundred MB
at batch 32, well inside one MI355X's 288 GB and mostly MALL-resident).
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

from ..models import resnet as R
from ..ops import _lib
from ..ops.conv import MODE_CONV, MODE_PW, ConvGemmLayer, Geometry
from ..ops.pack import pack_fragments, rowrun_weights
from .base import EngineBase, Step


def _fold(p: dict, conv: str, bn: str):
    """torch conv weight [O][I][kh][kw] + BN -> (w_nk [O][K] with k = tap*I + c, bias [O])."""
    w = p[conv].double()
    g, b = p[f"{bn}.weight"].double(), p[f"{bn}.bias"].double()
    m, v = p[f"{bn}.running_mean"].double(), p[f"{bn}.running_var"].double()
    s = g / torch.sqrt(v + R.BN_EPS)
    o, i, kh, kw = w.shape
    w_nk = w.permute(0, 2, 3, 1).reshape(o, kh * kw * i) * s[:, None]
    return w_nk, b - m * s


class ResNetEngine(EngineBase):
    model_name = "resnet50"

    def __init__(self, params: dict, max_batch: int = 32, device: str | torch.device = "cuda",
                 in_kind: str = "u8", buckets=None, tune_file: str | Path | None = None,
                 dtype: str = "fp16"):
        """``dtype``: "fp16" (BASELINE.json's "ResNet-50 224x224 fp16" config: IEEE half
        activations and weights on v_mfma_f32_16x16x32_f16, fp32 accumulation) or "bf16"."""
        super().__init__(device, max_batch, buckets)
        assert in_kind in ("u8", "f32")
        assert dtype in ("fp16", "bf16"), dtype
        self.in_kind = in_kind
        self.dtype = torch.float16 if dtype == "fp16" else torch.bfloat16
        self.dt = int(dtype == "fp16")
        self.size = R.INPUT_SIZE
        self.classes = params["fc.bias"].numel()
        self.shapes: dict[str, tuple[int, int, int, int]] = {}   # buffer -> (H, W, C, border)
        self._build(params)
        self._alloc()
        if tune_file and Path(tune_file).exists():
            self.load_tuning(tune_file)

    # ------------------------------------------------------------------ lowering
    def _build(self, p: dict) -> None:
        dev = self.device
        S = self.size
        # stem: 7x7/2 pad 3. uint8 input: row-run K layout (k = ky*32 + kx*3 + c, K = 224:
        # each lane's 8 k-slots are 8 consecutive image bytes, stem_rows_kernel); otherwise
        # K = 147 (k = tap*3 + c) padded to 160
        w, t = _fold(p, "conv1.weight", "bn1")
        self.stem_rows = self.in_kind == "u8" and os.environ.get("KDL_STEM_ROWS", "1") != "0"
        if self.stem_rows:
            self.stem_wp = pack_fragments(rowrun_weights(w, 7, 21, 32), 4, 7, self.dtype).to(dev).contiguous()
        else:
            self.stem_wp = pack_fragments(w, 4, 5, self.dtype).to(dev).contiguous()
        self.stem_bias = t.float().to(dev)
        oh = (S + 6 - 7) // 2 + 1                                   # 112
        self.steps.append(Step("stem", "conv1", src="input", dst="stem", geom=(S, S, oh, oh)))
        self.shapes["stem"] = (oh, oh, 64, 0)
        ph = (oh + 2 - 3) // 2 + 1                                  # 56
        self.steps.append(Step("pool", "maxpool", src="stem", dst="pool", geom=(oh, oh, ph, ph),
                               extra=dict(C=64)))
        H, cur, ping = ph, "pool", 0
        self.shapes["pool"] = (H, H, 64, 0)
        for blk in R.blocks():
            wdt, cout = blk.width, blk.cout
            oh = (H + 2 - 3) // blk.stride + 1
            tpad, tmid = f"pad{H}_{wdt}", f"mid{oh}_{wdt}"
            self.shapes[tpad] = (H, H, wdt, 1)
            self.shapes[tmid] = (oh, oh, wdt, 0)
            w1, b1 = _fold(p, f"{blk.prefix}.conv1.weight", f"{blk.prefix}.bn1")
            # split-K candidates where the output map is 14x14 or 7x7 (layer3 / layer4): M = 32 x 196 /
            # 32 x 49 rows fill only a fraction of the 256 CUs with whole-K tiles
            sk = (2, 3, 4) if oh <= 14 else ()
            l1 = ConvGemmLayer(f"{blk.prefix}.conv1", MODE_PW, w1, b1, cin_pad=blk.cin, n=wdt,
                               relu_out=1, device=dev, dtype=self.dtype, ksplit=sk if H <= 14 else ())
            self.steps.append(Step("conv", l1.name, l1, cur, tpad, geom=(H, H, H, H), extra=dict(opad=1)))
            w2, b2 = _fold(p, f"{blk.prefix}.conv2.weight", f"{blk.prefix}.bn2")
            l2 = ConvGemmLayer(f"{blk.prefix}.conv2", MODE_CONV, w2, b2, cin_pad=wdt, n=wdt,
                               stride=blk.stride, relu_out=1, device=dev, dtype=self.dtype, ksplit=sk)
            self.steps.append(Step("conv", l2.name, l2, tpad, tmid, geom=(H + 2, H + 2, oh, oh)))
            if blk.downsample:
                sc = f"sc{oh}_{cout}"
                self.shapes[sc] = (oh, oh, cout, 0)
                wd, bd = _fold(p, f"{blk.prefix}.downsample.0.weight", f"{blk.prefix}.downsample.1")
                ld = ConvGemmLayer(f"{blk.prefix}.downsample", MODE_PW, wd, bd, cin_pad=blk.cin, n=cout,
                                   stride=blk.stride, device=dev, dtype=self.dtype)
                self.steps.append(Step("conv", ld.name, ld, cur, sc, geom=(H, H, oh, oh)))
                res = sc
            else:
                res = cur
            ping ^= 1
            out = f"out{oh}x{cout}_{ping}"      # ping-pong within a stage
            self.shapes[out] = (oh, oh, cout, 0)
            w3, b3 = _fold(p, f"{blk.prefix}.conv3.weight", f"{blk.prefix}.bn3")
            l3 = ConvGemmLayer(f"{blk.prefix}.conv3", MODE_PW, w3, b3, cin_pad=wdt, n=cout, relu_out=2,
                               device=dev, dtype=self.dtype, ksplit=sk)
            self.steps.append(Step("conv", l3.name, l3, tmid, out, res=res, geom=(oh, oh, oh, oh)))
            cur, H = out, oh
        nf = (self.classes + 15) // 16
        self.fc_wp = pack_fragments(p["fc.weight"].float(), nf, 2048 // 32, self.dtype).to(dev).contiguous()
        self.fc_nf = nf
        self.fc_b = p["fc.bias"].float().to(dev)
        self.steps.append(Step("gap", "avgpool", src=cur, dst="feat", geom=(H, H, 1, 1), extra=dict(F=2048)))
        self.steps.append(Step("fc", "fc", src="feat", dst="logits", extra=dict(F=2048)))
        # K-rotated LDS-DMA GEMMs (each M tile starts its K loop at its own step): measured
        # +3.1 % img/s, p50 -2.4 % on ResNet-50 fp16 (profiles/krot_ab.txt)
        for st in self.steps:
            if getattr(st, "layer", None) is not None:
                st.layer.krot = 1

    def _alloc(self) -> None:
        B, S, dev = self.max_batch, self.size, self.device
        dt = torch.uint8 if self.in_kind == "u8" else torch.float32
        self.inp = torch.zeros((B, S, S, 3), dtype=dt, device=dev)
        self.bufs: dict[str, torch.Tensor] = {}
        for name, (h, w, c, border) in self.shapes.items():
            n = B * (h + 2 * border) * (w + 2 * border) * c
            self.bufs[name] = torch.zeros(n, dtype=self.dtype, device=dev)   # borders stay 0
        self.feat = torch.zeros(((B + 15) // 16 * 16, 2048), dtype=self.dtype, device=dev)
        self.bufs["feat"] = self.feat
        self.logits = torch.zeros((B, self.classes), dtype=torch.float32, device=dev)

    # ------------------------------------------------------------------ emission
    def _ptr(self, name: str) -> int:
        if name == "input":
            return self.input_ptr()
        if name == "logits":
            return self.output_ptr()
        return _lib.ptr(self.bufs[self._remap.get(name, name)])

    def scratch_buffers(self) -> list[str]:
        return []

    def _ld(self, name: str) -> int:
        return self.shapes[name][2]

    def _emit_conv(self, prog, step: Step, b: int, split=None, cfg=None) -> None:
        H, W, OH, OW = step.geom
        lay: ConvGemmLayer = step.layer
        lay.emit(prog, self._ptr(step.src), self._ptr(step.dst), Geometry(b, H, W, OH, OW),
                 res=self._ptr(step.res) if step.res else None, ldx=self._ld(step.src),
                 ldr=self._ld(step.res) if step.res else None, split=False, cfg=cfg,
                 opad=step.extra.get("opad", 0))

    def _emit(self, prog, step: Step, b: int) -> None:
        H, W, OH, OW = step.geom if step.geom else (0, 0, 0, 0)
        if step.kind == "stem":
            # uint8 pixels, or (f32 signature) the same 0..255 pixel values as floats
            sc = [1.0 / (255.0 * s) for s in R.STD]
            sh = [-m / s for m, s in zip(R.MEAN, R.STD)]
            prog.add_stem(step.name, dict(x=self.input_ptr(), wp=_lib.ptr(self.stem_wp),
                                          bias=_lib.ptr(self.stem_bias), y=self._ptr(step.dst),
                                          B=b, H=H, W=W, OH=OH, OW=OW, ldy=64,
                                          in_kind=0 if self.in_kind == "u8" else 1,
                                          KH=7, KW=7, stride=2, pad=3, cout=64, relu=1,
                                          scale0=sc[0], scale1=sc[1], scale2=sc[2],
                                          shift0=sh[0], shift1=sh[1], shift2=sh[2], dt=self.dt,
                                          rows=int(self.stem_rows)))
        elif step.kind == "pool":
            prog.add_pool_add(step.name, dict(x=self._ptr(step.src), res=None, y=self._ptr(step.dst),
                                              B=b, H=H, W=W, OH=OH, OW=OW, C=step.extra["C"],
                                              pad_top=1, pad_left=1, dt=self.dt,
                                              algo=1))   # pixel-per-thread: row-streaming measured -0.3 %
        elif step.kind == "conv":
            self._emit_conv(prog, step, b)
        elif step.kind == "gap":
            prog.add_gap(step.name, dict(x=self._ptr(step.src), y=None, yb=self._ptr("feat"), B=b, HW=H * W,
                                         ldx=self._ld(step.src), F=step.extra["F"], dt=self.dt))
        elif step.kind == "fc":
            prog.add_fc_mfma(step.name, dict(xb=self._ptr("feat"), wp=_lib.ptr(self.fc_wp),
                                             bias=_lib.ptr(self.fc_b), out=self._ptr("logits"), B=b,
                                             F=step.extra["F"], N=self.classes, NF=self.fc_nf, relu=0,
                                             dt=self.dt))
        else:  # pragma: no cover
            raise ValueError(step.kind)

    def flops_per_image(self) -> float:
        return 2.0 * R.macs_per_image()

