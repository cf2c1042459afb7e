"""MI355X executor for ViT-B/16 (BASELINE.json config 5).

Lowering (captured into one hipGraph per batch bucket; rows = B*197 tokens):

    patchify        uint8 image -> [B*196][768] bf16 patches, mean/std on load
    conv_gemm PW    patch embedding 768 -> 768 (+bias), written straight into token
                    rows 1..196 of each image (opad=2: the class token keeps row 0)
    embed           row 0 := cls + pos[0]; rows += pos[t]
    per layer (12):
      layernorm     ln_1
      conv_gemm PW  QKV 768 -> 2304 (+bias)
      attention     flash-style MFMA attention, 12 heads x 64, online softmax
      conv_gemm PW  out_proj 768 -> 768 (+bias) + residual (in place on X)
      layernorm     ln_2
      conv_gemm PW  mlp.0 768 -> 3072 (+bias, exact GELU epilogue)
      conv_gemm PW  mlp.3 3072 -> 768 (+bias) + residual (in place on X)
    layernorm       encoder.ln on the 32 class-token rows only
    fc_mfma         head 768 -> 1000

= 3 + 12*7 + 2 = 89 launches. Every linear layer runs on the same pipelined
LDS-DMA MFMA GEMM as the CNNs (a 1x1 conv over a 1 x rows "image").

fp8=True (BASELINE.json "fp8 MFMA" config): the four linears of every layer run on
gemm_f8.hip (OCP e4m3 x e4m3, block-scaled MFMA 16x16x128); ln_1 / ln_2 /
attention / the GELU GEMM write e4m3 directly with static per-tensor scales
calibrated on the fp32 oracle (amax x 1.25 / 448); weights per output channel.
The residual stream, QKV, softmax and the patch embedding / head stay bf16/fp32.
"""
from __future__ import annotations

from pathlib import Path

import torch

from ..models import vit as V
from ..ops import _lib
from ..ops.conv import MODE_PW, ConvGemmLayer, Geometry
from ..ops.pack import pack_fragments
from .base import EngineBase, Step


class ViTEngine(EngineBase):
    model_name = "vit_b16"

    def __init__(self, params: dict, max_batch: int = 32, device: str | torch.device = "cuda",
                 buckets=None, tune_file: str | Path | None = None, fp8: bool = False,
                 calib: torch.Tensor | None = None, calib_margin: float = 1.25):
        super().__init__(device, max_batch, buckets)
        self.fp8 = fp8
        if fp8:
            self.model_name = "vit_b16_fp8"
            if calib is None:   # synthetic calibration batch (serving would use real images)
                calib = torch.randint(0, 256, (2, V.INPUT_SIZE, V.INPUT_SIZE, 3),
                                      generator=torch.Generator().manual_seed(1234), dtype=torch.uint8)
            self.amax = V.activation_amax(params, calib)
            self.calib_margin = calib_margin
        self.size = V.INPUT_SIZE
        self.T = V.TOKENS
        self.np = self.T - 1
        self.classes = params["heads.head.bias"].numel()
        self._build(params)
        self._alloc()
        if tune_file and Path(tune_file).exists():
            self.load_tuning(tune_file)

    def _lin(self, name: str, w: torch.Tensor, b: torch.Tensor, relu_out: int = 0) -> ConvGemmLayer:
        # every linear is a hand-written MFMA GEMM (the hipBLASLt candidate of rounds 3-4 is gone:
        # tools/gemm_vs_vendor.py keeps the vendor as the yardstick). split-K candidates: N = 768 outputs (out_proj, mlp.3) are 120 tiles of 160 x 256 at the
        # bench's 6,304 token rows, under half of the 256 CUs; 2-4 splits fill the chip
        lay = ConvGemmLayer(name, MODE_PW, w.double(), b.float(), cin_pad=w.shape[1], n=w.shape[0],
                            relu_out=relu_out, device=self.device,
                            ksplit=(2, 3, 4) if w.shape[0] <= 768 and w.shape[1] % 384 == 0 else ())
        lay.krot = 1    # K-rotated LDS-DMA GEMM: bf16 +0.6 % img/s, p50 -2.9 % (profiles/krot_ab.txt)
        return lay

    def _build(self, p: dict) -> None:
        dev, D = self.device, V.DIM
        self.ln = {}
        self.steps.append(Step("patchify", "patchify", src="input", dst="patches"))
        w = p["conv_proj.weight"].reshape(D, 3 * V.PATCH * V.PATCH)
        self.steps.append(Step("conv", "conv_proj", self._lin("conv_proj", w, p["conv_proj.bias"]),
                               "patches", "X", extra=dict(kind="patch")))
        self.cls = p["class_token"].reshape(D).float().to(dev)
        self.pos = p["encoder.pos_embedding"].reshape(self.T, D).float().contiguous().to(dev)
        self.steps.append(Step("embed", "embed", src="X", dst="X"))       # in place on the patch embeddings
        self.f8scale: dict[str, float] = {}
        for i in range(V.DEPTH):
            L = f"encoder.layers.encoder_layer_{i}"
            self.ln[f"{L}.ln_1"] = (p[f"{L}.ln_1.weight"].float().to(dev), p[f"{L}.ln_1.bias"].float().to(dev))
            self.ln[f"{L}.ln_2"] = (p[f"{L}.ln_2.weight"].float().to(dev), p[f"{L}.ln_2.bias"].float().to(dev))
            if self.fp8:
                self._build_layer_f8(p, i, L)
                continue
            self.steps.append(Step("ln", f"{L}.ln_1", src="X", dst="Xn"))
            self.steps.append(Step("conv", f"{L}.qkv", self._lin(
                f"{L}.qkv", p[f"{L}.self_attention.in_proj_weight"], p[f"{L}.self_attention.in_proj_bias"]),
                "Xn", "QKV"))
            self.steps.append(Step("attn", f"{L}.attn", src="QKV", dst="A"))
            self.steps.append(Step("conv", f"{L}.out_proj", self._lin(
                f"{L}.out_proj", p[f"{L}.self_attention.out_proj.weight"],
                p[f"{L}.self_attention.out_proj.bias"]), "A", "X", res="X"))
            self.steps.append(Step("ln", f"{L}.ln_2", src="X", dst="Xn"))
            self.steps.append(Step("conv", f"{L}.mlp.0", self._lin(
                f"{L}.mlp.0", p[f"{L}.mlp.0.weight"], p[f"{L}.mlp.0.bias"], relu_out=3), "Xn", "Hd"))
            self.steps.append(Step("conv", f"{L}.mlp.3", self._lin(
                f"{L}.mlp.3", p[f"{L}.mlp.3.weight"], p[f"{L}.mlp.3.bias"]), "Hd", "X", res="X"))
        self.ln["encoder.ln"] = (p["encoder.ln.weight"].float().to(dev), p["encoder.ln.bias"].float().to(dev))
        self.steps.append(Step("ln", "encoder.ln", src="X", dst="CLS", extra=dict(cls_only=True)))
        nf = (self.classes + 15) // 16
        self.head_wp = pack_fragments(p["heads.head.weight"].float(), nf, D // 32).to(dev).contiguous()
        self.head_nf = nf
        self.head_b = p["heads.head.bias"].float().to(dev)
        self.steps.append(Step("fc", "heads.head", src="CLS", dst="logits"))

    def _build_layer_f8(self, p: dict, i: int, L: str) -> None:
        """One encoder layer with all four linears on the e4m3 GEMM (static scales)."""
        from ..ops.f8 import E4M3_MAX, F8Linear
        sc = {k: v * self.calib_margin / E4M3_MAX for k, v in self.amax[i].items()}
        for k, v in sc.items():
            self.f8scale[f"{L}.{k}"] = v
        dev = self.device
        self.steps.append(Step("ln", f"{L}.ln_1", src="X", dst="Xn8", extra=dict(out_scale=sc["ln_1"])))
        self.steps.append(Step("f8", f"{L}.qkv", F8Linear(
            f"{L}.qkv", p[f"{L}.self_attention.in_proj_weight"], p[f"{L}.self_attention.in_proj_bias"], sc["ln_1"],
            device=dev), "Xn8", "QKV"))
        self.steps.append(Step("attn", f"{L}.attn", src="QKV", dst="A8", extra=dict(out_scale=sc["attn"])))
        self.steps.append(Step("f8", f"{L}.out_proj", F8Linear(
            f"{L}.out_proj", p[f"{L}.self_attention.out_proj.weight"], p[f"{L}.self_attention.out_proj.bias"],
            sc["attn"], device=dev), "A8", "X", res="X"))
        self.steps.append(Step("ln", f"{L}.ln_2", src="X", dst="Xn8", extra=dict(out_scale=sc["ln_2"])))
        self.steps.append(Step("f8", f"{L}.mlp.0", F8Linear(
            f"{L}.mlp.0", p[f"{L}.mlp.0.weight"], p[f"{L}.mlp.0.bias"], sc["ln_2"], relu_out=3, device=dev),
            "Xn8", "Hd8", extra=dict(out_scale=sc["gelu"])))
        self.steps.append(Step("f8", f"{L}.mlp.3", F8Linear(
            f"{L}.mlp.3", p[f"{L}.mlp.3.weight"], p[f"{L}.mlp.3.bias"], sc["gelu"], device=dev),
            "Hd8", "X", res="X"))

    def _alloc(self) -> None:
        B, S, dev, D, T = self.max_batch, self.size, self.device, V.DIM, self.T
        self.inp = torch.zeros((B, S, S, 3), dtype=torch.uint8, device=dev)
        z = lambda *shape: torch.zeros(*shape, dtype=torch.bfloat16, device=dev)  # noqa: E731
        self.bufs = {"patches": z(B * self.np, D), "X": z(B * T, D), "Xn": z(B * T, D),
                     "QKV": z(B * T, 3 * D), "A": z(B * T, D), "Hd": z(B * T, V.MLP),
                     "CLS": z((B + 15) // 16 * 16, D)}
        self.ld = {"patches": D, "X": D, "Xn": D, "QKV": 3 * D, "A": D, "Hd": V.MLP, "CLS": D}
        if self.fp8:
            u8 = lambda *shape: torch.zeros(*shape, dtype=torch.uint8, device=dev)  # noqa: E731
            self.bufs.update({"Xn8": u8(B * T, D), "A8": u8(B * T, D), "Hd8": u8(B * T, V.MLP)})
            self.ld.update({"Xn8": D, "A8": D, "Hd8": V.MLP})
        self.logits = torch.zeros((B, self.classes), dtype=torch.float32, device=dev)

    def _ptr(self, name: str) -> int:
        return _lib.ptr(self.bufs[self._remap.get(name, name)])

    def scratch_buffers(self) -> list[str]:
        return []

    def _emit_conv(self, prog, step: Step, b: int, split=None, cfg=None) -> None:
        if step.kind == "f8":
            out_scale = step.extra.get("out_scale")
            kw = dict(x8=self._ptr(step.src), M=b * self.T, res=self._ptr(step.res) if step.res else None,
                      ldy=self.ld[step.dst])
            if out_scale is not None:
                kw.update(y8=self._wptr(step.dst), out_scale=out_scale)
            else:
                kw.update(y=self._wptr(step.dst))
            step.layer.emit(prog, cfg=cfg, **kw)
            return
        lay: ConvGemmLayer = step.layer
        if step.extra.get("kind") == "patch":
            g = Geometry(b, V.INPUT_SIZE // V.PATCH, V.INPUT_SIZE // V.PATCH,
                         V.INPUT_SIZE // V.PATCH, V.INPUT_SIZE // V.PATCH)
            opad = 2
        else:
            rows = b * self.T
            g = Geometry(1, 1, rows, 1, rows)
            opad = 0
        lay.emit(prog, self._ptr(step.src), self._wptr(step.dst), g,
                 res=self._ptr(step.res) if step.res else None, ldx=self.ld[step.src],
                 ldr=self.ld[step.res] if step.res else None, split=False, cfg=cfg, opad=opad)

    def _variants(self, step: Step):
        return step.layer.variants(None)

    def _emit(self, prog, step: Step, b: int) -> None:
        D = V.DIM
        if step.kind == "patchify":
            sc = [1.0 / (255.0 * s) for s in V.STD]
            sh = [-m / s for m, s in zip(V.MEAN, V.STD)]
            prog.add_patchify(step.name, dict(x=self.input_ptr(), y=self._ptr("patches"), B=b, H=self.size,
                                              W=self.size, P=V.PATCH, ldy=D, scale0=sc[0], scale1=sc[1],
                                              scale2=sc[2], shift0=sh[0], shift1=sh[1], shift2=sh[2]))
        elif step.kind in ("conv", "f8"):
            self._emit_conv(prog, step, b)
        elif step.kind == "embed":
            prog.add_embed(step.name, dict(x=self._ptr("X"), cls=_lib.ptr(self.cls), pos=_lib.ptr(self.pos),
                                           B=b, T=self.T, D=D))
        elif step.kind == "ln":
            g, bb = self.ln[step.name]
            if step.extra.get("cls_only"):
                prog.add_layernorm(step.name, dict(x=self._ptr("X"), y=self._ptr("CLS"), gamma=_lib.ptr(g),
                                                   beta=_lib.ptr(bb), rows=b, D=D, ldx=self.T * D, ldy=D,
                                                   eps=V.LN_EPS))
            else:
                osc = step.extra.get("out_scale")
                out = dict(y8=self._ptr(step.dst), inv_scale=1.0 / osc) if osc else dict(y=self._ptr(step.dst))
                prog.add_layernorm(step.name, dict(x=self._ptr(step.src), gamma=_lib.ptr(g), beta=_lib.ptr(bb),
                                                   rows=b * self.T, D=D, ldx=D, ldy=D, eps=V.LN_EPS, **out))
        elif step.kind == "attn":
            osc = step.extra.get("out_scale")
            out = dict(out8=self._ptr(step.dst), inv_scale=1.0 / osc) if osc else dict(out=self._ptr(step.dst))
            prog.add_attention(step.name, dict(qkv=self._ptr("QKV"), B=b, T=self.T, H=V.HEADS, dh=D // V.HEADS,
                                               scale=(D // V.HEADS) ** -0.5, **out))
        elif step.kind == "fc":
            prog.add_fc_mfma(step.name, dict(xb=self._ptr("CLS"), wp=_lib.ptr(self.head_wp),
                                             bias=_lib.ptr(self.head_b), out=self.output_ptr(), B=b, F=D,
                                             N=self.classes, NF=self.head_nf, relu=0))
        else:  # pragma: no cover
            raise ValueError(step.kind)

    def flops_per_image(self) -> float:
        return 2.0 * V.macs_per_image()
