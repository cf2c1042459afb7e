"""MI355X executor for EfficientNet-B7 at 600x600 (BASELINE.json
config 4: the large-activation / LDS-tiling stress case).

Lowering (captured into one hipGraph per batch bucket):

    stem_conv       3x3/2 pad 1, 3 -> 64 + BN + SiLU, mean/std applied on load
    per MBConv (55):
      conv_gemm PW  expand 1x1 + BN + SiLU                  (expand ratio 6 blocks)
      dwk           KxK/S depthwise + BN + SiLU; SE average pool + squeeze FC fused
                    (per-tile partials of fc1, which is linear in the pooled mean)
      se            SE tail: sum parts + bias + SiLU, fc2 + sigmoid -> per-(image, channel) scale
      conv_gemm PW  project 1x1 + BN (+ identity residual), the SE scale applied to its A
                    operand (the depthwise output) between LDS / registers and the MFMAs, per
                    image and channel (ConvGemmArgs.ascale; round 6: replaced per-image copies of
                    the project weights written by an extra launch, +3.1 % img/s,
                    profiles/b7_se_apath_r6.txt). KDL_SEFOLD=0 rewrites the depthwise output in
                    place instead ("chscale", a read + write of the largest tensors)
    conv_gemm PW    head 1x1 640 -> 2560 + BN + SiLU
    gap + fc_mfma   global pool (bf16) -> classifier 2560 -> 1000

(A fused expand + depthwise kernel that kept the expanded tensor in LDS was measured
2x slower than this unfused pair -- per 32-channel block the workgroup waited a full
memory round trip for the next block's parameters, profiles/entry_flow_r2.txt -- and
was removed in round 3.)

Activations are NHWC bf16 with channels padded to multiples of 32 (zeros); the
largest tensor (stage-2 expand at 300x300x192) is 34.6 MB per image, so at batch
32 the static plan is ~2 GB -- trivial against 288 GB of HBM3E.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

from ..models import efficientnet as E
from ..ops import _lib
from ..ops.conv import MODE_PW, PIPE_BASE, SEP_BASE, ConvGemmLayer, Geometry, default_config
from ..ops.pack import pack_fragments, round_up
from .base import EngineBase, Step


def _fold(p, conv, bn):
    w = p[conv].double()
    s = p[f"{bn}.weight"].double() / torch.sqrt(p[f"{bn}.running_var"].double() + E.BN_EPS)
    t = p[f"{bn}.bias"].double() - p[f"{bn}.running_mean"].double() * s
    return w, s, t


class EfficientNetEngine(EngineBase):
    model_name = "efficientnet_b7"

    def __init__(self, params: dict, max_batch: int = 32, device: str | torch.device = "cuda",
                 buckets=None, tune_file: str | Path | None = None, size: int = E.INPUT_SIZE):
        super().__init__(device, max_batch, buckets)
        self.size = size
        self.sefold = os.environ.get("KDL_SEFOLD", "1") != "0"   # SE scale on the project GEMM's A operand
        self.classes = params["classifier.1.bias"].numel()
        self.bufsz: dict[str, int] = {}            # buffer -> elements per image (max over uses)
        self._build(params)
        self._alloc()
        if tune_file and Path(tune_file).exists():
            self.load_tuning(tune_file)

    def _need(self, name: str, per_image: int) -> None:
        self.bufsz[name] = max(self.bufsz.get(name, 0), per_image)

    def _pw(self, name, p, conv, bn, cin, cout, act):
        w, s, t = _fold(p, conv, bn)
        cin_pad = round_up(cin, 32)
        wn = torch.zeros(cout, cin_pad, dtype=torch.float64)
        wn[:, :cin] = w[:, :, 0, 0] * s[:, None]
        return ConvGemmLayer(name, MODE_PW, wn, t, cin_pad=cin_pad, n=cout, relu_out=act, device=self.device)

    def _build(self, p: dict) -> None:
        dev = self.device
        w, s, t = _fold(p, "features.0.0.weight", "features.0.1")
        wnk = (w.permute(0, 2, 3, 1).reshape(E.STEM, 27) * s[:, None])
        self.stem_wp = pack_fragments(wnk, E.STEM // 16, 1).to(dev).contiguous()
        self.stem_b = t.float().to(dev)
        H = (self.size + 2 - 3) // 2 + 1
        self.steps.append(Step("stem", "stem", src="input", dst="X0", geom=(self.size, self.size, H, H)))
        self._need("X0", H * H * E.STEM)
        cur, ldc, ping = "X0", E.STEM, 0
        self.dw, self.se = {}, {}
        C = _lib.lib()
        for blk in E.blocks():
            n = blk.names()
            ce = blk.cexp
            oh = (H + 2 * ((blk.k - 1) // 2) - blk.k) // blk.stride + 1
            src = cur
            wd, sd, td = _fold(p, f"{n['dw']}.0.weight", f"{n['dw']}.1")
            dww = (wd[:, 0] * sd[:, None, None]).permute(1, 2, 0).reshape(blk.k * blk.k, ce)
            self.dw[blk.prefix] = (dww.float().contiguous().to(dev), td.float().to(dev))
            se = n["se"]
            self.se[blk.prefix] = (p[f"{se}.fc1.weight"].reshape(blk.csq, ce).float().contiguous().to(dev),
                                   p[f"{se}.fc1.bias"].float().to(dev),
                                   p[f"{se}.fc2.weight"].reshape(ce, blk.csq).t().float().contiguous().to(dev),
                                   p[f"{se}.fc2.bias"].float().to(dev))
            if "expand" in n:
                lay = self._pw(n["expand"], p, f"{n['expand']}.0.weight", f"{n['expand']}.1", blk.cin, ce, 4)
                self.steps.append(Step("conv", lay.name, lay, cur, "E", geom=(H, H, H, H), extra=dict(ldx=ldc)))
                self._need("E", H * H * ce)
                src = "E"
            self.steps.append(Step("dwk", f"{blk.prefix}.dw", src=src, dst="D", geom=(H, H, oh, oh),
                                   extra=dict(C=ce, Cs=blk.csq, K=blk.k, S=blk.stride, blk=blk.prefix)))
            self._need("D", oh * oh * ce)
            self.steps.append(Step("se", f"{blk.prefix}.se", src="pool", dst="scale", geom=(H, H, oh, oh),
                                   extra=dict(C=ce, Cs=blk.csq, K=blk.k, S=blk.stride, blk=blk.prefix)))
            ping ^= 1
            out = f"X{ping}"
            lay = self._pw(n["project"], p, f"{n['project']}.0.weight", f"{n['project']}.1", ce, blk.cout, 0)
            if self.sefold:
                # the SE scale rides the project GEMM's A operand: the LDS-DMA GEMM with per-image
                # M tiles, or the streaming GEMM (its table ids are accepted by apply_tuning)
                lay.candidates = [c for c in lay.candidates if PIPE_BASE <= c < SEP_BASE]
                if lay.cfg not in lay.candidates:
                    lay.cfg = default_config(MODE_PW, blk.cout, 0) if default_config(MODE_PW, blk.cout, 0) in \
                        lay.candidates else lay.candidates[0]
            else:
                # in place on D (src == dst); reads the SE scales
                self.steps.append(Step("chscale", f"{blk.prefix}.scale", src="D", dst="D", res="scale",
                                       geom=(oh, oh, oh, oh), extra=dict(C=ce)))
            self.steps.append(Step("conv", lay.name, lay, "D", out, res=cur if blk.residual else None,
                                   geom=(oh, oh, oh, oh),
                                   extra=dict(ldx=ce, ldr=ldc, ascale=ce if self.sefold else 0)))
            self._need(out, oh * oh * lay.ldy)
            cur, ldc, H = out, lay.ldy, oh
        lay = self._pw("features.8", p, "features.8.0.weight", "features.8.1", E.blocks()[-1].cout, E.HEAD, 4)
        self.steps.append(Step("conv", lay.name, lay, cur, "E", geom=(H, H, H, H), extra=dict(ldx=ldc)))
        self._need("E", H * H * E.HEAD)
        self.steps.append(Step("gap", "avgpool", src="E", dst="feat", geom=(H, H, 1, 1)))
        nf = (self.classes + 15) // 16
        self.fc_wp = pack_fragments(p["classifier.1.weight"].float(), nf, E.HEAD // 32).to(dev).contiguous()
        self.fc_nf = nf
        self.fc_b = p["classifier.1.bias"].float().to(dev)
        self.steps.append(Step("fc", "classifier", src="feat", dst="logits"))
        # SE pooling partials: ntiles of each dw launch (host mirror of the kernel's tiling)
        self.ntiles = {}
        mx = 1
        for st in self.steps:
            if st.kind == "dwk":
                H_, W_, oh_, ow_ = st.geom
                g = dict(B=1, H=H_, W=W_, C=st.extra["C"], OH=oh_, OW=ow_, K=st.extra["K"], S=st.extra["S"],
                         pad=(st.extra["K"] - 1) // 2, Cs=st.extra["Cs"])
                nt = C.dwk_tiles(g)[3]
                self.ntiles[st.extra["blk"]] = nt
                mx = max(mx, nt * st.extra["Cs"])
        self.pool_per_image = mx

    def _alloc(self) -> None:
        B, S, dev = self.max_batch, self.size, self.device
        self.inp = torch.zeros((B, S, S, 3), dtype=torch.uint8, device=dev)
        self.bufs = {k: torch.zeros(B * v, dtype=torch.bfloat16, device=dev) for k, v in self.bufsz.items()}
        self.pool = torch.zeros(B * self.pool_per_image, dtype=torch.float32, device=dev)
        self.scale = torch.zeros(B * max(b.cexp for b in E.blocks()), dtype=torch.float32, device=dev)
        self.feat = torch.zeros(((B + 15) // 16 * 16, E.HEAD), dtype=torch.bfloat16, device=dev)
        # by name, so stages.py can version / privatise them like the activations
        self.bufs.update(pool=self.pool, scale=self.scale, feat=self.feat)
        self.logits = torch.zeros((B, self.classes), dtype=torch.float32, device=dev)

    def _ptr(self, name: str) -> int:
        if name == "logits":
            return self.output_ptr()
        return _lib.ptr(self.bufs[self._remap.get(name, name)])

    def scratch_buffers(self) -> list[str]:
        """SE partial pools (written by the dw kernel, not a step dst) and scales: used
        within one block, so each pipeline stage gets its own (stages.py)."""
        return ["pool", "scale"]

    def _emit_conv(self, prog, step: Step, b: int, split=None, cfg=None) -> None:
        H, W, OH, OW = step.geom
        ascale = (self._ptr("scale"), step.extra["ascale"]) if step.extra.get("ascale") else None
        step.layer.emit(prog, self._ptr(step.src), self._ptr(step.dst), Geometry(b, H, W, OH, OW),
                        res=self._ptr(step.res) if step.res else None, ldx=step.extra["ldx"],
                        ldr=step.extra.get("ldr") if step.res else None, split=False, cfg=cfg,
                        ascale=ascale)

    def _emit(self, prog, step: Step, b: int) -> None:
        H, W, OH, OW = step.geom if step.geom else (0, 0, 0, 0)
        if step.kind == "stem":
            sc = [1.0 / (255.0 * s) for s in E.STD]
            sh = [-m / s for m, s in zip(E.MEAN, E.STD)]
            prog.add_stem(step.name, dict(x=self.input_ptr(), wp=_lib.ptr(self.stem_wp), bias=_lib.ptr(self.stem_b),
                                          y=self._ptr("X0"), B=b, H=H, W=W, OH=OH, OW=OW, ldy=E.STEM, in_kind=0,
                                          KH=3, KW=3, stride=2, pad=1, cout=E.STEM, relu=2,
                                          scale0=sc[0], scale1=sc[1], scale2=sc[2],
                                          shift0=sh[0], shift1=sh[1], shift2=sh[2]))
        elif step.kind == "conv":
            self._emit_conv(prog, step, b)
        elif step.kind == "dwk":
            w, bias = self.dw[step.extra["blk"]]
            w1 = self.se[step.extra["blk"]][0]
            K = step.extra["K"]
            prog.add_dwk(step.name, dict(x=self._ptr(step.src), w=_lib.ptr(w), bias=_lib.ptr(bias),
                                         y=self._ptr("D"), pool=self._ptr("pool"), w1=_lib.ptr(w1),
                                         Cs=step.extra["Cs"], B=b, H=H, W=W, C=step.extra["C"], OH=OH, OW=OW,
                                         K=K, S=step.extra["S"], pad=(K - 1) // 2, act=2))
        elif step.kind == "se":
            _, b1, w2t, b2 = self.se[step.extra["blk"]]
            prog.add_se(step.name, dict(pool=self._ptr("pool"), b1=_lib.ptr(b1),
                                        w2t=_lib.ptr(w2t), b2=_lib.ptr(b2), scale=self._ptr("scale"), B=b,
                                        ntiles=self.ntiles[step.extra["blk"]], HW=OH * OW, C=step.extra["C"],
                                        Cs=step.extra["Cs"]))
        elif step.kind == "chscale":
            prog.add_chscale(step.name, dict(y=self._ptr("D"), scale=self._ptr("scale"), B=b, HW=OH * OW,
                                             C=step.extra["C"]))
        elif step.kind == "gap":
            prog.add_gap(step.name, dict(x=self._ptr("E"), y=None, yb=self._ptr("feat"), B=b, HW=H * W,
                                         ldx=E.HEAD, F=E.HEAD))
        elif step.kind == "fc":
            prog.add_fc_mfma(step.name, dict(xb=self._ptr("feat"), wp=_lib.ptr(self.fc_wp),
                                             bias=_lib.ptr(self.fc_b), out=self.output_ptr(), B=b, F=E.HEAD,
                                             N=self.classes, NF=self.fc_nf, relu=0))
        else:  # pragma: no cover
            raise ValueError(step.kind)

    def flops_per_image(self) -> float:
        return 2.0 * E.macs_per_image(self.size)
