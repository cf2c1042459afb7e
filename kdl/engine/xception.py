"""MI355X executor for Keras Xception (+ clothing head).

Walks ``kdl.models.xception.SPEC`` and lowers it to fused HIP launches:

    stem_conv            block1_conv1 + BN + ReLU (normalisation folded, uint8 in)
    conv_gemm MODE_CONV  block1_conv2 3x3 + BN + ReLU (implicit GEMM)
    conv_gemm MODE_DW    every SeparableConv2D + BN (+ReLU in/out)(+residual add)
    conv_gemm MODE_PW    residual 1x1/2 convs + BN
    pool_add             TF-'same' 3x3/2 max-pool + residual add
    entry_block          blocks 2 and 3 (both separable convs, the pool and the residual conv)
                         as ONE persistent launch each (kdl/ops/entry_block.py; KDL_ENTRY_BLOCK)
    head_dense           GAP -> Dense(100)+ReLU -> Dense(10) logits

= 44 launches per forward with the tuned table (vs ~168 unfused TF ops; split
separable convs count twice: depthwise + GEMM), captured into
one hipGraph per batch bucket. All buffers are allocated once for the largest
bucket (static memory plan); smaller buckets use prefixes of the same buffers.
The reference equivalent is TF-Serving's SavedModel session run
(`tf-serving.dockerfile:2-5`).
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

from ..models import xception as X
from ..models.layers import tf_same_pad
from ..ops import _lib
from ..ops.conv import MODE_CONV, MODE_DW, MODE_PW, ConvGemmLayer, Geometry, conv_weights_nk
from ..ops.pack import bn_scale_shift, pack_fragments, round_up, rowrun_weights
from .base import EngineBase, Step


class XceptionEngine(EngineBase):
    model_name = "xception"

    def __init__(self, params: dict, max_batch: int = 32, device: str | torch.device = "cuda",
                 in_kind: str = "u8", head: X.Head = X.DEFAULT_HEAD, buckets=None,
                 tune_file: str | Path | None = None):
        super().__init__(device, max_batch, buckets)
        self.in_kind = in_kind
        self.head = head
        # fused entry blocks (entry_block.hip): block numbers lowered to one launch each.
        # KDL_ENTRY_BLOCK: a list "2,3" / "2:4,3" (block[:kernel config]), "1" = blocks 2 and 3,
        # "0" = none. Default "2:15,3": block2 on the warp-specialized kernel (producer waves run the
        # depthwise of later rows while consumer waves run the GEMMs of earlier ones and one dw2 unit
        # each; config 13 +0.8 % over the round-4 default 2:2 in 4 of 4 interleaved pairs, config 15
        # +1.0 % over 13 in 3 of 3) and block3, whose lighter stage 1 moves the stage cut to
        # block8_sepconv3 (profiles/entry_block_ab_r4.txt)
        eb = os.environ.get("KDL_ENTRY_BLOCK", "2:15,3")
        spec = "2,3" if eb == "1" else ("" if eb == "0" else eb)
        self.fused_blocks = {}
        for v in filter(None, (x.strip() for x in spec.split(","))):
            blk, _, cfg = v.partition(":")
            self.fused_blocks[int(blk)] = int(cfg) if cfg else None
        self.size = X.INPUT_SIZE
        self.shapes: dict[str, tuple[int, int, int]] = {}  # buffer -> (H, W, C) per image
        self._build(params)
        self._alloc()
        if tune_file and Path(tune_file).exists():
            self.load_tuning(tune_file)

    # ------------------------------------------------------------------ lowering
    def _build(self, p: dict) -> None:
        dev = self.device
        S = self.size
        st = X.SPEC
        # --- stem 1: 3x3/2 valid, 3 -> 32, folded BN (+ folded normalisation for uint8)
        c1 = st[0].main[0]
        s, t = bn_scale_shift(p, c1.bn)
        w = p[f"{c1.name}/kernel"].double().reshape(27, 32).t() * s[:, None]   # [32][27], k = tap*3+c
        if self.in_kind == "u8":
            bias = t - w.sum(1)
            w = w / 127.5
        else:
            bias = t
        oh1 = (S - 3) // 2 + 1
        # uint8 input: row-run K layout (k = ky*16 + kx*3 + c, 2 k-steps; stem_rows_kernel)
        self.stem_rows = self.in_kind == "u8" and os.environ.get("KDL_STEM_ROWS", "1") != "0"
        if self.stem_rows:
            self.stem_wp = pack_fragments(rowrun_weights(w, 3, 9, 16), 2, 2).to(dev).contiguous()
        else:
            self.stem_wp = pack_fragments(w, 2, 1).to(dev).contiguous()
        self.stem_bias = bias.float().to(dev)
        self.steps.append(Step("stem", c1.name, src="input", dst="stem1", geom=(S, S, oh1, oh1)))
        self.shapes["stem1"] = (oh1, oh1, 32)
        # --- stem 2: 3x3 valid 32 -> 64 implicit GEMM
        c2 = st[0].main[1]
        s, t = bn_scale_shift(p, c2.bn)
        w = conv_weights_nk(p[f"{c2.name}/kernel"], 32) * s[:, None]
        lay = ConvGemmLayer(c2.name, MODE_CONV, w, t, cin_pad=32, n=64, relu_out=True, device=dev)
        h = oh1 - 2
        self.steps.append(Step("conv", c2.name, lay, "stem1", "stem2", geom=(oh1, oh1, h, h)))
        self.shapes["stem2"] = (h, h, 64)
        cur, H = "stem2", h
        for bi, blk in enumerate(st[1:], start=1):
            if blk.kind in ("entry", "exit"):
                rc = blk.res_conv
                oh = (H - 1) // 2 + 1
                rname = f"{rc.name}_out"
                lay = self._pw(p, rc, dev)
                _, pt, _ = tf_same_pad(H, 3, 2)
                out = f"block{bi + 1}_out"
                if bi + 1 in self.fused_blocks:
                    from ..ops.entry_block import EntryBlock
                    s1, s2 = (self._sep(p, op, dev) for op in blk.main)
                    # KDL_ENTRY_GRID: workgroups per fused block launch (default one per CU per
                    # resident workgroup); fewer leave CUs to the other pipeline stage
                    g = os.environ.get("KDL_ENTRY_GRID")
                    fb = EntryBlock(f"block{bi + 1}", s1, s2, lay, cfg=self.fused_blocks[bi + 1], device=dev,
                                    grid=int(g) if g else None)
                    self.steps.append(Step("block", f"block{bi + 1}", src=cur, dst=out, geom=(H, H, oh, oh),
                                           extra=dict(eb=fb)))
                    self.shapes[out] = (oh, oh, s2.ldy)
                    cur, H = out, oh
                    continue
                self.steps.append(Step("conv", rc.name, lay, cur, rname, geom=(H, H, oh, oh)))
                self.shapes[rname] = (oh, oh, lay.ldy)
                y = cur
                for op in blk.main:
                    lay = self._sep(p, op, dev)
                    dst = f"{op.name}_out"
                    self.steps.append(Step("conv", op.name, lay, y, dst, geom=(H, H, H, H)))
                    self.shapes[dst] = (H, H, lay.ldy)
                    y = dst
                C = self.shapes[y][2]
                self.steps.append(Step("pool", f"block{bi + 1}_pool", src=y, dst=out, res=rname,
                                       geom=(H, H, oh, oh), extra=dict(pad=pt, C=C)))
                self.shapes[out] = (oh, oh, C)
                cur, H = out, oh
            elif blk.kind == "middle":
                y = cur
                for k, op in enumerate(blk.main):
                    lay = self._sep(p, op, dev)
                    dst = f"{op.name}_out"
                    res = cur if k == len(blk.main) - 1 else None
                    self.steps.append(Step("conv", op.name, lay, y, dst, res=res, geom=(H, H, H, H)))
                    self.shapes[dst] = (H, H, lay.ldy)
                    y = dst
                cur = y
            else:  # block14
                for op in blk.main:
                    lay = self._sep(p, op, dev)
                    dst = f"{op.name}_out"
                    self.steps.append(Step("conv", op.name, lay, cur, dst, geom=(H, H, H, H)))
                    self.shapes[dst] = (H, H, lay.ldy)
                    cur = dst
        # --- head
        hd = self.head
        self.w1 = p[f"{hd.hidden}/kernel"].float().t().contiguous().to(dev)   # Keras [F][H1] -> [H1][F]
        self.b1 = p[f"{hd.hidden}/bias"].float().to(dev)
        self.w2 = p[f"{hd.out}/kernel"].float().contiguous().to(dev)      # Keras [H1][NC]
        self.b2 = p[f"{hd.out}/bias"].float().to(dev)
        self.steps.append(Step("head", "head", src=cur, dst="logits", geom=(H, H, 1, 1)))
        self.feat_buf = cur
        self._hoist_relus()

    def _hoist_relus(self) -> None:
        """Move each pre-activation ReLU of a separable conv into its producer's
        epilogue when that producer's output feeds nothing else: relu(bf16(v)) ==
        bf16(relu(v)), so results are bit-identical, and the ReLU runs once per output
        element in the GEMM epilogue instead of once per depthwise tap read (9x, on the
        VALU of the fused kernels and the dw3x3 staging). The block inputs of the
        middle flow keep theirs: they are also the (pre-ReLU) residual."""
        uses: dict[str, int] = {}
        for st in self.steps:
            for b in (st.src, st.res):
                if b:
                    uses[b] = uses.get(b, 0) + 1
        for a, b in zip(self.steps, self.steps[1:]):
            if (a.kind == "conv" and b.kind == "conv" and b.src == a.dst and uses.get(a.dst) == 1
                    and a.res is None and a.layer.relu_out == 0 and b.layer.mode == MODE_DW and b.layer.relu_in):
                a.layer.relu_out, b.layer.relu_in = 1, False

    @staticmethod
    def _pw(p, rc, dev) -> ConvGemmLayer:
        s, t = bn_scale_shift(p, rc.bn)
        cin_pad = round_up(rc.cin, 32)
        w = torch.zeros(rc.cout, cin_pad, dtype=torch.float64)
        w[:, :rc.cin] = p[f"{rc.name}/kernel"].double()[0, 0].t() * s[:, None]
        return ConvGemmLayer(rc.name, MODE_PW, w, t, cin_pad=cin_pad, n=rc.cout, stride=2, device=dev)

    @staticmethod
    def _sep(p, op, dev) -> ConvGemmLayer:
        s, t = bn_scale_shift(p, op.bn)
        cin_pad = round_up(op.cin, 32)
        w = torch.zeros(op.cout, cin_pad, dtype=torch.float64)
        w[:, :op.cin] = p[f"{op.name}/pointwise_kernel"].double()[0, 0].t() * s[:, None]
        dww = torch.zeros(9, cin_pad, dtype=torch.float32)
        dww[:, :op.cin] = p[f"{op.name}/depthwise_kernel"].float()[:, :, :, 0].reshape(9, op.cin)
        # block14 (10x10 maps: M = 3,200 rows at batch 32, 160-200 output tiles): split-K candidates
        # for its split lowering's GEMM
        return ConvGemmLayer(op.name, MODE_DW, w, t, cin_pad=cin_pad, n=op.cout, dww=dww,
                             relu_in=op.relu_in, relu_out=op.relu_out, device=dev,
                             ksplit=(2, 3, 4) if op.cout >= 1536 else ())

    def _alloc(self) -> None:
        B, S, dev = self.max_batch, self.size, self.device
        if self.in_kind == "u8":
            self.inp = torch.zeros((B, S, S, 3), dtype=torch.uint8, device=dev)
        else:
            self.inp = torch.zeros((B, S, S, 3), dtype=torch.float32, device=dev)
        self.bufs: dict[str, torch.Tensor] = {}
        for name, (h, w, c) in self.shapes.items():
            self.bufs[name] = torch.zeros(B * h * w * c, dtype=torch.bfloat16, device=dev)
        self.logits = torch.zeros((B, self.head.classes), dtype=torch.float32, device=dev)
        self.head_feat = torch.zeros((B, self.head.features), dtype=torch.float32, device=dev)
        self.head_hid = torch.zeros((self.head.features // 64, B, self.head.hidden_units), dtype=torch.float32,
                                    device=dev)   # dense1 K-split partials
        # scratch for split separable convs (depthwise output), sized for the largest layer
        n = 1
        for st in self.conv_steps():
            if st.layer.mode == MODE_DW:
                H, W, _, _ = st.geom
                n = max(n, B * H * W * st.layer.cin_pad)
        self.dwtmp = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        self.bufs["__dwtmp"] = self.dwtmp     # by name, so stages.py can give each stage its own

    # ------------------------------------------------------------------ programs
    def _ptr(self, name: str) -> int:
        if name == "input":
            return self.input_ptr()
        if name == "logits":
            return self.output_ptr()
        return _lib.ptr(self.bufs[self._remap.get(name, name)])


    def scratch_buffers(self) -> list[str]:
        """Buffers a step uses that are not its src / dst / res (stages.py privatises them)."""
        return ["__dwtmp"]

    def _emit(self, prog, step: Step, b: int) -> None:
        H, W, OH, OW = step.geom
        if step.kind == "stem":
            prog.add_stem(step.name, dict(x=self.input_ptr(), wp=_lib.ptr(self.stem_wp),
                                          bias=_lib.ptr(self.stem_bias), y=self._ptr(step.dst),
                                          B=b, H=H, W=W, OH=OH, OW=OW, ldy=32,
                                          in_kind=0 if self.in_kind == "u8" else 1, rows=int(self.stem_rows)))
        elif step.kind == "conv":
            self._emit_conv(prog, step, b)
        elif step.kind == "pool":
            prog.add_pool_add(step.name, dict(x=self._ptr(step.src), res=self._ptr(step.res),
                                              y=self._ptr(step.dst), B=b, H=H, W=W, OH=OH, OW=OW,
                                              C=step.extra["C"], pad_top=step.extra["pad"],
                                              pad_left=step.extra["pad"]))
        elif step.kind == "block":
            step.extra["eb"].emit(prog, self._ptr(step.src), self._ptr(step.dst), b, H, W)
        elif step.kind == "head":
            hd = self.head
            prog.add_head(step.name, dict(x=self._ptr(step.src), w1=_lib.ptr(self.w1),
                                          b1=_lib.ptr(self.b1), w2=_lib.ptr(self.w2),
                                          b2=_lib.ptr(self.b2), out=self._ptr("logits"),
                                          feat=_lib.ptr(self.head_feat), hid=_lib.ptr(self.head_hid),
                                          B=b, HW=H * W, ldx=self.shapes[step.src][2],
                                          F=hd.features, H1=hd.hidden_units, NC=hd.classes))

    def _emit_conv(self, prog, step: Step, b: int, split=None, cfg=None) -> None:
        H, W, OH, OW = step.geom
        step.layer.emit(prog, self._ptr(step.src), self._ptr(step.dst), Geometry(b, H, W, OH, OW),
                        res=self._ptr(step.res) if step.res else None, ldx=self.shapes[step.src][2],
                        ldr=self.shapes[step.res][2] if step.res else None, tmp=self._ptr("__dwtmp"),
                        split=split, cfg=cfg)

    def flops_per_image(self) -> float:
        return 2 * 8.356e9
