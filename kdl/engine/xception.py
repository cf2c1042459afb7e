"""MI355X executor for Keras Xception (+ clothing head).

Walks ``kdl.models.xception.SPEC`` and lowers it to fused HIP launches:

    stem_conv            block1_conv1 + BN + ReLU (normalisation folded, uint8 in)
    conv_gemm MODE_CONV  block1_conv2 3x3 + BN + ReLU (implicit GEMM)
    conv_gemm MODE_DW    every SeparableConv2D + BN (+ReLU in/out)(+residual add)
    conv_gemm MODE_PW    residual 1x1/2 convs + BN (KDL_POOLFUSE=1: with the block's
                         3x3/2 max-pool of the main branch added in the epilogue, "convpool")
    seppool              KDL_SEP_POOL=1: an entry block's last SeparableConv2D + its 3x3/2
                         max-pool + the residual add in ONE kernel (sepconv_2dwp_kernel,
                         "seppool" steps; measured slower, off by default); otherwise:
    pool_add             TF-'same' 3x3/2 max-pool + residual add
    head_dense           GAP -> Dense(100)+ReLU -> Dense(10) logits

    chain                KDL_CHAIN=<ws cfg>: the middle flow's separable convs as ONE ticketed
                         launch per program (sepconv_chain_kernel; off by default, see __init__)

= 41 launches per forward (vs ~168 unfused TF ops), captured into
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
from ..ops.conv import (CHAIN_CONFIGS, MODE_CONV, MODE_DW, MODE_PW, SEPW_BASE, ConvGemmLayer, Geometry,
                        cfg_tile, config_applicable, conv_weights_nk, pool_configs)
from ..ops.pack import bn_scale_shift, pack_fragments, round_up, rowrun_weights
from .base import EngineBase, Step


CHAIN_MAX_LAYERS = 32          # launch.h ChainArgs::MAXL


class XceptionEngine(EngineBase):
    model_name = "xception"

    def __init__(self, params: dict, max_batch: int = 32, device: str | torch.device = "cuda",
                 in_kind: str = "u8", head: X.Head = X.DEFAULT_HEAD, buckets=None,
                 tune_file: str | Path | None = None):
        super().__init__(device, max_batch, buckets)
        self.in_kind = in_kind
        self.head = head
        # KDL_BRANCHES=1: residual convs on a side branch of the captured graph. Off by
        # default: a forked hipGraph measured 16 % SLOWER in the stage-pipelined bench
        # (17.7k vs 21.1k img/s, profiles/stages_ab.txt) -- the graph's second branch
        # competes for the hardware queues the two stages already use
        self.branches = int(os.environ.get("KDL_BRANCHES", "0"))
        # KDL_POOLFUSE=1: residual 1x1/2 conv + block max-pool as ONE launch (the pool in the
        # conv's epilogue, step kind "convpool"). Off by default: measured 3 % SLOWER in the
        # stage-pipelined bench (20.8-20.9k vs 21.5k img/s, same box): the epilogue's nine
        # dependent 16-B pool reads per output chunk are latency-bound inside the GEMM's store
        # loop, so the fused launch (80.8 us at block2) costs what conv + pool_add did (82.6)
        self.poolfuse = os.environ.get("KDL_POOLFUSE", "0") == "1" and not self.branches
        # KDL_SEP_POOL=1: the block's last separable conv writes maxpool + residual directly
        # (sepconv_2dwp_kernel); bit-identical to conv + pool_add. Off by default: block2's
        # pooled launch took 275 us vs ~170 for sepconv + pool_add (it recomputes the pool
        # windows' overlap rows), 20.5-21.1k vs 22.6k img/s in the pipelined bench
        # (profiles/seppool_chain_ab_r3.txt)
        self.seppool = os.environ.get("KDL_SEP_POOL", "0") == "1" and not self.poolfuse
        self.seppool_cfg = int(os.environ.get("KDL_SEP_POOL_CFG", "0"))
        # KDL_CHAIN=<cfg> (0 = off): each run of same-geometry separable convs inside one
        # program (the middle flow: blocks 5-12, split only at a stage cut) becomes ONE chained
        # launch (sepconv_chain_kernel, launch.h ChainArgs) with that ws tile. Alone it is 7 %
        # faster per layer (29.6 vs ~32 us at batch 32: no launch, fill or drain per layer), but
        # in the stage-pipelined bench the other stream's kernels already fill those gaps while
        # the chain's dependency-waiting workgroups hold CUs: 21.9k vs 22.5k img/s
        # (profiles/seppool_chain_ab_r3.txt). Off by default.
        self.chain_cfg = int(os.environ.get("KDL_CHAIN", "0"))
        self.chain_min = int(os.environ.get("KDL_CHAIN_MIN", "2"))      # shortest run worth chaining
        self._chain_sync: dict[tuple, torch.Tensor] = {}
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
                rlay = lay
                if not self.poolfuse:
                    # the residual 1x1/2 conv only depends on the block input: in the captured
                    # graph it may run on a side branch beside the block's separable convs
                    self.steps.append(Step("conv", rc.name, lay, cur, rname, geom=(H, H, oh, oh),
                                           extra=dict(branch=self.branches)))
                    self.shapes[rname] = (oh, oh, lay.ldy)
                y = cur
                _, pt, _ = tf_same_pad(H, 3, 2)
                out = f"block{bi + 1}_out"
                pooled = False
                for k, op in enumerate(blk.main):
                    lay = self._sep(p, op, dev)
                    dst = f"{op.name}_out"
                    pcfgs = pool_configs(lay.K, lay.n, pt) if self.seppool and k == len(blk.main) - 1 else []
                    if pcfgs and rlay.ldy == lay.ldy:
                        # separable conv + block max-pool + residual in one kernel: no full-res output
                        cfg = self.seppool_cfg if self.seppool_cfg in pcfgs else pcfgs[0]
                        self.steps.append(Step("seppool", op.name, lay, y, out, res=rname, geom=(H, H, oh, oh),
                                               extra=dict(pad=pt, cfg=cfg)))
                        self.shapes[out] = (oh, oh, lay.ldy)
                        pooled = True
                        break
                    self.steps.append(Step("conv", op.name, lay, y, dst, geom=(H, H, H, H)))
                    self.shapes[dst] = (H, H, lay.ldy)
                    y = dst
                if pooled:
                    cur, H = out, oh
                    continue
                C = self.shapes[y][2]
                if self.poolfuse:
                    # residual conv of the block input, + maxpool(main branch) in its epilogue,
                    # straight into the block output (reads: src = block input, res = main branch)
                    assert rlay.ldy == C, (rc.name, rlay.ldy, C)
                    self.steps.append(Step("convpool", rc.name, rlay, cur, out, res=y, geom=(H, H, oh, oh),
                                           extra=dict(pad=pt)))
                else:
                    self.steps.append(Step("pool", f"block{bi + 1}_pool", src=y, dst=out, res=rname,
                                           geom=(H, H, oh, oh), extra=dict(pad=pt, C=C, join=self.branches)))
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
            if (a.kind == "conv" and b.kind in ("conv", "seppool") and b.src == a.dst and uses.get(a.dst) == 1
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
        return ConvGemmLayer(op.name, MODE_DW, w, t, cin_pad=cin_pad, n=op.cout, dww=dww,
                             relu_in=op.relu_in, relu_out=op.relu_out, device=dev)

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
        elif step.kind in ("conv", "convpool", "seppool"):
            self._emit_conv(prog, step, b)
        elif step.kind == "pool":
            prog.add_pool_add(step.name, dict(x=self._ptr(step.src), res=self._ptr(step.res),
                                              y=self._ptr(step.dst), B=b, H=H, W=W, OH=OH, OW=OW,
                                              C=step.extra["C"], pad_top=step.extra["pad"],
                                              pad_left=step.extra["pad"]))
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
        if step.kind == "seppool":
            step.layer.emit(prog, self._ptr(step.src), self._ptr(step.dst), Geometry(b, H, W, OH, OW),
                            res=self._ptr(step.res), ldx=self.shapes[step.src][2], ldr=self.shapes[step.res][2],
                            split=False, cfg=step.extra["cfg"], pool=dict(ppad=step.extra["pad"]))
            return
        if step.kind == "convpool":
            ph, pw, pc = self.shapes[step.res]
            step.layer.emit(prog, self._ptr(step.src), self._ptr(step.dst), Geometry(b, H, W, OH, OW),
                            ldx=self.shapes[step.src][2], split=split, cfg=cfg,
                            pool=dict(px=self._ptr(step.res), pH=ph, pW=pw, pld=pc, ppad=step.extra["pad"]))
            return
        step.layer.emit(prog, self._ptr(step.src), self._ptr(step.dst), Geometry(b, H, W, OH, OW),
                        res=self._ptr(step.res) if step.res else None, ldx=self.shapes[step.src][2],
                        ldr=self.shapes[step.res][2] if step.res else None, tmp=self._ptr("__dwtmp"),
                        split=split, cfg=cfg)

    # ------------------------------------------------------------------ chained middle flow
    def _chainable(self, st: Step, first: Step | None) -> bool:
        lay = st.layer
        if (st.kind != "conv" or lay.mode != MODE_DW or lay.split or st.extra.get("branch") or st.extra.get("join")
                or st.geom[0] != st.geom[2] or st.geom[1] != st.geom[3] or lay.relu_out not in (0, 1)):
            return False
        if first is None:
            return (self.chain_cfg in CHAIN_CONFIGS and config_applicable(self.chain_cfg, st.geom[1], lay.K, lay.n)
                    and cfg_tile(self.chain_cfg)[0] >= st.geom[1] + 1)   # 3x3 halo within M tiles mi +- 1
        f = first.layer
        return (st.geom == first.geom and lay.K == f.K and lay.n == f.n and lay.cin_pad == f.cin_pad
                and self.shapes[st.src][2] == self.shapes[first.src][2]
                and (st.res is None or self.shapes[st.res][2] == lay.ldy))

    def _chain_end(self, steps: list[Step], i: int) -> int:
        if not self.chain_cfg or not self._chainable(steps[i], None):
            return i + 1
        j = i + 1
        while j < len(steps) and j - i < CHAIN_MAX_LAYERS and self._chainable(steps[j], steps[i]):
            j += 1
        return j if j - i >= self.chain_min else i + 1

    def chain_layer_args(self, steps: list[Step], b: int, maps: list[dict] | None = None) -> dict:
        """Launch arguments of one chained launch over ``steps`` (see launch.h ChainArgs)."""
        cfg = self.chain_cfg
        layers, g0 = [], None
        for k, st in enumerate(steps):
            self._remap = maps[k] if maps else {}
            H, W, OH, OW = st.geom
            a = st.layer.args(self._ptr(st.src), self._ptr(st.dst), Geometry(b, H, W, OH, OW),
                              self._ptr(st.res) if st.res else None, ldx=self.shapes[st.src][2],
                              ldr=self.shapes[st.res][2] if st.res else None, cfg=cfg)
            if g0 is None:
                g0 = dict(a, relu_out=0, relu_in=0)
            else:
                for key in ("B", "H", "W", "M", "ldx", "ldy", "K", "NF", "nstore"):
                    assert a[key] == g0[key], (st.name, key, a[key], g0[key])
            if a["res"] is not None:
                assert a["ldr"] == g0["ldy"], (st.name, a["ldr"])
            layers.append({k2: a[k2] for k2 in ("x", "wp", "dwk", "res", "y", "bias", "relu_in", "relu_out")})
        g0["ldr"] = g0["ldy"]
        nM, nN = _lib.lib().sepconv_chain_tiles(cfg - SEPW_BASE, g0["M"], g0["NF"])
        # bounded waits: ~1 us per poll, so a lost dependency costs a wait ~0.3 s, not a hang
        return dict(g=g0, layers=layers, nM=nM, nN=nN, spin_limit=1 << 18)

    def _emit_chain(self, prog, steps: list[Step], maps: list[dict], b: int) -> None:
        d = self.chain_layer_args(steps, b, maps)
        key = (self._slot, b, tuple(st.name for st in steps), tuple(tuple(sorted(m.items())) for m in maps))
        n = 4 + len(steps) * d["nM"]
        sync = self._chain_sync.get(key)
        if sync is None:
            # one counter block per (program, chain): programs of other slots / parities may run
            # concurrently on other streams
            sync = self._chain_sync[key] = torch.zeros(round_up(n, 64), dtype=torch.int32, device=self.device)
        d["sync"] = _lib.ptr(sync)       # zeroed by the launch itself (chain_reset_kernel)
        prog.add_chain(f"chain[{steps[0].name}..{steps[-1].name}]", self.chain_cfg - SEPW_BASE, d)

    def flops_per_image(self) -> float:
        return 2 * 8.356e9
