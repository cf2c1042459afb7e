"""Model-agnostic MI355X executor machinery shared by every model family.

A model engine lowers its network into a list of ``Step`` s (fused HIP launches
over statically planned NHWC bf16 buffers). This base class owns what does not
depend on the network: one native ``Program`` per (batch bucket, capture) with
a hipGraph per bucket, per-op profiling, per-layer tile autotuning over the
conv-GEMM config table, and the tuning-table round trip
(``kdl/tuning/<model>_b<batch>.json``). The reference equivalent is a
TF-Serving servable's session run (`tf-serving.dockerfile:2-5`).
"""
from __future__ import annotations

import contextlib
import json
from dataclasses import dataclass, field
from pathlib import Path

import torch

from ..ops import _lib
from ..ops.conv import MODE_DW, STREAM_IDS, ConvGemmLayer, is_splitk, splitk_parts


@dataclass
class Step:
    kind: str                  # conv | stem | pool | head | gap | fc | ...
    name: str
    layer: object = None
    src: str = ""
    dst: str = ""
    res: str | None = None
    geom: tuple = ()           # (H, W, OH, OW) per image
    extra: dict = field(default_factory=dict)


class EngineBase:
    model_name = "model"

    def __init__(self, device, max_batch: int, buckets=None):
        self.device = torch.device(device)
        self.max_batch = max_batch
        self.buckets = sorted(set(buckets or [max_batch]))
        assert self.buckets[-1] <= max_batch
        self.steps: list[Step] = []
        self.programs: dict[tuple[int, bool, int], object] = {}
        self.stream = torch.cuda.Stream(device=self.device)
        self.inputs: list[torch.Tensor] = []   # input slots (self.inp is slot 0)
        self.outputs: list[torch.Tensor] = []  # per-slot logits (self.logits is slot 0)
        self._slot = 0
        self._remap: dict[str, str] = {}      # buffer-name overrides while emitting (stages.py)

    # ---------------------------------------------------------------- input slots
    def input_ptr(self) -> int:
        """Device pointer of the input slot the program being built reads."""
        return _lib.ptr(self.inputs[self._slot] if self.inputs else self.inp)

    def output_ptr(self) -> int:
        """Device pointer of the logits buffer the program being built writes."""
        return _lib.ptr(self.outputs[self._slot] if self.outputs else self.logits)

    def slot_logits(self, slot: int) -> torch.Tensor:
        return self.outputs[slot] if self.outputs else self.logits

    def add_input_slots(self, n: int) -> list[torch.Tensor]:
        """Extra static input AND logits buffers, each slot with its own captured
        graphs, so a pipelined caller can H2D batch i+1 into one slot while the graph
        of batch i reads another, and D2H batch i's logits while batch i+1's graph
        writes its own (no device-to-device copies on the compute stream)."""
        if not self.inputs:
            self.inputs = [self.inp]
            self.outputs = [self.logits]
        while len(self.inputs) < n:
            self.inputs.append(torch.zeros_like(self.inp))
            self.outputs.append(torch.zeros_like(self.logits))
        return self.inputs

    # ---------------------------------------------------------------- hooks
    def _emit(self, prog, step: Step, b: int) -> None:
        raise NotImplementedError

    def _emit_conv(self, prog, step: Step, b: int, split=None, cfg=None) -> None:
        """Emit (prog) or launch now (prog=None) one conv step with an explicit variant."""
        raise NotImplementedError

    # ---------------------------------------------------------------- programs
    def conv_steps(self) -> list[Step]:
        """Steps with a tunable GEMM layer (bf16 conv-GEMM or fp8 linear)."""
        return [s for s in self.steps if s.kind in ("conv", "f8")]

    def program(self, b: int, capture: bool = True, slot: int = 0):
        key = (b, capture, slot)
        if key in self.programs:
            return self.programs[key]
        assert 1 <= b <= self.max_batch
        prog = _lib.lib().Program()
        self._slot = slot
        try:
            self._emit_steps(prog, self.steps, [{}] * len(self.steps), b)
        finally:
            self._slot, self._remap = 0, {}
        if capture:
            with torch.cuda.device(self.device):
                prog.capture(int(self.stream.cuda_stream))
        self.programs[key] = prog
        return prog

    def _wptr(self, name: str) -> int:
        """Destination pointer of a step: a residual GEMM (res == dst) may write a different
        physical copy than it reads (stages.py versioning puts that under ``name@w``)."""
        return self._ptr(name + "@w") if (name + "@w") in self._remap else self._ptr(name)

    def alias_buffer(self, name: str, alias: str) -> None:
        """Another physical copy of an activation buffer (``stages.StagePipe`` gives each
        pipeline stage / batch parity its own copy of the buffers it shares)."""
        if alias not in self.bufs:
            self.bufs[alias] = torch.zeros_like(self.bufs[name])

    def program_range(self, b: int, lo: int, hi: int, capture: bool = True, slot: int = 0,
                      remap=None):
        """Program of steps[lo:hi] only, with buffer names remapped (``stages.py``):
        ``remap`` is one dict for all steps or a list with one dict per step."""
        n = hi - lo
        maps = list(remap) if isinstance(remap, (list, tuple)) else [dict(remap or {})] * n
        assert len(maps) == n
        key = (b, capture, slot, lo, hi, tuple(tuple(sorted(m.items())) for m in maps))
        if key in self.programs:
            return self.programs[key]
        prog = _lib.lib().Program()
        self._slot = slot
        try:
            self._emit_steps(prog, self.steps[lo:hi], maps, b)
        finally:
            self._slot, self._remap = 0, {}
        if capture:
            with torch.cuda.device(self.device):
                prog.capture(int(self.stream.cuda_stream))
        self.programs[key] = prog
        return prog

    def _emit_steps(self, prog, steps: list[Step], maps: list[dict], b: int) -> None:
        """Emit a run of steps, each with its buffer remap, on the engine's device (a vendor
        GEMM node builds its plan and workspace for the CURRENT device at emission time)."""
        ctx = torch.cuda.device(self.device) if self.device.type == "cuda" else contextlib.nullcontext()
        with ctx:
            for st, m in zip(steps, maps):
                self._remap = m
                self._emit(prog, st, b)

    def invalidate(self) -> None:
        self.programs.clear()

    def bucket_for(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        raise ValueError(f"batch {n} exceeds max bucket {self.buckets[-1]}")

    def launch(self, b: int, stream: torch.cuda.Stream | None = None, capture: bool = True,
               slot: int = 0) -> None:
        """Run the forward for the first ``b`` images already in input slot ``slot``."""
        s = stream or self.stream
        self.program(b, capture, slot).launch(int(s.cuda_stream))

    @torch.no_grad()
    def forward(self, x: torch.Tensor, capture: bool = True) -> torch.Tensor:
        """x: [n, H, W, 3] in the engine's input dtype, any device -> fp32 logits [n, classes]."""
        n = x.shape[0]
        assert tuple(x.shape[1:]) == tuple(self.inp.shape[1:]), (x.shape, self.inp.shape)
        assert x.dtype == self.inp.dtype, (x.dtype, self.inp.dtype)
        b = self.bucket_for(n)
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.inp[:n].copy_(x, non_blocking=True)
            self.launch(b, self.stream, capture)
            out = self.logits[:n].clone()
        cur.wait_stream(self.stream)
        return out

    # ---------------------------------------------------------------- observability / tuning
    def profile(self, b: int, iters: int = 20) -> list[tuple[str, float]]:
        prog = self.program(b, capture=False)
        ms = prog.profile(int(self.stream.cuda_stream), iters)
        return list(zip(prog.op_names(), ms))

    def _variants(self, step: Step) -> list[tuple[bool, int]]:
        v = step.layer.variants(step.geom[1])
        if step.res and not getattr(step.layer, "stream_ok", lambda res=False: True)(res=True):
            v = [x for x in v if x[1] not in STREAM_IDS]
        return v

    def autotune(self, b: int, iters: int = 10, verbose: bool = False) -> dict[str, list[int]]:
        """Pick the fastest (split, tile config) per conv layer by timing on the device."""
        s = self.stream
        chosen = {}
        with torch.cuda.stream(s):
            for step in self.conv_steps():
                lay: ConvGemmLayer = step.layer
                best = None
                for split, cfg in self._variants(step):
                    def run():
                        self._emit_conv(None, step, b, split=split, cfg=cfg)
                    for _ in range(2):
                        run()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(iters):
                        run()
                    e1.record(s)
                    e1.synchronize()
                    t = e0.elapsed_time(e1) / iters
                    if best is None or t < best[0]:
                        best = (t, split, cfg)
                    if verbose:
                        print(f"  {step.name:24s} split={int(split)} cfg {cfg}: {t * 1e3:8.1f} us", flush=True)
                lay.split, lay.cfg = best[1], best[2]
                chosen[step.name] = [int(best[1]), best[2]]
        self.invalidate()
        return chosen

    def tuning(self) -> dict[str, list[int]]:
        return {s.name: [int(s.layer.split), s.layer.cfg] for s in self.conv_steps()}

    def save_tuning(self, path) -> None:
        Path(path).write_text(json.dumps(self.tuning(), indent=1))

    def load_tuning(self, path) -> None:
        self.apply_tuning(json.loads(Path(path).read_text()))

    def apply_tuning(self, d: dict) -> None:
        for s in self.conv_steps():
            v = d.get(s.name)
            if v is None:
                continue
            split, cfg = (False, v) if isinstance(v, int) else (bool(v[0]), int(v[1]))
            ok = cfg in s.layer.candidates       # (ids 1000-1999, the retired hipBLASLt node, are refused)
            if cfg in STREAM_IDS:
                ok = getattr(s.layer, "stream_ok", lambda res=False: False)(res=bool(s.res))
            if is_splitk(cfg):
                sk, base = splitk_parts(cfg)
                ok = sk in getattr(s.layer, "ksplit", ()) and base in s.layer.candidates
            if ok and (not split or getattr(s.layer, "mode", -1) == MODE_DW):
                s.layer.split, s.layer.cfg = split, cfg
        self.invalidate()
