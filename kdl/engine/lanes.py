"""Split-batch lanes: one logical batch-B engine made of L batch-B/L engines whose
hipGraphs replay concurrently on L HIP streams.

Why: the Xception forward is a chain of ~40 launches, and the small late-flow
layers (19x19 maps, M = 32*361 rows) give each GEMM only ~250 workgroups, i.e.
about one per CU on a 256-CU chip, so every layer ends in a tail where most CUs
idle. Two or more independent half-batches on separate streams let one lane's
tail overlap another lane's body (measured: `profiles/lanes_probe.txt`, +3-4 %
on the graph alone). Each lane keeps the batch-B tile table (the tile choice is
made for the combined occupancy, not for one lane alone).

The group looks like an engine to `bench.py` and the serving executor: its
input slots and per-slot logits are single contiguous [B, ...] tensors (one H2D
or RCCL scatter per batch), and each lane's captured graph reads/writes its row
range of them as views, so there are no device-to-device copies. ``launch``
forks the caller's stream into the lanes with events and joins them back, so
events recorded on the caller's stream afterwards cover every lane.

The reference has no equivalent (TF-Serving runs one session per batch,
`tf-serving.dockerfile:2-5`); this is MI355X occupancy engineering.
"""
from __future__ import annotations

import os
import warnings

import torch


def hw_queues() -> int:
    """Hardware queues HIP gives this process (``GPU_MAX_HW_QUEUES``, HIP default 4)."""
    try:
        return max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))
    except ValueError:
        return 4


class LaneGroup:
    def __init__(self, info, params: dict, max_batch: int, device, lanes: int, make=None):
        """``make(b)``: optional engine factory (e.g. the serving executor's
        Xception with a custom head / f32 input); default ``info.engine``."""
        assert lanes >= 1 and max_batch % lanes == 0, (max_batch, lanes)
        if lanes > 2:
            # measured in the full bench pipeline (profiles/lanes4_vs2.txt): 4 lanes
            # run at 12.0k img/s vs 17.9k for 2 with GPU_MAX_HW_QUEUES=4, and at 7.7k
            # with 8 queues, so the loss is not queue sharing; cause not isolated yet.
            warnings.warn(f"{lanes} lanes measured much slower than 2 on MI355X "
                          f"(hardware queues: {hw_queues()})", stacklevel=2)
        self.device = torch.device(device)
        self.max_batch = max_batch
        self.lanes = lanes
        self.b = max_batch // lanes
        make = make or (lambda b: info.engine(params, b, self.device))
        self.engines = [make(self.b) for _ in range(lanes)]
        e0 = self.engines[0]
        self.stream = e0.stream
        self.classes = e0.logits.shape[1]
        self.inputs: list[torch.Tensor] = []
        self.outputs: list[torch.Tensor] = []
        self.add_input_slots(1)
        self.inp, self.logits = self.inputs[0], self.outputs[0]
        self._fork = [torch.cuda.Event() for _ in range(lanes)]
        self._join = [torch.cuda.Event() for _ in range(lanes)]

    # ---------------------------------------------------------------- tuning
    def load_tuning(self, path) -> None:
        for e in self.engines:
            e.load_tuning(path)

    def apply_tuning(self, d: dict) -> None:
        for e in self.engines:
            e.apply_tuning(d)

    def tuning(self) -> dict:
        return self.engines[0].tuning()

    def save_tuning(self, path) -> None:
        self.engines[0].save_tuning(path)

    def autotune(self, b: int | None = None, iters: int = 10, verbose: bool = False,
                 concurrent: bool = False) -> dict:
        """Per-layer tile choice. ``concurrent``: time each (split, cfg) variant with
        every lane running the layer at once on its own stream (the lanes start
        together and do identical work, so they stay roughly layer-aligned); the
        winner is the variant that fills the chip best next to its twin, not the
        fastest one alone. Off by default: on Xception b32 the concurrently tuned
        table measured 17.2k img/s against 17.9k for the single-lane b32 table
        (profiles/lanes_tuning_ab.txt) -- in the real graph the lanes drift out of
        layer alignment, so the solo-fastest tile is the better proxy."""
        if not concurrent or self.lanes == 1:
            t = self.engines[0].autotune(self.b, iters=iters, verbose=verbose)
            for e in self.engines[1:]:
                e.apply_tuning(t)
            return t
        s0 = self.engines[0].stream
        per_lane = [e.conv_steps() for e in self.engines]
        chosen = {}
        for idx, step in enumerate(per_lane[0]):
            best = None
            for split, cfg in self.engines[0]._variants(step):
                def run():
                    for e, steps in zip(self.engines, per_lane):
                        with torch.cuda.stream(e.stream):
                            e._emit_conv(None, steps[idx], self.b, split=split, cfg=cfg)
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for rep in range(2):                  # rep 0 warms up
                    t0.record(s0)
                    for k, e in enumerate(self.engines[1:], 1):
                        e.stream.wait_event(t0)
                    for _ in range(2 if rep == 0 else iters):
                        run()
                    for k, e in enumerate(self.engines[1:], 1):
                        self._join[k].record(e.stream)
                        s0.wait_event(self._join[k])
                    t1.record(s0)
                    t1.synchronize()
                t = t0.elapsed_time(t1) / iters
                if best is None or t < best[0]:
                    best = (t, split, cfg)
                if verbose:
                    print(f"  {step.name:24s} split={int(split)} cfg {cfg}: {t * 1e3:8.1f} us "
                          f"({self.lanes} lanes)", flush=True)
            chosen[step.name] = [int(best[1]), best[2]]
        self.apply_tuning(chosen)
        return chosen

    # ---------------------------------------------------------------- slots
    def add_input_slots(self, n: int) -> list[torch.Tensor]:
        """Contiguous [B, ...] input / logits buffers per slot; lane k's graphs use
        rows [k*b, (k+1)*b) of each (set before any program is built)."""
        e0 = self.engines[0]
        while len(self.inputs) < n:
            self.inputs.append(torch.zeros((self.max_batch,) + tuple(e0.inp.shape[1:]),
                                           dtype=e0.inp.dtype, device=self.device))
            self.outputs.append(torch.zeros((self.max_batch, self.classes),
                                            dtype=torch.float32, device=self.device))
        for k, e in enumerate(self.engines):
            r = slice(k * self.b, (k + 1) * self.b)
            e.inputs = [x[r] for x in self.inputs]
            e.outputs = [y[r] for y in self.outputs]
            e.invalidate()
        return self.inputs

    def slot_logits(self, slot: int) -> torch.Tensor:
        return self.outputs[slot]

    # ---------------------------------------------------------------- execution
    def program(self, b: int, capture: bool = True, slot: int = 0):
        assert b == self.max_batch, "lanes run full batches only"
        return [e.program(self.b, capture, slot) for e in self.engines]

    def launch(self, b: int, stream: torch.cuda.Stream | None = None, capture: bool = True,
               slot: int = 0) -> None:
        """Lane 0 replays on ``stream``; lanes 1.. fork from it and join back into it."""
        assert b == self.max_batch, "lanes run full batches only"
        s = stream or self.stream
        for k, e in enumerate(self.engines[1:], 1):
            self._fork[k].record(s)
            e.stream.wait_event(self._fork[k])
            e.launch(self.b, e.stream, capture, slot)
            self._join[k].record(e.stream)
        self.engines[0].launch(self.b, s, capture, slot)
        for k in range(1, self.lanes):
            s.wait_event(self._join[k])

    def launch_async(self, b: int, wait: list, done: list, capture: bool = True, slot: int = 0) -> None:
        """Free-running lanes: lane k's stream waits only on ``wait`` (e.g. this
        slot's ingress and egress events), replays its graph and records ``done[k]``.
        Unlike ``launch`` there is no fork from / join into one stream, so lane k of
        batch i+1 starts as soon as lane k of batch i is done instead of waiting for
        the slowest lane. Measured 1-3 % SLOWER than the joined lanes in bench.py
        (``--lanes-free``, profiles/ingress_hostsync_ab.txt): lanes that stay
        layer-aligned share the chip better than lanes that drift, so this is an
        option, not the default."""
        assert b == self.max_batch and len(done) == self.lanes, "lanes run full batches only"
        for e, d in zip(self.engines, done):
            for w in wait:
                e.stream.wait_event(w)
            e.launch(self.b, e.stream, capture, slot)
            d.record(e.stream)

    @torch.no_grad()
    def forward(self, x: torch.Tensor, capture: bool = True) -> torch.Tensor:
        n = x.shape[0]
        assert n == self.max_batch, (n, self.max_batch)
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.inp.copy_(x, non_blocking=True)
            self.launch(n, self.stream, capture)
            out = self.logits.clone()
        cur.wait_stream(self.stream)
        return out

    def profile(self, b: int, iters: int = 20):
        return self.engines[0].profile(self.b, iters)
