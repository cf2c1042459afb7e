"""Stage pipelining inside one GPU: the forward is cut into two stages that run
on two HIP streams, so stage 1 (stem + entry flow) of batch i+1 replays while
stage 2 (middle + exit flow + head) of batch i does.

Why (measured, profiles/stages_ab.txt): the two halves of Xception stress the
chip differently. The entry flow (147x147 / 74x74 maps) is bound by activation
traffic and launches persistent, chip-filling kernels; the middle flow (19x19x728,
M = 361 rows per image) is bound by per-workgroup latency with about one 512-
thread workgroup per CU. Two half-batch lanes of the SAME layers (``lanes.py``)
compete for the same resource at the same time; two stages of DIFFERENT layers
can fill each other's gaps. Each stage runs the full batch, so every kernel keeps
the b32 tile table.

Every buffer written by stage 1 and read by stage 2 (the cut step's output, and
inside a middle-flow block also the block input that comes back as the residual)
is double-buffered by batch parity: stage 1 of batch i+2 may overwrite copy
i % 2 only after stage 2 of batch i has read it (a device-side event wait on the
stage-1 stream). Scratch buffers are per stage.

Interface: like an engine for ``bench.py`` / the serving executor (input slots,
per-slot logits, ``launch`` joins into the caller's stream) plus
``launch_async`` (free-running: the caller waits on ``done`` events instead).
The reference has no equivalent (TF-Serving runs one session per batch).
"""
from __future__ import annotations

import torch


class StagePipe:
    pipelined = True          # consecutive batches overlap (graph_tune times it free-running)

    def __init__(self, engine, split_after: str):
        self.engine = engine
        self.device = engine.device
        self.max_batch = engine.max_batch
        names = [s.name for s in engine.steps]
        if split_after not in names:
            raise ValueError(f"no step {split_after!r}; steps: {names}")
        self.cut = names.index(split_after) + 1
        st1, st2 = engine.steps[:self.cut], engine.steps[self.cut:]
        # double-buffer (by batch parity) EVERY buffer stage 1 writes and stage 2 reads:
        # the cut step's output and, inside a middle-flow block, the block input that the
        # block's last separable conv adds back as its residual
        written = {s.dst for s in st1}
        read2 = {b for s in st2 for b in (s.src, s.res) if b}
        self.boundary = sorted(written & read2 - {"input", "logits"})
        for b in self.boundary:
            engine.alias_buffer(b, b + "#1")
        # stage-private scratch: the split (dw kernel + GEMM) separable convs of both stages
        # would otherwise share one depthwise scratch buffer while running concurrently
        engine.alias_buffer("__dwtmp", "__dwtmp#2")
        self.remaps = [({}, {"__dwtmp": "__dwtmp#2"}),
                       ({b: b + "#1" for b in self.boundary},
                        {**{b: b + "#1" for b in self.boundary}, "__dwtmp": "__dwtmp#2"})]
        self.streams = [engine.stream, torch.cuda.Stream(device=self.device)]
        self.stream = self.streams[0]
        self.s1_done = [torch.cuda.Event() for _ in range(2)]
        self.s2_done = [torch.cuda.Event() for _ in range(2)]
        self._fork = torch.cuda.Event()
        for e in self.s1_done + self.s2_done:     # "done" before the first batch
            e.record(self.streams[0])
        self._n = 0                               # batches issued (parity of the next one)
        self.inputs = engine.inputs
        self.outputs = engine.outputs
        engine.add_input_slots(1)
        self.inp, self.logits = engine.inputs[0], engine.outputs[0]
        self.classes = self.logits.shape[1]

    # ---------------------------------------------------------------- tuning (engine's table)
    def load_tuning(self, path) -> None:
        self.engine.load_tuning(path)

    def apply_tuning(self, d: dict) -> None:
        self.engine.apply_tuning(d)

    def tuning(self) -> dict:
        return self.engine.tuning()

    def save_tuning(self, path) -> None:
        self.engine.save_tuning(path)

    def autotune(self, b: int | None = None, iters: int = 10, verbose: bool = False) -> dict:
        return self.engine.autotune(b or self.max_batch, iters=iters, verbose=verbose)

    def conv_steps(self):
        return self.engine.conv_steps()

    def _variants(self, step):
        return self.engine._variants(step)

    # ---------------------------------------------------------------- slots
    def add_input_slots(self, n: int) -> list[torch.Tensor]:
        r = self.engine.add_input_slots(n)
        self.inputs, self.outputs = self.engine.inputs, self.engine.outputs
        return r

    def slot_logits(self, slot: int) -> torch.Tensor:
        return self.engine.slot_logits(slot)

    def invalidate(self) -> None:
        self.engine.invalidate()

    # ---------------------------------------------------------------- execution
    def _progs(self, b: int, capture: bool, slot: int, parity: int):
        e, (rm1, rm2) = self.engine, self.remaps[parity]
        return (e.program_range(b, 0, self.cut, capture, slot, rm1),
                e.program_range(b, self.cut, len(e.steps), capture, slot, rm2))

    def program(self, b: int, capture: bool = True, slot: int = 0):
        return [self._progs(b, capture, slot, p) for p in (0, 1)]

    def launch_async(self, b: int, wait: list, done: list, capture: bool = True, slot: int = 0) -> None:
        """Stage 1 waits on ``wait`` (input ready, logits drained) and on stage 2 of the
        batch two back (boundary reuse); stage 2 waits on stage 1; ``done[0]`` fires when
        the logits of slot ``slot`` are final."""
        assert b == self.max_batch
        p = self._n & 1
        self._n += 1
        p1, p2 = self._progs(b, capture, slot, p)
        s1, s2 = self.streams
        for w in wait:
            s1.wait_event(w)
        s1.wait_event(self.s2_done[p])
        p1.launch(int(s1.cuda_stream))
        self.s1_done[p].record(s1)
        s2.wait_event(self.s1_done[p])
        p2.launch(int(s2.cuda_stream))
        self.s2_done[p].record(s2)
        done[0].record(s2)

    def launch(self, b: int, stream: torch.cuda.Stream | None = None, capture: bool = True,
               slot: int = 0) -> None:
        """Joined form: forks from / joins into ``stream`` (no cross-batch overlap)."""
        s = stream or self.stream
        self._fork.record(s)
        d = torch.cuda.Event()
        self.launch_async(b, [self._fork], [d], capture, slot)
        s.wait_event(d)

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
        return self.engine.profile(b, iters)
