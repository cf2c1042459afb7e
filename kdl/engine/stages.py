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

Buffers are renamed per version (SSA over the step list): a version that crosses
a cut (the cut step's output; inside a middle-flow block also the block input that
comes back as the residual) is double-buffered by batch parity, and its writer
stage of batch i+2 waits for its last reader stage of batch i (a device-side
event wait); versions used inside one stage and the engine's scratch buffers get
stage-private copies, since the stages run concurrently (ResNet reuses its
per-stage pad / mid / ping-pong buffers across blocks).

Interface: like an engine for ``bench.py`` / the serving executor (input slots,
per-slot logits, ``launch`` joins into the caller's stream) plus
``launch_async`` (free-running: the caller waits on ``done`` events instead).
The reference has no equivalent (TF-Serving runs one session per batch).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch


def _cu_mask(k: int, shares: list, n_cu: int = 256) -> list[int]:
    """32-bit mask words giving stage k its share of the CUs, interleaved over the CU
    index (i mod 20 buckets) so every stage gets CUs on every XCD whatever the bit order."""
    bounds, acc = [], 0.0
    for f in shares:
        acc += f
        bounds.append(round(acc * 20))
    lo = 0 if k == 0 else bounds[k - 1]
    hi = bounds[k]
    words = [0] * ((n_cu + 31) // 32)
    for i in range(n_cu):
        if lo <= i % 20 < hi:
            words[i // 32] |= 1 << (i % 32)
    return words


def cu_masked_stream(device, words: list[int]) -> torch.cuda.ExternalStream:
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                  ctypes.POINTER(ctypes.c_uint32)]
    arr = (ctypes.c_uint32 * len(words))(*words)
    ptr = ctypes.c_void_p()
    with torch.cuda.device(device):
        err = hip.hipExtStreamCreateWithCUMask(ctypes.byref(ptr), len(words), arr)
    if err != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({err})")
    return torch.cuda.ExternalStream(ptr.value, device=device)


@dataclass
class StagePlan:
    ranges: list            # [(lo, hi)] step ranges, one per stage
    remaps: list            # [parity][step] -> {name: physical name} (name@w: write pointer)
    boundary: list          # buffers with a version that crosses a cut
    wait_for: list          # per stage: the last later stage it must wait for (parity reuse)
    aliases: dict           # physical copy -> base buffer to allocate it like


def plan_stages(steps, split_after, scratch=()) -> StagePlan:
    """Pure analysis (no GPU): stage ranges and per-step buffer renaming for a cut list.

    A read of X at step i sees the last write of X before i (SSA over the sequential
    step list). A version read only inside its writer's stage a lives in a stage-private
    copy (X in stage 0 or when no other stage touches X, X#s<a> otherwise: stages run
    concurrently); a version read by a later stage is double-buffered by batch parity
    (X#x<a>p0 / X#x<a>p1), and stage a then waits for its last reader stage two
    batches back before overwriting it. ``scratch`` buffers get a copy per stage."""
    cuts = split_after.split(",") if isinstance(split_after, str) else list(split_after)
    names = [s.name for s in steps]
    for c in cuts:
        if c not in names:
            raise ValueError(f"no step {c!r}; steps: {names}")
    bounds = [0] + sorted(names.index(c) + 1 for c in cuts) + [len(names)]
    ranges = [(lo, hi) for lo, hi in zip(bounds, bounds[1:]) if hi > lo]
    K = len(ranges)
    stage = [k for k, (lo, hi) in enumerate(ranges) for _ in range(lo, hi)]
    last_write: dict = {}
    reads = []                               # per step: {name: writer step or -1}
    readers: dict = {}                       # writer step -> max reader stage
    for i, st in enumerate(steps):
        r = {}
        for nm in (st.src, st.res):
            if nm and nm not in ("input", "logits"):
                w = last_write.get(nm, -1)
                r[nm] = w
                if w >= 0:
                    readers[w] = max(readers.get(w, stage[w]), stage[i])
        reads.append(r)
        # a true in-place step (src == dst, one pointer: e.g. EfficientNet's channel scale)
        # modifies the version it read instead of creating a new one
        if st.dst and st.dst not in ("input", "logits") and st.src != st.dst:
            last_write[st.dst] = i
    touched: dict = {}                       # stages that read or write each name
    for i, st in enumerate(steps):
        for nm in (st.src, st.res, st.dst):
            if nm:
                touched.setdefault(nm, set()).add(stage[i])

    def phys(nm: str, w: int, p: int) -> str:
        a = stage[w]
        if readers.get(w, a) > a:
            return f"{nm}#x{a}p{p}"
        return nm if a == 0 or len(touched[nm]) == 1 else f"{nm}#s{a}"

    remaps, aliases, boundary = [[], []], {}, set()
    wait_for = list(range(K))
    for i, st in enumerate(steps):
        for p in (0, 1):
            m = {nm: phys(nm, w, p) for nm, w in reads[i].items() if w >= 0}
            if st.dst and st.dst not in ("input", "logits") and st.src != st.dst:
                ph = phys(st.dst, i, p)
                # a residual GEMM with res == dst reads and writes through separate
                # pointers, so the version it reads and the one it writes may differ
                if st.res == st.dst:
                    m[st.dst + "@w"] = ph      # write pointer, see EngineBase._wptr
                else:
                    m[st.dst] = ph
            for k_name in scratch:
                if stage[i]:
                    m[k_name] = f"{k_name}#s{stage[i]}"
            for key, ph in m.items():
                base = key[:-2] if key.endswith("@w") else key
                if ph != base:
                    aliases[ph] = base
            remaps[p].append(m)
        if st.dst and readers.get(i, stage[i]) > stage[i]:
            boundary.add(st.dst)
            wait_for[stage[i]] = max(wait_for[stage[i]], readers[i])
    return StagePlan(ranges, remaps, sorted(boundary), wait_for, aliases)


class StagePipe:
    pipelined = True          # consecutive batches overlap (graph_tune times it free-running)

    def __init__(self, engine, split_after, cu_share: list | None = None, priorities: list | None = None):
        """``split_after``: one step name (two stages) or a comma-separated list / list of
        names (one stage per segment, one HIP stream each). ``cu_share``: optional
        fraction of the CUs per stage (CU-masked streams, hipExtStreamCreateWithCUMask),
        so the stages run on disjoint CU sets; measured 20-65 % SLOWER than letting both
        stages share every CU (profiles/stages_ab.txt), kept for experiments only.
        ``priorities``: optional HIP stream priority per stage (lower = higher; env
        ``KDL_STAGE_PRIO``, e.g. "0,-1"), so the hardware dispatcher places one stage's
        workgroups first when both stages wait for free CUs."""
        self.engine = engine
        self.device = engine.device
        self.max_batch = engine.max_batch
        plan = plan_stages(engine.steps, split_after, getattr(engine, "scratch_buffers", lambda: [])())
        for alias, base in plan.aliases.items():
            engine.alias_buffer(base, alias)
        self.ranges, self.remaps = plan.ranges, plan.remaps
        self.boundary, self.wait_for = plan.boundary, plan.wait_for
        self.cut = self.ranges[0][1]
        K = len(self.ranges)
        self.cu_share = cu_share
        if cu_share:
            self.streams = [cu_masked_stream(self.device, _cu_mask(k, cu_share)) for k in range(K)]
            engine.stream = self.streams[0]
        else:
            if priorities is None and os.environ.get("KDL_STAGE_PRIO"):
                priorities = [int(v) for v in os.environ["KDL_STAGE_PRIO"].split(",")]
            if priorities:
                assert len(priorities) == K, (priorities, K)
                self.streams = [torch.cuda.Stream(device=self.device, priority=p) for p in priorities]
                engine.stream = self.streams[0]
            else:
                self.streams = [engine.stream] + [torch.cuda.Stream(device=self.device) for _ in range(K - 1)]
        self.priorities = priorities
        self.stream = self.streams[0]
        self.done = [[torch.cuda.Event() for _ in range(K)] for _ in range(2)]   # [parity][stage]
        self._fork = torch.cuda.Event()
        for e in self.done[0] + self.done[1]:     # "done" before the first batch
            e.record(self.streams[0])
        self._n = 0                               # batches issued (parity of the next one)
        self.trace: list | None = None            # [(batch, stage, start event, end event)] when a list
        engine.add_input_slots(1)
        self.inputs, self.outputs = engine.inputs, engine.outputs
        self.inp, self.logits = engine.inputs[0], engine.outputs[0]
        self.classes = self.logits.shape[1]

    @property
    def out_stream(self) -> torch.cuda.Stream:
        """Stream on which the logits become final (the last stage's)."""
        return self.streams[-1]

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
        e = self.engine
        return [e.program_range(b, lo, hi, capture, slot, self.remaps[parity][lo:hi])
                for lo, hi in self.ranges]

    def program(self, b: int, capture: bool = True, slot: int = 0):
        return [self._progs(b, capture, slot, p) for p in (0, 1)]

    def launch_async(self, b: int, wait: list, done: list, capture: bool = True, slot: int = 0) -> None:
        """Stage 0 waits on ``wait`` (input ready, logits drained); stage k waits on stage
        k-1 of this batch and on the last later-stage reader of its double-buffered
        outputs two batches back; ``done[0]`` fires when the logits of ``slot`` are final."""
        assert b == self.max_batch
        p = self._n & 1
        self._n += 1
        progs = self._progs(b, capture, slot, p)
        ev = self.done[p]
        for k, (prog, st) in enumerate(zip(progs, self.streams)):
            if k == 0:
                for w in wait:
                    st.wait_event(w)
            else:
                st.wait_event(ev[k - 1])
            if self.wait_for[k] > k:
                st.wait_event(ev[self.wait_for[k]])   # recorded by batch i-2: its reader is done
            if self.trace is not None:            # diagnostic timeline (bench.py --timeline)
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record(st)
            prog.launch(int(st.cuda_stream))
            if self.trace is not None:
                t1.record(st)
                self.trace.append((self._n - 1, k, t0, t1))
            ev[k].record(st)
        done[0].record(self.streams[-1])

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
