"""Servables, signature runners and per-device executors.

Request path: gRPC/REST handler thread -> C++ DynamicBatcher
(``kdl._rt``; deadline-aware, bucketed) -> one executor per device which copies the
formed batch into pinned staging, H2D, replays the captured hipGraph of the bucket,
D2H of the logits -> ``finish`` wakes the handlers. On GPUs the executor loop is
native (``kdl._rt.Executor`` driving ``kdl._C.HipExecBackend`` from a C++ thread:
no Python and no GIL per batch, per-stage tracing in C++); ``KDL_NATIVE_EXEC=0``
selects the Python loop below instead.

Backends:
  * ``gpu``: the model family's MI355X engine (``kdl.engine.registry``: fused HIP
    kernels, hipGraph per bucket), one executor per MI355X (data parallel over
    the node's GPUs: each GPU pulls whole batches from the shared batcher,
    host-direct H2D over its own PCIe link).
  * ``cpu``: the family's fp32 torch oracle ("config #1: plumbing, no GPU").

Families: ``xception`` (the reference's clothing model; SavedModel ingest,
``serving_default`` = f32 ``input_8`` like TF-Serving, plus ``serving_uint8`` and
``serving_image`` = uint8 images of any size, resized on the GPU: resize.py),
and ``resnet50`` / ``vit_b16`` / ``efficientnet_b7`` (BASELINE.json configs;
torchvision-layout safetensors or synthetic weights, uint8 ``images`` input).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np
import torch

from ..models import xception as X
from ..ops import _lib
from . import protos as P
from .config import ServerConfig
from .metrics import BATCH_BUCKETS, METRICS
from .resize import IMAGE_SIGNATURE, ImageRunner

log = logging.getLogger("kdl.serving")

IMG = X.INPUT_SIZE
NATIVE_SIGNATURE = "serving_uint8"     # native fast path: uint8 HWC images (4x fewer bytes)
NATIVE_INPUT_KEY = "images"


class ServingError(Exception):
    """Carries a gRPC status code name + message (mapped to HTTP on REST)."""

    def __init__(self, code: str, msg: str):
        super().__init__(msg)
        self.code = code


@dataclass
class SignatureInfo:
    name: str
    input_key: str
    input_dtype: int
    output_key: str
    method_name: str = "tensorflow/serving/predict"
    input_shape: tuple = (-1, IMG, IMG, 3)
    output_shape: tuple = (-1, 10)


@dataclass
class ModelSource:
    """Where a version's weights come from."""
    params: dict
    head: X.Head | None
    signatures: dict[str, SignatureInfo] = field(default_factory=dict)
    origin: str = ""
    family: str = "xception"
    input_size: int = IMG
    classes: int = 10


def _family_source(family: str, params: dict | None, seed: int, origin: str) -> ModelSource:
    """Non-Xception families: uint8 NHWC images in, fp32 logits out."""
    from ..engine import registry
    info = registry.get(family)
    if params is None:
        params = info.init_params(seed)
    S, n = info.input_size, info.classes
    sigs = {name: SignatureInfo(name, NATIVE_INPUT_KEY, P.DT_UINT8, "logits", input_shape=(-1, S, S, 3),
                                output_shape=(-1, n)) for name in ("serving_default", NATIVE_SIGNATURE)}
    sigs[IMAGE_SIGNATURE] = SignatureInfo(IMAGE_SIGNATURE, NATIVE_INPUT_KEY, P.DT_UINT8, "logits",
                                          input_shape=(-1, -1, -1, 3), output_shape=(-1, n))
    return ModelSource(params=params, head=None, signatures=sigs, origin=origin, family=family,
                       input_size=S, classes=n)


def load_version_dir(path: Path, synthetic: bool = False) -> ModelSource:
    """SavedModel (saved_model.pb + variables/), packed kdl safetensors, or synthetic."""
    path = Path(path)
    sigs: dict[str, SignatureInfo] = {}
    if (path / "saved_model.pb").exists():
        from ..ingest.keras_map import to_xception_params
        from ..ingest.savedmodel import SavedModelDir
        sm = SavedModelDir(path)
        params, head = to_xception_params(sm.variables())
        for name, s in sm.signatures.items():
            if not s.inputs or not s.outputs:
                continue
            (ik, ispec), = list(s.inputs.items())[:1]
            (ok, ospec), = list(s.outputs.items())[:1]
            sigs[name] = SignatureInfo(name, ik, ispec.dtype, ok, s.method_name, ispec.shape, ospec.shape)
        origin = "saved_model"
    elif (path / "kdl_params.safetensors").exists():
        from safetensors.torch import load_file
        from ..ingest.fold import unpack
        params = unpack(load_file(str(path / "kdl_params.safetensors")))
        meta = json.loads((path / "kdl_model.json").read_text()) if (path / "kdl_model.json").exists() else {}
        if meta.get("family", "xception") != "xception":
            return _family_source(meta["family"], params, 0, "kdl_safetensors")
        head = X.Head(**meta.get("head", {}))
        for name, s in meta.get("signatures", {}).items():
            sigs[name] = SignatureInfo(name=name, input_key=s["input_key"], input_dtype=s.get("input_dtype", 1),
                                       output_key=s["output_key"])
        origin = "kdl_safetensors"
    elif synthetic or (path / "synthetic.json").exists():
        seed, family = 0, "xception"
        if (path / "synthetic.json").exists():
            meta = json.loads((path / "synthetic.json").read_text())
            seed, family = meta.get("seed", 0), meta.get("model", "xception")
        if family != "xception":
            return _family_source(family, None, seed, f"synthetic({family}, seed={seed})")
        params, head = X.init_params(seed=seed), X.DEFAULT_HEAD
        origin = f"synthetic(seed={seed})"
    else:
        raise FileNotFoundError(f"no servable artifact in {path}")
    if "serving_default" not in sigs:
        sigs["serving_default"] = SignatureInfo("serving_default", "input_8", P.DT_FLOAT, head.out)
    out_key = sigs["serving_default"].output_key
    sigs.setdefault(NATIVE_SIGNATURE, SignatureInfo(NATIVE_SIGNATURE, NATIVE_INPUT_KEY, P.DT_UINT8, out_key,
                                                    output_shape=(-1, head.classes)))
    # any-size uint8 images, resized on the GPU (serving/resize.py)
    sigs.setdefault(IMAGE_SIGNATURE, SignatureInfo(IMAGE_SIGNATURE, NATIVE_INPUT_KEY, P.DT_UINT8, out_key,
                                                   input_shape=(-1, -1, -1, 3), output_shape=(-1, head.classes)))
    return ModelSource(params=params, head=head, signatures=sigs, origin=origin, classes=head.classes)


# ---------------------------------------------------------------------- fault injection
class FaultInjector:
    """Test hook (SURVEY.md §5 "fault-injection hooks (env/flag) to fail a device or
    delay a batch"): ``KDL_FAULT_INJECT="fail=gpu1:-1,delay=cpu:50"`` makes every
    executor whose name contains ``gpu1`` raise on its batches (count -1 = forever,
    n = the next n batches) and delays batches of executors matching ``cpu`` by 50 ms."""

    def __init__(self, spec: str | None = None):
        if spec is None:
            spec = os.environ.get("KDL_FAULT_INJECT", "")
            # a --procs child restarted by the launcher (KDL_CHILD_RESTARTS > 0) models a fresh
            # process on a repaired device: the injected fault was transient unless made sticky
            if int(os.environ.get("KDL_CHILD_RESTARTS", "0")) > 0 and os.environ.get("KDL_FAULT_INJECT_STICKY") != "1":
                spec = ""
        self.fail: dict[str, int] = {}
        self.delay: dict[str, float] = {}
        self._lock = threading.Lock()
        for rule in filter(None, (r.strip() for r in spec.split(","))):
            kind, _, rest = rule.partition("=")
            pat, _, val = rest.partition(":")
            if kind == "fail":
                self.fail[pat] = int(val or -1)
            elif kind == "delay":
                self.delay[pat] = float(val or 0) / 1e3
            else:
                raise ValueError(f"bad KDL_FAULT_INJECT rule {rule!r}")

    def native_args(self, executor: str) -> tuple[int, int]:
        """(fail_batches, delay_us) for a native executor named ``executor``: the C++ loop
        applies them itself (kdl/csrc/runtime/executor.cpp)."""
        fail = next((n for pat, n in self.fail.items() if pat in executor), 0)
        delay = sum(sec for pat, sec in self.delay.items() if pat in executor)
        return fail, int(delay * 1e6)

    def before_batch(self, executor: str) -> None:
        for pat, sec in self.delay.items():
            if pat in executor:
                time.sleep(sec)
        with self._lock:
            for pat, left in self.fail.items():
                if pat in executor and left != 0:
                    if left > 0:
                        self.fail[pat] = left - 1
                    raise RuntimeError(f"injected fault on {executor}")


# ---------------------------------------------------------------------- executors
class _Executor(threading.Thread):
    """Pulls batches from a DynamicBatcher and runs them on one device.

    Per-device fault isolation: after ``max_failures`` consecutive failed batches
    the executor marks its device unhealthy and stops pulling, so the shared
    batcher routes everything to the remaining devices; the servable reports not
    ready once no healthy executor is left."""

    max_failures = 3

    def __init__(self, runner: "SignatureRunner", name: str):
        super().__init__(name=name, daemon=True)
        self.runner = runner
        self.stop = threading.Event()
        self.ready = threading.Event()
        self.error: BaseException | None = None
        self._healthy = True
        self.failures = 0
        self.faults = runner.faults
        bp = runner.cfg.batching
        self.eager = bool(runner.cfg.enable_batching and getattr(bp, "eager_when_idle", True))

    @property
    def healthy(self) -> bool:
        return self._healthy

    def run(self):
        try:
            self.setup()
        except BaseException as e:  # noqa: BLE001
            self.error = e
            log.exception("executor %s failed to start", self.name)
            self.ready.set()
            return
        if getattr(self, "native", None) is not None:
            self.run_native()
            return
        self.ready.set()
        METRICS.gauge("kdl_executor_healthy", lambda: float(self.healthy), executor=self.name)
        b = self.runner.batcher
        rt = _lib.rt()
        # pipelined executors (GPU, depth >= 2): batch n+1 is pulled into the next pinned
        # staging slot (host copy of the payloads) and its H2D + graph are issued while
        # batch n still runs on the device; batch n is finished (results scattered to
        # the waiting handlers) once its completion event has fired
        depth = max(1, getattr(self, "depth", 1))
        pending = []                           # (batch, handle, t0) in issue order
        slot = 0
        while not self.stop.is_set():
            poll = 0 if pending else 100_000   # with work in flight, never sleep in the batcher
            # device idle: dispatch what is queued now (work-conserving) instead of waiting
            # out the batch timeout; device busy: only full (or timed-out) batches
            batch = b.next_batch(self.staging_ptr(slot), poll, self.eager and not pending)
            if batch is not None:
                t0 = time.perf_counter()
                METRICS.observe("kdl_stage_ms", (rt.now_us() - batch.oldest_enqueue_us) / 1e3, stage="queue_wait")
                try:
                    if any(batch.dev_src):
                        raise RuntimeError("device-resident items need a native executor")
                    self.faults.before_batch(self.name)
                    handle = self.issue(batch.bucket, batch.n_real, slot)
                except BaseException:  # noqa: BLE001 - fail the batch, keep serving
                    if self._failed(b, batch):
                        return
                    continue
                pending.append((batch, handle, t0))
                slot = (slot + 1) % depth
            if pending and (batch is None or len(pending) >= depth):
                done, handle, t0 = pending.pop(0)
                try:
                    out_ptr = self.complete(handle)
                except BaseException:  # noqa: BLE001
                    if self._failed(b, done):
                        for rest, _, _ in pending:   # leaving: fail what is still in flight
                            b.finish(rest, 0, rt.ST_ERROR)
                        return
                    continue
                b.finish(done, out_ptr, rt.ST_OK)
                self.failures = 0
                self._observe(done, t0)
        for rest, _, _ in pending:
            b.finish(rest, 0, rt.ST_SHUTDOWN)

    def _failed(self, b, batch) -> bool:
        """Fail one batch; True when this executor gives up its device."""
        rt = _lib.rt()
        log.exception("batch %d failed on %s", batch.id, self.name)
        b.finish(batch, 0, rt.ST_ERROR)
        METRICS.inc("kdl_batch_errors_total", executor=self.name)
        self.failures += 1
        if self.failures < self.max_failures:
            return False
        self._healthy = False
        log.error("executor %s: %d consecutive failures, marking device unhealthy and leaving "
                  "the batcher to the other devices", self.name, self.failures)
        if not self.runner.healthy():
            # nobody is left to pull from the queue: fail what is queued (waiters with
            # no deadline would otherwise block forever) and refuse new submits
            log.error("no healthy executor left for %s: failing queued requests", self.runner.sig.name)
            b.shutdown()
        return True

    def _observe(self, batch, t0: float) -> None:
        dt = (time.perf_counter() - t0) * 1e3
        METRICS.observe("kdl_batch_exec_ms", dt, executor=self.name)
        METRICS.observe("kdl_batch_size", batch.n_real, buckets=BATCH_BUCKETS, signature=self.runner.sig.name)
        METRICS.inc("kdl_batches_total", signature=self.runner.sig.name)
        METRICS.inc("kdl_padded_items_total", batch.bucket - batch.n_real, signature=self.runner.sig.name)

    # synchronous executors implement execute(); pipelined ones override issue/complete
    def issue(self, bucket: int, n_real: int, slot: int):
        return self.execute(bucket, n_real)

    def complete(self, handle) -> int:
        return handle


class GPUExecutor(_Executor):
    def __init__(self, runner, device: int, engine_kwargs: dict, index: int = 0):
        super().__init__(runner, f"gpu{device}/{runner.sig.name}" + (f"#{index}" if index else ""))
        self.device = device
        self.engine_kwargs = engine_kwargs
        self.native = None
        self._busy = (0.0, time.perf_counter())

    @property
    def healthy(self) -> bool:
        return self.native.healthy() if self.native is not None else self._healthy

    def engine_buckets(self) -> list[int]:
        """Batch sizes the local engine captures graphs for (data parallel: per-rank shards)."""
        return self.runner.buckets

    def staging_rows(self) -> int:
        """Images per pinned staging slot (data parallel: the whole node's batch)."""
        return self.engine_buckets()[-1]

    def setup(self):
        from ..engine import registry
        from ..engine.tuning import tuning_path
        torch.cuda.set_device(self.device)
        r = self.runner
        src = r.source
        bs = self.engine_buckets()
        fam = registry.variant(src.family, r.cfg.dtype)      # --dtype picks the engine variant
        cap = bool(self.engine_kwargs.get("graph", True))      # --graph off: eager launches
        in_kind = "u8" if r.sig.input_dtype == P.DT_UINT8 else "f32"
        dev = f"cuda:{self.device}"
        def make(b, buckets=None):
            if fam == "xception":
                from ..engine.xception import XceptionEngine
                return XceptionEngine(src.params, max_batch=b, device=dev, in_kind=in_kind,
                                      head=src.head, buckets=buckets)
            return registry.get(fam).engine(src.params, b, dev, buckets=buckets)
        self.engine = make(bs[-1], bs)
        info = registry.get(fam)
        tp = tuning_path(info.tuning or fam, bs[-1])
        if tp.exists():
            self.engine.load_tuning(tp)
        # KDL_LANES=2: full batches of the top bucket run as concurrent split-batch
        # lanes (kdl/engine/lanes.py, same tile table); smaller buckets use the engine.
        # Off by default here: the closed-loop server is host-bound (one synchronous
        # batch per executor) and the extra graph launch + fork/join cost 4 % at
        # 16 clients x 8 images (profiles/serve_lanes_ab.txt), unlike bench.py.
        self.lanes = None
        nl = int(self.engine_kwargs.get("lanes") or os.environ.get("KDL_LANES", "1"))
        if nl > 1 and bs[-1] % nl == 0 and bs[-1] // nl >= 4:
            from ..engine.lanes import LaneGroup
            self.lanes = LaneGroup(None, None, bs[-1], dev, nl, make=make)
            if tp.exists():
                self.lanes.load_tuning(tp)
            self.lanes.program(bs[-1], capture=cap)
            self.lanes.launch(bs[-1], capture=cap)
        # stage pipelining of full top-bucket batches (kdl/engine/stages.py): stage 1 of
        # batch n+1 overlaps stage 2 of batch n. Default: the family's cut (Xception:
        # after block8_sepconv3) unless lanes were asked for; KDL_STAGES=none disables.
        self.pipe = None
        cut = self.engine_kwargs.get("stages") or os.environ.get("KDL_STAGES", "")
        if not cut:
            cut = info.stage_cut
        if cut and cut != "none" and self.lanes is None and hasattr(self.engine, "alias_buffer"):
            from ..engine.stages import StagePipe
            # its own engine ON PURPOSE: a top-bucket batch in the pipe and a small-bucket batch
            # in self.engine's graphs can be in flight together (depth >= 2, different streams),
            # so they must not share activation buffers; the duplicate costs ~50 MB of packed
            # weights + the activations of one batch, next to 288 GB of HBM
            self.pipe = StagePipe(make(bs[-1]), cut)
            if tp.exists():
                self.pipe.load_tuning(tp)
        # pipelining depth (batches in flight per GPU): staging / output slots, each with
        # its own captured graphs (engine input slots), so the host can form batch n+1
        # while batch n runs
        self.depth = max(1, int(self.engine_kwargs.get("depth") or os.environ.get("KDL_EXEC_DEPTH", "2")))
        self.capture = cap
        for e in (self.engine, self.lanes, self.pipe):
            if e is not None:
                e.add_input_slots(self.depth)
        dt = torch.uint8 if in_kind == "u8" else torch.float32
        S = src.input_size
        self.copy_stream = torch.cuda.Stream(device=self.device)
        # native executor (default): the C++ loop + HIP backend own the pinned staging; the
        # split-batch lanes variant exists only on the Python loop
        want_native = os.environ.get("KDL_NATIVE_EXEC", "1") != "0" and self.lanes is None
        if not want_native:
            self.staging = [torch.zeros((bs[-1], S, S, 3), dtype=dt).pin_memory() for _ in range(self.depth)]
            self.out = [torch.zeros((bs[-1], src.classes), dtype=torch.float32).pin_memory()
                        for _ in range(self.depth)]
        self.h2d_done = [torch.cuda.Event() for _ in range(self.depth)]
        self.done = [torch.cuda.Event() for _ in range(self.depth)]
        self._rt = _lib.lib()
        for slot in range(self.depth):        # warm-up + capture one hipGraph per (bucket, slot)
            for bk in bs:
                self.engine.program(bk, capture=cap, slot=slot)
                self.engine.launch(bk, capture=cap, slot=slot)
            for big in (self.lanes, self.pipe):
                if big is not None:
                    big.program(bs[-1], capture=cap, slot=slot)
                    big.launch(bs[-1], capture=cap, slot=slot)
        torch.cuda.synchronize(self.device)
        if want_native:
            self._build_native(S * S * 3 * (1 if in_kind == "u8" else 4), src.classes)

    def _build_native(self, item_bytes: int, classes: int) -> None:
        """Hand every bucket's captured graphs to the native executor: a kdl._C.HipExecBackend
        (pinned staging, H2D -> graphs -> D2H per slot, HIP-event stage times) driven by a
        kdl._rt.Executor C++ thread that pulls from the signature's batcher."""
        r, rt = self.runner, _lib.rt()
        bs = self.engine_buckets()
        be = self._rt.HipExecBackend(self.device, self.depth, item_bytes, self.staging_rows(), classes,
                                     copy_stream=self.copy_stream.cuda_stream, timing=True)
        keep = []
        for bk in bs:
            if self.pipe is not None and bk == self.pipe.max_batch:
                e = self.pipe
                progs = [[e._progs(bk, self.capture, slot, p) for p in (0, 1)] for slot in range(self.depth)]
                streams, wait_for = [s.cuda_stream for s in e.streams], [int(w) for w in e.wait_for]
            else:
                e = self.engine
                progs = [[[e.program(bk, self.capture, slot)]] * 2 for slot in range(self.depth)]
                streams, wait_for = [e.stream.cuda_stream], [0]
            keep.append(progs)                # the backend holds raw Program pointers
            be.add_recipe(bk, streams, wait_for, progs, [e.inputs[s].data_ptr() for s in range(self.depth)],
                          [e.slot_logits(s).data_ptr() for s in range(self.depth)])
        self._native_keep = keep
        self.backend = be
        if r.batcher is None:                 # a data-parallel follower: no batcher, no executor thread
            return
        fail, delay_us = self.faults.native_args(self.name)
        wrapped = self.wrap_backend(be)
        # the HIP backend copies device-resident rows itself (issue_dev); a DP leader does not
        self.takes_device_items = wrapped is be
        self.native = rt.Executor(r.batcher, wrapped, r.exec_group, name=self.name, eager=self.eager,
                                  max_failures=self.max_failures, fail_batches=fail, delay_us=delay_us)

    def wrap_backend(self, be):
        """The device backend handed to the native executor (data parallel: rank 0's DpLeader)."""
        return be

    def run_native(self) -> None:
        self.native.start()
        self.ready.set()
        METRICS.gauge("kdl_executor_healthy", lambda: float(self.healthy), executor=self.name)
        METRICS.gauge("kdl_gpu_busy_ratio", self._busy_ratio, executor=self.name)
        METRICS.collector(f"exec/{self.name}", self._native_metrics)
        self.stop.wait()
        self.native.stop()
        METRICS.drop_collector(f"exec/{self.name}")

    def _busy_ratio(self) -> float:
        """Device utilisation since the previous scrape: summed device forward time of the
        completed batches over wall time (stage-pipelined batches overlap, so it can exceed 1)."""
        s = self.native.stats()["stages"]["device_forward"]["sum_ms"] / 1e3
        now = time.perf_counter()
        s0, t0 = self._busy
        self._busy = (s, now)
        return (s - s0) / max(1e-6, now - t0)

    def _native_metrics(self) -> list[str]:
        st = self.native.stats()
        lbl = f'executor="{self.name}"'
        out = [f"kdl_exec_batches_total{{{lbl}}} {st['batches']}", f"kdl_exec_items_total{{{lbl}}} {st['items']}",
               f"kdl_exec_padded_items_total{{{lbl}}} {st['padded_items']}",
               f"kdl_exec_failed_batches_total{{{lbl}}} {st['failed_batches']}"]
        for stage, h in st["stages"].items():
            acc = 0
            for le, c in zip(st["le_ms"], h["buckets"]):
                acc += c
                out.append(f'kdl_exec_stage_ms_bucket{{{lbl},stage="{stage}",le="{"+Inf" if le > 1e29 else le}"}} {acc}')
            out.append(f'kdl_exec_stage_ms_sum{{{lbl},stage="{stage}"}} {h["sum_ms"]:g}')
            out.append(f'kdl_exec_stage_ms_count{{{lbl},stage="{stage}"}} {h["count"]}')
        return out

    def staging_ptr(self, slot: int = 0) -> int:
        return self.staging[slot].data_ptr()

    def issue(self, bucket: int, n_real: int, slot: int) -> int:
        """H2D on the copy stream (no device-side wait on a graph event: the slot's
        previous batch was completed on the host before the batcher refilled it),
        then the bucket's graph and the logits D2H on the engine stream."""
        big = self.lanes or self.pipe
        e = big if big is not None and bucket == big.max_batch else self.engine
        C = self._rt
        stg, inp = self.staging[slot], e.inputs[slot]
        nbytes = bucket * stg[0].numel() * stg.element_size()
        C.memcpy_async(inp.data_ptr(), stg.data_ptr(), nbytes, 1, self.copy_stream.cuda_stream)
        self.h2d_done[slot].record(self.copy_stream)
        if e is self.pipe:                    # free-running stages; logits final on stage 2's stream
            e.launch_async(bucket, [self.h2d_done[slot]], [self.done[slot]], capture=self.capture, slot=slot)
            out_stream = e.out_stream
        else:
            e.stream.wait_event(self.h2d_done[slot])
            e.launch(bucket, e.stream, capture=self.capture, slot=slot)
            out_stream = e.stream
        lg = e.slot_logits(slot)
        C.memcpy_async(self.out[slot].data_ptr(), lg.data_ptr(), bucket * lg.shape[1] * 4, 2, out_stream.cuda_stream)
        self.done[slot].record(out_stream)
        return slot

    def complete(self, slot: int) -> int:
        self.done[slot].synchronize()
        return self.out[slot].data_ptr()

    def execute(self, bucket: int, n_real: int) -> int:
        return self.complete(self.issue(bucket, n_real, 0))


class CPUExecutor(_Executor):
    def __init__(self, runner, index: int = 0):
        super().__init__(runner, f"cpu{index}/{runner.sig.name}")

    def setup(self):
        bs = self.runner.buckets[-1]
        src = self.runner.source
        u8 = self.runner.sig.input_dtype == P.DT_UINT8
        S = src.input_size
        self.staging = torch.zeros((bs, S, S, 3), dtype=torch.uint8 if u8 else torch.float32)
        self.out = torch.zeros((bs, src.classes), dtype=torch.float32)
        self.u8 = u8
        if src.family != "xception":
            from ..engine import registry
            self.oracle = registry.get(src.family).oracle

    def staging_ptr(self, slot: int = 0) -> int:
        return self.staging.data_ptr()

    def execute(self, bucket: int, n_real: int) -> int:
        x = self.staging[:n_real]
        src = self.runner.source
        if src.family != "xception":
            self.out[:n_real] = self.oracle(src.params, x)
            return self.out.data_ptr()
        x = x.float() / 127.5 - 1.0 if self.u8 else x
        self.out[:n_real] = X.xception_forward(src.params, x, head=src.head)
        return self.out.data_ptr()


class NullExecutor(_Executor):
    """``--device null``: the native C++ executor loop over kdl._rt.FakeBackend (no device
    time; result row = {first byte of the item + k}). Everything in front of the device --
    gRPC, the request codec, the batcher, the executor, the response path -- runs for real,
    so a closed-loop run against it measures the serving front-end's own ceiling
    (tools/serve_bench.py --device null)."""

    def __init__(self, runner, index: int = 0):
        # a --procs child names its GPU slot (gpu<i>:null<k>) so KDL_FAULT_INJECT can target one child
        gi = runner.cfg.gpu_index
        super().__init__(runner, (f"gpu{gi}:" if gi >= 0 else "") + f"null{index}/{runner.sig.name}")
        self.native = None

    @property
    def healthy(self) -> bool:
        return self.native.healthy() if self.native is not None else self._healthy

    def setup(self):
        r, rt = self.runner, _lib.rt()
        S = r.source.input_size
        item = S * S * 3 * (1 if r.sig.input_dtype == P.DT_UINT8 else 4)
        self.fake = rt.FakeBackend(nslots=2, item_bytes=item, max_batch=r.buckets[-1], out_cols=r.source.classes)
        fail, delay_us = self.faults.native_args(self.name)
        self.native = rt.Executor(r.batcher, self.fake, r.exec_group, name=self.name, eager=self.eager,
                                  max_failures=self.max_failures, fail_batches=fail, delay_us=delay_us)

    def run_native(self) -> None:
        self.native.start()
        self.ready.set()
        METRICS.gauge("kdl_executor_healthy", lambda: float(self.healthy), executor=self.name)
        self.stop.wait()
        self.native.stop()


class SignatureRunner:
    """One C++ batcher + the executors serving one signature of one version."""

    def __init__(self, sig: SignatureInfo, source: ModelSource, cfg: ServerConfig, devices: list[int]):
        self.sig, self.source, self.cfg = sig, source, cfg
        bp = cfg.batching
        self.buckets = cfg.rank_buckets()
        dp = cfg.scatter == "rccl" and cfg.dp_rank == 0 and sig.name == cfg.dp_signature
        if dp:                  # one collective step serves world x a per-GPU bucket (serving/dp.py)
            self.buckets = [b * cfg.dp_world for b in self.buckets]
        self.max_batch = self.buckets[-1]
        S = source.input_size
        item_bytes = self.item_bytes = S * S * 3 * (1 if sig.input_dtype == P.DT_UINT8 else 4)
        timeout = bp.batch_timeout_micros if cfg.enable_batching else 0
        self.batcher = _lib.rt().DynamicBatcher(max_batch_size=self.max_batch, batch_timeout_us=timeout,
                                                max_enqueued_batches=bp.max_enqueued_batches,
                                                allowed_batch_sizes=self.buckets, item_bytes=item_bytes,
                                                out_cols=source.classes,
                                                # threads for a batch's payload copy into pinned staging
                                                copy_threads=int(os.environ.get("KDL_COPY_THREADS", "4")))
        self.executors: list[_Executor] = []
        self.faults = FaultInjector()
        self.exec_group = _lib.rt().ExecGroup()     # native executors: last one out shuts the batcher
        if dp:
            from .dp import make_executor_class, make_native_executor_class, native_ok
            dev = torch.device("cuda", devices[0]) if devices else torch.device("cpu")
            cls = make_native_executor_class() if native_ok(cfg, dev) else make_executor_class()
            self.executors.append(cls(self, dev, cfg.dp_world))
        elif devices:
            for d in devices:
                for i in range(cfg.executors_for(len(devices))):
                    self.executors.append(GPUExecutor(self, d, cfg.engine_kwargs(), index=i))
        elif cfg.device == "null":
            for i in range(cfg.executors_for(1)):
                self.executors.append(NullExecutor(self, i))
        else:
            for i in range(cfg.executors_for(1)):
                self.executors.append(CPUExecutor(self, i))
        for ex in self.executors:
            ex.start()
        for ex in self.executors:
            ex.ready.wait()
            if ex.error is not None:
                raise ex.error
        METRICS.gauge("kdl_batch_queue_items", lambda: self.batcher.stats()["queue_items"], signature=sig.name)

    def predict(self, payload, n: int, deadline_us: int) -> np.ndarray:
        """payload: buffer of n items (uint8 or f32 images); returns f32 [n, classes]."""
        mv = memoryview(payload).cast("B")
        ib = self.item_bytes
        return self._run(n, lambda s, k: (self.batcher.submit(mv[s * ib:(s + k) * ib], k, deadline_us),
                                          mv[s * ib:(s + k) * ib]))

    def takes_device_items(self) -> bool:
        """Every executor is a native one whose backend copies device-resident rows itself
        (HipExecBackend::issue_dev): predict_device() may be used."""
        return bool(self.executors) and all(getattr(ex, "takes_device_items", False) for ex in self.executors)

    def predict_device(self, ptr: int, n: int, deadline_us: int) -> np.ndarray:
        """Like predict(), for n items already in device memory at address ``ptr``."""
        if not self.takes_device_items():
            raise ServingError("INTERNAL", f"signature {self.sig.name} has no executor for device-resident items")
        ib = self.item_bytes
        return self._run(n, lambda s, k: (self.batcher.submit_device(ptr + s * ib, k, deadline_us), None))

    def _run(self, n: int, submit) -> np.ndarray:
        rt = _lib.rt()
        if not self.healthy():
            raise ServingError("UNAVAILABLE", f"no healthy device left for signature {self.sig.name}")
        ncls = self.source.classes
        out = np.empty((n, ncls), dtype=np.float32)
        tickets = []
        for s in range(0, n, self.max_batch):
            k = min(self.max_batch, n - s)
            t, keep = submit(s, k)
            if t < 0:
                for ss, tt, _ in tickets:  # drain what was already queued, each into a buffer of its size
                    self.batcher.wait(tt, np.empty((min(self.max_batch, n - ss), ncls), np.float32))
                raise ServingError("RESOURCE_EXHAUSTED" if -t == rt.ST_QUEUE_FULL else "UNAVAILABLE",
                                   f"batcher rejected request (status {-t})")
            tickets.append((s, t, keep))
        status = rt.ST_OK
        for s, t, keep in tickets:
            buf = np.empty((min(self.max_batch, n - s), ncls), dtype=np.float32)
            st = self.batcher.wait(t, buf)
            del keep
            if st == rt.ST_OK:
                out[s:s + buf.shape[0]] = buf
            elif status == rt.ST_OK:
                status = st
        if status == rt.ST_DEADLINE:
            raise ServingError("DEADLINE_EXCEEDED", "deadline exceeded while queued for batching")
        if status != rt.ST_OK:
            raise ServingError("INTERNAL" if status == rt.ST_ERROR else "UNAVAILABLE", f"batch failed (status {status})")
        return out

    def healthy(self) -> bool:
        return any(ex.healthy and ex.error is None for ex in self.executors)

    def close(self):
        for ex in self.executors:
            ex.stop.set()
        self.batcher.shutdown()
        for ex in self.executors:
            ex.join(timeout=5)


class Servable:
    """One loaded model version (all its signatures)."""

    def __init__(self, name: str, version: int, source: ModelSource, cfg: ServerConfig, devices: list[int]):
        self.name, self.version, self.source = name, version, source
        self.signatures = source.signatures
        self.runners: dict[str, SignatureRunner] = {}
        self._devices, self._cfg = devices, cfg
        self._lock = threading.RLock()     # serving_image builds its serving_uint8 runner inside
        # serving_default is warmed eagerly (readiness = its graphs are captured), plus any
        # --warm_signatures (TF-Serving's warmup analogue: engines built before traffic arrives)
        self.runner("serving_default")
        warm = list(cfg.warm_signatures)
        # f32 requests of exact 8-bit pixels are served by the uint8 signature (grpc_server.py):
        # build it before traffic too, or the first such request waits for its graph captures
        if getattr(cfg, "f32_exact_u8", False) and NATIVE_SIGNATURE not in warm:
            warm.append(NATIVE_SIGNATURE)
        for name in warm:
            if name in self.signatures:
                self.runner(name)

    def runner(self, sig_name: str) -> SignatureRunner:
        with self._lock:
            r = self.runners.get(sig_name)
            if r is None:
                if sig_name not in self.signatures:
                    raise ServingError("INVALID_ARGUMENT", f"Serving signature name: \"{sig_name}\" not found "
                                       "in signature def")
                if sig_name == IMAGE_SIGNATURE and NATIVE_SIGNATURE in self.signatures:
                    r = ImageRunner(self.signatures[sig_name], self.runner(NATIVE_SIGNATURE), self._devices)
                else:
                    r = SignatureRunner(self.signatures[sig_name], self.source, self._cfg, self._devices)
                self.runners[sig_name] = r
            return r

    def healthy(self) -> bool:
        with self._lock:
            return all(r.healthy() for r in self.runners.values())

    def device_alive(self) -> bool:
        """False once every signature that has been given work has lost all its executors.
        Signatures nobody has called are no evidence either way (a dead device fails only the
        signatures that reach it), and one failing signature (e.g. a shape-specific kernel fault)
        beside a working one leaves the device alive."""
        with self._lock:
            runners = list(self.runners.values())
        used = [r for r in runners if r.batcher.stats()["submitted"] > 0]
        return not used or any(r.healthy() for r in used)

    def close(self):
        for r in self.runners.values():
            r.close()


def pick_devices(cfg: ServerConfig) -> list[int]:
    if cfg.device in ("cpu", "null"):
        return []
    if cfg.gpu_index >= 0 and (cfg.device == "gpu" or (torch.cuda.device_count() > 0 and _lib.available())):
        n = torch.cuda.device_count()     # one-process-per-GPU (--procs): this process's GPU only
        if n == 0:
            raise RuntimeError("--gpu_index given but no GPU is visible")
        return [cfg.gpu_index % n]
    if torch.cuda.is_available() and _lib.available():
        n = torch.cuda.device_count()
        k = n if cfg.gpus <= 0 else min(cfg.gpus, n)
        return list(range(k))
    if cfg.device == "gpu":
        raise RuntimeError("--device gpu requested but no GPU / kdl._C available")
    return []
