"""``--scatter rccl``: one front-end, data parallel over the node's GPUs on RCCL.

The north star's serving topology: ONE server process
(rank 0) owns the gRPC/REST front-end and the dynamic batcher; it forms batches of up
to ``world x per-rank bucket`` images and runs them as one collective step with every
other rank (one process per GPU):

    C1  share_source       rank 0 read the model version from disk -> every rank, once per
                           version (torch.distributed broadcast of the flattened weights)
    C2  scatter            rank 0's uint8 batch (268 KB/img; one pinned staging slot) -> each
                           follower's shard, straight into its engine's static input slot
    C3  gather             every follower's fp32 logits -> rank 0 -> D2H -> handlers

GPU (default): the NATIVE path (kdl/csrc/runtime/comm.cpp). Rank 0's C++ executor thread drives
a ``DpLeader`` -- rank 0's own HipExecBackend (its shard goes H2D straight into its engine and
its stage-pipelined graphs start at once) plus ncclSend / ncclRecv of a control word, the
shards and the logits on two RCCL communicators -- with ``--exec_depth`` steps in flight.
Followers run ``DpFollower.run()``: a C++ loop, GIL released, keyed by the received control
word (per-rank bucket -> which captured graph), no Python per step. CPU / gloo: the
torch.distributed reference implementation of the same protocol (``kdl.parallel.dp``).

Hot reload: when rank 0's model manager loads a new version, the new DP executor asks the
current leader to send DP_RELOAD(version); followers leave their loop, receive the new weights
(C1), rebuild, and join the new communicators. The DP signature is unavailable while the
followers rebuild (rank 0's other signatures keep serving); the old version's executor fails
its remaining batches (UNAVAILABLE to clients) until it is retired.

The reference scales by Deployment replicas behind a Service
(`tf-serving-clothing-model-deployment.yaml:8`); ``--procs N`` (one independent server per
GPU on a shared port) is the other topology here.
"""
from __future__ import annotations

import logging

import torch
import torch.distributed as dist

from ..models import xception as X
from ..parallel import dp as D
from . import protos as P

log = logging.getLogger("kdl.serving")


def init_group(cfg, rank: int, world: int) -> torch.device:
    """Join the node's process group; returns this rank's device. Collectives time out after
    KDL_DP_TIMEOUT_S (default 120 s): a rank that died fails rank 0's batches (the executor
    then marks itself unhealthy) instead of hanging the front-end."""
    from datetime import timedelta
    import os
    timeout = timedelta(seconds=float(os.environ.get("KDL_DP_TIMEOUT_S", "120")))
    use_gpu = cfg.device != "cpu" and torch.cuda.device_count() > 0
    if use_gpu:
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if native_ok(cfg, dev):
            # every per-batch byte moves on the native RCCL communicators (comm.cpp); the process
            # group only carries control (comm ids, model metadata) and the one-time weight
            # broadcast, on the CPU: a torch RCCL communicator beside the native ones would be a
            # third per rank (a second one cost the bench 17 %, profiles/dist_path_r5.txt)
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timeout)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, timeout=timeout)
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timeout)
    return dev


# ---------------------------------------------------------------------- C1: the model
def share_source(source, dev: torch.device):
    """Rank 0 passes its ModelSource, the others None; every rank returns an equivalent one
    (metadata by object broadcast, the weights as one flattened collective)."""
    from .backend import ModelSource
    rank, _ = D.rank_world()
    meta = [None]
    if rank == 0:
        keys = sorted(k for k, v in source.params.items() if torch.is_floating_point(v))
        meta[0] = dict(keys=keys, shapes={k: tuple(source.params[k].shape) for k in keys},
                       dtypes={k: str(source.params[k].dtype) for k in keys}, head=source.head,
                       signatures=source.signatures, origin=source.origin, family=source.family,
                       input_size=source.input_size, classes=source.classes)
    dist.broadcast_object_list(meta, src=0)
    m = meta[0]
    params = {k: v.float() for k, v in source.params.items()} if rank == 0 else None
    bdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    flat = D.broadcast_params(params, m["keys"], m["shapes"], bdev)
    flat = {k: v.to(getattr(torch, m["dtypes"][k].split(".")[-1])) for k, v in flat.items()}
    if rank == 0:
        return source
    return ModelSource(params=flat, head=m["head"], signatures=m["signatures"], origin=m["origin"] + " (C1 broadcast)",
                       family=m["family"], input_size=m["input_size"], classes=m["classes"])


# ---------------------------------------------------------------------- local forward
def local_forward(source, sig, dev: torch.device, buckets: list[int]):
    """(static input of the largest per-rank bucket, forward(k) -> logits [>=k, classes])."""
    u8 = sig.input_dtype == P.DT_UINT8
    S, maxb = source.input_size, buckets[-1]
    if dev.type == "cpu":
        inp = torch.zeros((maxb, S, S, 3), dtype=torch.uint8 if u8 else torch.float32)
        if source.family != "xception":
            from ..engine import registry
            oracle = registry.get(source.family).oracle

            def fwd(k):
                return oracle(source.params, inp[:k]).float()
            return inp, fwd

        def fwd(k):
            x = inp[:k].float() / 127.5 - 1.0 if u8 else inp[:k]
            return X.xception_forward(source.params, x, head=source.head)
        return inp, fwd
    from ..engine import registry
    from ..engine.tuning import tuning_path
    fam = source.family
    if fam == "xception":
        from ..engine.xception import XceptionEngine
        eng = XceptionEngine(source.params, max_batch=maxb, device=dev, in_kind="u8" if u8 else "f32",
                             head=source.head, buckets=buckets)
    else:
        eng = registry.get(fam).engine(source.params, maxb, dev, buckets=buckets)
    info = registry.get(fam)
    tp = tuning_path(info.tuning or fam, maxb)
    if tp.exists():
        eng.load_tuning(tp)
    for b in buckets:                       # capture every bucket's graph before serving
        eng.launch(b, eng.stream, capture=True)
    torch.cuda.synchronize(dev)

    def fwd(k):
        cur = torch.cuda.current_stream(dev)
        eng.stream.wait_stream(cur)          # the scatter wrote the input on the current stream
        eng.launch(eng.bucket_for(k), eng.stream, capture=True)
        cur.wait_stream(eng.stream)          # the gather reads the logits on it
        return eng.logits
    return eng.inp, fwd


# ---------------------------------------------------------------------- followers
def native_ok(cfg, dev: torch.device) -> bool:
    """The C++/RCCL path (comm.cpp) runs on GPUs unless KDL_DP_NATIVE=0."""
    import os
    return dev.type == "cuda" and os.environ.get("KDL_DP_NATIVE", "1") != "0"


class _FollowerRunner:
    """What a GPUExecutor reads from its SignatureRunner, for a follower (no batcher)."""

    def __init__(self, source, sig, cfg):
        from .backend import FaultInjector
        self.source, self.sig, self.cfg = source, sig, cfg
        self.buckets = cfg.rank_buckets()
        self.batcher = None
        self.exec_group = None
        self.faults = FaultInjector("")


def _comms(rank: int, world: int, device: int):
    """Two RCCL communicators (scatter, gather) on fresh unique ids from rank 0."""
    from ..ops import _lib
    C = _lib.lib()
    ids = [C.rccl_unique_id(), C.rccl_unique_id()] if rank == 0 else [None, None]
    dist.broadcast_object_list(ids, src=0)
    return [C.RcclComm(i, world, rank, device) for i in ids]


def liveness_s() -> float:
    """A follower that hears no control word (batch, command or heartbeat) from rank 0 for this
    long treats it as dead and exits non-zero (KDL_DP_LIVENESS_S, default 30 s)."""
    import os
    return float(os.environ.get("KDL_DP_LIVENESS_S", "30"))


def ping_s() -> float:
    """Rank 0's heartbeat period while idle (KDL_DP_PING_S, default a sixth of the liveness)."""
    import os
    return float(os.environ.get("KDL_DP_PING_S", str(liveness_s() / 6)))


def follow_native(cfg, rank: int, world: int, dev: torch.device) -> int:
    """A follower's life: per model version, receive the weights (C1), build the engine and
    its graphs, join the version's communicators, then serve rank 0's steps in C++ until a
    DP_STOP (exit) or DP_RELOAD (next version) control word. Every wait is bounded
    (kdl/csrc/runtime/dp_core.h): a silent leader ends this rank with a non-zero status."""
    from ..ops import _lib
    from .backend import GPUExecutor
    C = _lib.lib()
    while True:
        source = share_source(None, dev)
        sig = source.signatures[cfg.dp_signature]
        ex = GPUExecutor(_FollowerRunner(source, sig, cfg), dev.index, cfg.engine_kwargs())
        ex.setup()                      # engines, captured graphs, HipExecBackend recipes
        comms = _comms(rank, world, dev.index)
        f = C.DpFollower(ex.backend, *comms)
        log.info("dp rank %d/%d on %s ready (native RCCL, %s, per-rank buckets %s)", rank, world, dev,
                 cfg.dp_signature, cfg.rank_buckets())
        try:
            cmd, version, seq = f.run(liveness_s())
        except RuntimeError as e:       # rank 0 silent past the liveness window, or RCCL failed
            log.error("dp rank %d: %s -- exiting so the supervisor restarts the group", rank, e)
            return 3
        log.info("dp rank %d: %s after %d steps", rank, "reload" if cmd == C.DP_RELOAD else "stop", f.steps)
        del f, comms, ex
        torch.cuda.synchronize(dev)
        if cmd != C.DP_RELOAD:
            return 0


def follow(cfg, rank: int, world: int) -> int:
    """Ranks >= 1: receive the model (C1), build the DP signature's engine on this rank's
    GPU, then run rank 0's collective steps until it broadcasts stop. SIGTERM / SIGINT are
    ignored: the launcher stops rank 0, whose stop broadcast ends this loop; a dead rank 0 ends
    it through the liveness window (native path), a dead follower fails rank 0's next step within
    KDL_DP_TIMEOUT_S."""
    import signal
    for sg in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sg, signal.SIG_IGN)
    dev = init_group(cfg, rank, world)
    if native_ok(cfg, dev):
        rc = follow_native(cfg, rank, world, dev)
        if rc == 0:                     # a dead rank 0 would leave the group's teardown hanging
            dist.destroy_process_group()
        return rc
    source = share_source(None, dev)
    sig = source.signatures[cfg.dp_signature]
    buckets = cfg.rank_buckets()
    inp, fwd = local_forward(source, sig, dev, buckets)
    runner = D.DPRunner(inp, fwd, buckets, dev, source.classes)
    dist.barrier()
    log.info("dp rank %d/%d on %s ready (%s, per-rank buckets %s)", rank, world, dev, cfg.dp_signature, buckets)
    n = runner.serve_forever()
    log.info("dp rank %d: stop after %d steps", rank, n)
    dist.destroy_process_group()
    return 0


# ---------------------------------------------------------------------- rank 0 executor
_ACTIVE = {"leader": None, "lock": None}


def _active_lock():
    import threading
    if _ACTIVE["lock"] is None:
        _ACTIVE["lock"] = threading.Lock()
    return _ACTIVE["lock"]


def make_native_executor_class():
    from ..ops import _lib
    from .backend import GPUExecutor

    class DPNativeExecutor(GPUExecutor):
        """Rank 0's executor of the data-parallel signature on the native path: the C++
        executor thread issues each batch of world x shard images to a DpLeader (comm.cpp)."""

        def __init__(self, runner, dev: torch.device, world: int, version: int | None = None):
            super().__init__(runner, dev.index, runner.cfg.engine_kwargs())
            self.name = f"dp{world}/{runner.sig.name}"
            self.world, self.version = world, version
            self.leader = None

        def engine_buckets(self) -> list[int]:
            return self.runner.cfg.rank_buckets()

        def staging_rows(self) -> int:
            return self.world * self.engine_buckets()[-1]

        def setup(self):
            import os
            C = _lib.lib()
            with _active_lock():
                old = _ACTIVE["leader"]
                if old is not None:          # a newer version: followers leave the old loop first
                    _ACTIVE["leader"] = None
                    if old.send_ctrl(C.DP_RELOAD, int(self.version or 0)) != 0:
                        # a follower is gone (or the old leader already failed): the group cannot
                        # take the new version; fail the load loudly instead of hanging in C1
                        raise RuntimeError("dp: followers did not take DP_RELOAD; the data-parallel group "
                                           "is broken (its ranks exit on their liveness window)")
                # C1 for this version (the initial one was shared by server.main before loading)
                if old is not None:
                    share_source(self.runner.source, self.device_obj())
                super().setup()              # engines, graphs, HipExecBackend; -> wrap_backend
                self.timeout_s = float(os.environ.get("KDL_DP_TIMEOUT_S", "120"))
                _ACTIVE["leader"] = self.leader

        def device_obj(self) -> torch.device:
            return torch.device("cuda", self.device)

        def wrap_backend(self, be):
            import os
            self.comms = _comms(0, self.world, self.device)
            self.leader = _lib.lib().DpLeader(be, *self.comms, self.engine_buckets(),
                                              float(os.environ.get("KDL_DP_TIMEOUT_S", "120")), ping_s())
            return self.leader

        def run_native(self) -> None:
            try:
                super().run_native()
            finally:
                with _active_lock():
                    if _ACTIVE["leader"] is self.leader and self.leader is not None:
                        if self.leader.send_ctrl(_lib.lib().DP_STOP, 0) != 0:    # release the followers
                            log.warning("dp: DP_STOP not delivered; followers exit on their liveness window")
                        _ACTIVE["leader"] = None
    return DPNativeExecutor


def make_executor_class():
    from .backend import _Executor

    class DPExecutor(_Executor):
        """Rank 0's executor of the data-parallel signature: each batch from the batcher is
        ONE collective step (C2 scatter -> every rank's engine -> C3 gather)."""

        def __init__(self, runner, dev: torch.device, world: int):
            super().__init__(runner, f"dp{world}/{runner.sig.name}")
            self.dev, self.world = dev, world

        def setup(self):
            if self.dev.type == "cuda":
                torch.cuda.set_device(self.dev)   # the current device is per thread
            r = self.runner
            src = r.source
            u8 = r.sig.input_dtype == P.DT_UINT8
            S = src.input_size
            self.buckets = r.cfg.rank_buckets()         # the batcher's are world x these
            inp, fwd = local_forward(src, r.sig, self.dev, self.buckets)
            self.dpr = D.DPRunner(inp, fwd, self.buckets, self.dev, src.classes)
            pin = self.dev.type == "cuda"
            st = torch.zeros((r.buckets[-1], S, S, 3), dtype=torch.uint8 if u8 else torch.float32)
            out = torch.zeros((r.buckets[-1], src.classes), dtype=torch.float32)
            self.staging = st.pin_memory() if pin else st
            self.out = out.pin_memory() if pin else out
            dist.barrier()                    # every follower has its engine

        def staging_ptr(self, slot: int = 0) -> int:
            return self.staging.data_ptr()

        def execute(self, bucket: int, n_real: int) -> int:
            _, logits = self.dpr.step(self.staging[:n_real], n_real)
            self.out[:n_real].copy_(logits)   # D2H of the gathered logits (synchronous)
            return self.out.data_ptr()

        def run(self):
            try:
                super().run()
            finally:
                if getattr(self, "dpr", None) is not None:
                    self.dpr.stop()           # release the followers' serve_forever
    return DPExecutor

