"""``--scatter rccl``: one front-end, data parallel over the node's GPUs on RCCL.

The north star's serving topology: ONE server process
(rank 0) owns the gRPC/REST front-end and the dynamic batcher; it forms batches of up
to ``world x per-rank bucket`` images and runs them as one collective step with every
other rank (one process per GPU, ``torch.distributed`` backend "nccl" = RCCL over
xGMI; "gloo" on CPU):

    C1  broadcast_params   rank 0 read the model version from disk -> every rank, once
    ctrl broadcast_ctrl    (n_real, per-rank shard, stop)
    C2  scatter_batch      rank 0's uint8 / f32 batch (one H2D on GPU 0) -> each rank's
                           shard, written straight into its engine's static input
    C3  gather_logits      every rank's fp32 logits -> rank 0 -> D2H -> handlers

(``kdl.parallel.dp``). The reference scales by Deployment replicas behind a Service
(`tf-serving-clothing-model-deployment.yaml:8`); ``--procs N`` (one independent server
per GPU on a shared port) is the other topology here and the default of the k8s
manifest: rank 0's single Python front-end tops out near 29k img/s
(``profiles/serve_closed_loop_r3.jsonl``, null device), below one node's GPUs, while
``--procs`` has no such ceiling. This mode is the collective path for deployments that
want one endpoint, one batcher and one model load.

One signature (``--dp_signature``, default ``serving_default``) runs data parallel; the
others are served by rank 0's own GPU. Version hot-reload is off in this mode (the
followers build their engines once).
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
    flat = D.broadcast_params(params, m["keys"], m["shapes"], dev)
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
def follow(cfg, rank: int, world: int) -> int:
    """Ranks >= 1: receive the model (C1), build the DP signature's engine on this rank's
    GPU, then run rank 0's collective steps until it broadcasts stop. SIGTERM / SIGINT are
    ignored: the launcher stops rank 0, whose stop broadcast ends this loop (a follower that
    died first would leave rank 0's collectives hanging)."""
    import signal
    for sg in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sg, signal.SIG_IGN)
    dev = init_group(cfg, rank, world)
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

