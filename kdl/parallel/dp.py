"""Data-parallel serving over one node: one process per GPU, RCCL over xGMI.

SURVEY.md §2.7/§2.8: the model (21 M params, 42 MB bf16) is replicated on every
GPU; requests are batch-sharded. Collectives (``torch.distributed`` backend
"nccl" == RCCL on ROCm; "gloo" for CPU tests):

  C1 ``broadcast_params``  rank 0 (which read the SavedModel) -> all ranks, once.
  C2 ``scatter_batch``     ingress rank 0 -> every rank: its shard of the uint8
                           image batch (268 KB/img, 4x fewer bytes than f32),
                           written straight into the rank's static engine input.
  C3 ``gather_logits``     every rank -> rank 0: fp32 logits [shard, 10].
  ctrl ``broadcast_ctrl``  rank 0 -> all: (n_real, per-rank bucket, stop flag).

xGMI is point-to-point (7 links/GPU): a scatter from the root uses all 7 links
in parallel, unlike a ring all-reduce; only tiny messages go the other way.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable

import torch
import torch.distributed as dist


@dataclass
class Ctrl:
    n_real: int       # real images in the global batch
    per_rank: int     # images per rank (padded shard size = graph bucket)
    stop: bool = False


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def rank_world() -> tuple[int, int]:
    if not is_dist():
        return 0, 1
    return dist.get_rank(), dist.get_world_size()


def broadcast_params(params: dict[str, torch.Tensor] | None, keys: list[str], shapes: dict[str, tuple],
                     device: torch.device, src: int = 0) -> dict[str, torch.Tensor]:
    """C1: every rank returns the same parameter dict (flattened into one
    buffer -> one collective instead of 238)."""
    total = sum(math.prod(shapes[k]) for k in keys)
    buf = torch.empty(total, dtype=torch.float32, device=device)
    rank, _ = rank_world()
    if rank == src:
        off = 0
        for k in keys:
            n = math.prod(shapes[k])
            buf[off:off + n].copy_(params[k].reshape(-1))
            off += n
    if is_dist():
        dist.broadcast(buf, src=src)
    out, off = {}, 0
    for k in keys:
        n = math.prod(shapes[k])
        out[k] = buf[off:off + n].view(shapes[k]).cpu()
        off += n
    return out


def broadcast_ctrl(ctrl: Ctrl | None, device: torch.device, src: int = 0) -> Ctrl:
    t = torch.zeros(3, dtype=torch.int64, device=device)
    if rank_world()[0] == src:
        t[0], t[1], t[2] = ctrl.n_real, ctrl.per_rank, int(ctrl.stop)
    if is_dist():
        dist.broadcast(t, src=src)
    v = t.tolist()
    return Ctrl(n_real=v[0], per_rank=v[1], stop=bool(v[2]))


def plan_shards(n_real: int, world: int, buckets: list[int]) -> int:
    """Per-rank shard size: ceil(n/world) rounded up to a captured bucket."""
    need = max(1, -(-n_real // world))
    for b in sorted(buckets):
        if b >= need:
            return b
    raise ValueError(f"shard of {need} images exceeds the largest bucket {max(buckets)}")


def scatter_batch(global_batch: torch.Tensor | None, local_out: torch.Tensor, src: int = 0) -> None:
    """C2: rank `src` holds [world*per_rank, ...]; every rank receives its
    [per_rank, ...] slice into `local_out` (a view of its engine input)."""
    rank, world = rank_world()
    if world == 1:
        local_out.copy_(global_batch[:local_out.shape[0]])
        return
    chunks = list(global_batch.chunk(world)) if rank == src else None
    dist.scatter(local_out, chunks, src=src)


def gather_logits(local: torch.Tensor, global_out: torch.Tensor | None, dst: int = 0) -> None:
    """C3: rank `dst` receives [world*per_rank, classes]."""
    rank, world = rank_world()
    if world == 1:
        global_out.copy_(local)
        return
    chunks = list(global_out.chunk(world)) if rank == dst else None
    dist.gather(local, chunks, dst=dst)


class DPRunner:
    """Collective step shared by the bench and the distributed server.

    ``forward(per_rank) -> logits view`` runs the local model on the first
    `per_rank` images already in ``local_input``."""

    def __init__(self, local_input: torch.Tensor, forward: Callable[[int], torch.Tensor], buckets: list[int],
                 device: torch.device, classes: int = 10):
        self.rank, self.world = rank_world()
        self.local_input = local_input
        self.forward = forward
        self.buckets = sorted(buckets)
        self.device = device
        self.classes = classes
        maxb = self.buckets[-1]
        if self.rank == 0:
            self.global_in = torch.empty((self.world * maxb,) + tuple(local_input.shape[1:]),
                                         dtype=local_input.dtype, device=device)
            self.global_out = torch.empty((self.world * maxb, classes), dtype=torch.float32, device=device)

    def step(self, host_batch: torch.Tensor | None = None,
             n_real: int | None = None) -> tuple[bool, torch.Tensor | None]:
        """Rank 0 passes the host batch; other ranks pass nothing. Returns
        (stopped, gathered logits [n_real, classes] on rank 0 / None elsewhere)."""
        if self.rank == 0:
            n = host_batch.shape[0] if n_real is None else n_real
            ctrl = Ctrl(n_real=n, per_rank=plan_shards(n, self.world, self.buckets))
        else:
            ctrl = None
        ctrl = broadcast_ctrl(ctrl, self.device)
        if ctrl.stop:
            return True, None
        k = ctrl.per_rank
        gin = None
        if self.rank == 0:
            gin = self.global_in[:self.world * k]
            gin[:ctrl.n_real].copy_(host_batch[:ctrl.n_real], non_blocking=True)
        scatter_batch(gin, self.local_input[:k])
        logits = self.forward(k)[:k]
        gout = self.global_out[:self.world * k] if self.rank == 0 else None
        gather_logits(logits.contiguous(), gout)
        return False, (gout[:ctrl.n_real] if self.rank == 0 else None)

    def stop(self) -> None:
        if self.rank == 0:
            broadcast_ctrl(Ctrl(0, 0, True), self.device)

    def serve_forever(self) -> int:
        """Non-zero ranks: follow rank 0's steps until it broadcasts stop.
        Returns the number of steps served."""
        n = 0
        while True:
            stopped, _ = self.step()
            if stopped:
                return n
            n += 1
