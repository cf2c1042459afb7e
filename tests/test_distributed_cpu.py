"""Data-parallel collectives over gloo with 2 CPU processes (fake multi-GPU
topology, SURVEY.md §4.2 'distributed (CPU)'): param broadcast, uint8 batch
scatter, logits gather, ragged global batches padded to per-rank buckets."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kdl.parallel.dp import DPRunner, broadcast_params, plan_shards


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    # C1: only rank 0 has the weights
    shapes = {"w": (4, 3), "b": (3,)}
    params = {"w": torch.arange(12.).view(4, 3), "b": torch.tensor([1., 2., 3.])} if rank == 0 else None
    p = broadcast_params(params, ["w", "b"], shapes, dev)
    assert torch.equal(p["w"], torch.arange(12.).view(4, 3)) and torch.equal(p["b"], torch.tensor([1., 2., 3.]))
    # toy "model": logits = per-image pixel mean * (rank+1) marker in column 1
    inp = torch.zeros((8, 5, 5, 3), dtype=torch.uint8)
    out = torch.zeros((8, 10))

    def forward(k):
        out[:k, 0] = inp[:k].float().mean(dim=(1, 2, 3))
        out[:k, 1] = rank
        return out

    runner = DPRunner(inp, forward, buckets=[1, 2, 4, 8], device=dev, classes=10)
    if rank == 0:
        results = []
        for n in (1, 3, 8, 13):
            batch = torch.stack([torch.full((5, 5, 3), i, dtype=torch.uint8) for i in range(n)])
            stopped, logits = runner.step(batch)
            assert not stopped
            results.append(logits.clone())
        runner.stop()
        q.put(("ok", [r.tolist() for r in results]))
    else:
        q.put(("served", runner.serve_forever()))
    dist.destroy_process_group()


def test_plan_shards():
    assert plan_shards(1, 2, [1, 2, 4]) == 1
    assert plan_shards(5, 2, [1, 2, 4]) == 4
    assert plan_shards(64, 8, [8, 16, 32]) == 8
    with pytest.raises(ValueError):
        plan_shards(100, 2, [1, 2, 4])


def test_dp_scatter_gather_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    msgs = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = dict(msgs)
    assert res["served"] == 4
    for n, logits in zip((1, 3, 8, 13), res["ok"]):
        assert len(logits) == n
        per = plan_shards(n, world, [1, 2, 4, 8])
        for i, row in enumerate(logits):
            assert row[0] == pytest.approx(i)            # image i routed back in order
            assert row[1] == (i // per)                  # computed by the rank owning its shard
