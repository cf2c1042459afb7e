#!/usr/bin/env python
"""Headline benchmark: Xception 299x299 serving throughput (images/s, whole node)
and p50 batch latency on 1..8 MI355X (BASELINE.json metric/config).

One process per GPU (``torch.distributed.run``), RCCL over xGMI. A timed step is
one dynamic batch of 32 images per GPU (weak scaling, global batch 32*N):

  1. ingress (default ``--ingress local``): every rank copies its own uint8 batch
     [32,299,299,3] host(pinned)->device on a copy stream, straight into one of its
     engine's input slots -- what the server's per-GPU executors do with their pinned
     staging (kdl/serving/backend.py). Each GPU has its own PCIe link;
  2. forward: hipGraph replays of the fused HIP-kernel model, stage-pipelined
     (kdl/engine/stages.py: stage 1 of batch i+1 runs beside stage 2 of batch i);
  3. gather: RCCL gather of the fp32 logits to rank 0 + D2H on a comm stream (one
     GPU: D2H behind the last stage), so compute stages / H2D / comm each own one
     of the 4 hardware queues.
Steps are software-pipelined: batch i+depth's H2D overlaps batch i's forward.

``--ingress scatter`` is the single-ingress variant: rank 0 H2Ds the
whole node's batch [32N,...] and RCCL-scatters uint8 shards (4x fewer bytes than f32)
over xGMI. Measured pinned H2D on one MI355X: 50 GB/s, so rank 0's 68.7 MB per step at
N=8 takes 1.37 ms against a 1.5 ms forward (profiles/h2d_bandwidth.txt): the rank-0
PCIe link, not xGMI, would bound the node, which is why it is not the default. Data
is synthetic (random uint8 images) and the weights are random-init of the exact
architecture (no network for checkpoints).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

BASELINE_IMG_S = None  # the reference publishes no throughput number


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle", type=float, default=0.5,
                    help="seconds of untimed graph replays before the warmup steps (GPU clock ramp)")
    ap.add_argument("--batch", type=int, default=32, help="images per GPU per step")
    ap.add_argument("--model", default="xception",
                    help="xception (headline) | resnet50 | vit_b16 | vit_b16_fp8 | efficientnet_b7")
    ap.add_argument("--ingress", choices=["scatter", "local", "none"], default="local",
                    help="local: each rank H2Ds its own batch; scatter: rank 0 H2Ds all and RCCL-scatters; none: DIAGNOSTIC ONLY (no host->device copy; the graphs re-read stale "
                         "slots) to measure what ingress overlap costs; never a reported number")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--depth", type=int, default=3,
                    help="ingress prefetch distance in batches (input slots = depth + 1)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="split each GPU's batch into this many concurrent hipGraph lanes "
                         "(kdl/engine/lanes.py; default 2 when the batch is even)")
    ap.add_argument("--stages", default=None, metavar="STEP",
                    help="stage-pipeline the forward (kdl/engine/stages.py): cut after this step; stage 1 "
                         "of batch i+1 overlaps stage 2 of batch i. Default: the model's cut (Xception: "
                         "block7_sepconv1, measured +10 %% over 2 lanes); 'none' = lanes")
    ap.add_argument("--cu-share", default=None, help="stage CU shares, e.g. 0.6,0.4 (CU-masked stage streams)")
    ap.add_argument("--lanes-free", action="store_true",
                    help="free-running lane streams (LaneGroup.launch_async) instead of forking/joining "
                         "the lanes through one stream every batch (measured 1-3 %% slower on one GPU)")
    ap.add_argument("--copy", choices=["raw", "torch"], default="raw",
                    help="ingress/egress copies: raw hipMemcpyAsync (kdl._C.memcpy_async) or torch copy_")
    ap.add_argument("--no-tune", action="store_true")
    ap.add_argument("--retune", action="store_true", help="autotune even if a tuning table exists")
    ap.add_argument("--tuning", default=None, help="tuning table to load instead of kdl/tuning/<model>_b<batch>.json")
    ap.add_argument("--profile-layers", action="store_true")
    ap.add_argument("--save-tuning", default=None, help="write the autotune result (rank 0) to this path")
    ap.add_argument("--dist-backend", default="nccl", help=argparse.SUPPRESS)   # gloo: pipeline logic checks
    ap.add_argument("--egress", choices=["gather", "local"], default="gather",
                    help="gather: RCCL-gather every step's logits to rank 0 (+ D2H there); local: each rank "
                         "D2Hs its own logits (what per-GPU serving executors do)")
    ap.add_argument("--force-dist", action="store_true",
                    help="take the multi-rank code path (process group, RCCL gather) even with one rank: "
                         "measures the collective overhead on a 1-GPU box")
    a = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_on = world > 1 or a.force_dist
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # --force-dist without a launcher: a world of one (torchrun sets all of these)
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.dist_backend)

    from kdl.engine import registry
    from kdl.ops import _lib
    C = _lib.lib()
    from kdl.engine.tuning import tuning_path

    B = a.batch
    info = registry.get(a.model)
    S = info.input_size
    params = info.init_params(0)
    if a.stages is None and a.lanes is None:
        a.stages = info.stage_cut or None    # Xception: stage pipelining (kdl/engine/stages.py)
    if a.stages == "none":
        a.stages = None
    if a.lanes is None:
        a.lanes = 2 if a.batch % 2 == 0 and not a.stages else 1
    if a.stages:
        from kdl.engine.stages import StagePipe
        assert a.lanes == 1, "--stages and --lanes > 1 are exclusive"
        eng = StagePipe(info.engine(params, B, dev), a.stages,
                        cu_share=[float(f) for f in a.cu_share.split(",")] if a.cu_share else None)
    elif a.lanes > 1:
        from kdl.engine.lanes import LaneGroup
        eng = LaneGroup(info, params, B, dev, a.lanes)
    else:
        eng = info.engine(params, B, dev)
    tname = info.tuning or a.model
    tp = Path(a.tuning) if a.tuning else tuning_path(tname, B, a.lanes)
    if not a.tuning and not tp.exists():
        tp = tuning_path(tname, B)          # no lanes-tuned table: the single-lane one
    if tp.exists() and not a.retune:
        eng.load_tuning(tp)
    elif not a.no_tune:
        eng.autotune(B)
    if a.save_tuning and rank == 0:
        eng.save_tuning(a.save_tuning)
    use_graph = not a.no_graph

    g = torch.Generator().manual_seed(1234 + rank)
    n_global = B * world
    # synthetic request batch in pinned host memory (every rank; only rank 0 for scatter).
    # Ingress is double-buffered: the H2D of batch i+1 runs on a copy stream while
    # batch i computes (what the serving executor does with its pinned staging).
    n_host = n_global if a.ingress == "scatter" else B
    has_host = a.ingress == "local" or (a.ingress == "scatter" and rank == 0)
    # one pinned host batch per slot (a server's requests land in distinct staging buffers;
    # re-issuing copies from ONE pinned buffer while its previous copy is still queued
    # blocked hipMemcpyAsync on the host for ~0.6 ms per step)
    NS = a.depth + 1
    hosts = ([torch.randint(0, 256, (n_host, S, S, 3), generator=g, dtype=torch.uint8).pin_memory()
              for _ in range(NS)] if has_host else None)
    # NS engine slots (input + logits buffer, each with its own captured graph): batch
    # i+depth lands in one slot (H2D, or RCCL scatter) and batch i-1's logits leave
    # another while batch i's graph runs; no device-to-device copies anywhere.
    slots = eng.add_input_slots(NS)
    direct = not dist_on or a.ingress != "scatter"    # H2D straight into the slot
    gather = dist_on and a.egress == "gather"
    stage = ([torch.empty((n_host, S, S, 3), dtype=torch.uint8, device=dev) for _ in range(NS)]
             if has_host and not direct else [None] * NS)
    NC = info.classes
    # gathered logits (rank 0, world > 1) and their pinned host copies, per slot
    logits_all = [torch.zeros((n_global, NC), dtype=torch.float32, device=dev) for _ in range(NS)]
    out_host = [torch.zeros((n_global, NC), dtype=torch.float32).pin_memory() for _ in range(NS)]
    s = eng.stream                          # compute: graph replays
    cs = torch.cuda.Stream(device=dev)      # ingress H2D
    ms = torch.cuda.Stream(device=dev) if gather or not direct else None   # RCCL scatter / gather + egress D2H
    # egress D2H (one GPU); stage-pipelined engines copy out on their last stage's stream
    # instead, so compute stages + H2D + egress stay within GPU_MAX_HW_QUEUES (4)
    ds = torch.cuda.Stream(device=dev) if not gather and not a.stages else None
    E = lambda: [torch.cuda.Event() for _ in range(NS)]  # noqa: E731
    ready, scattered, drained = E(), E(), E()
    # free[j]: slot j's input and logits are final -- one event per lane (free-running
    # lanes, LaneGroup.launch_async) or one for the single graph
    nl = a.lanes if a.lanes > 1 and a.lanes_free else 1
    free_running = nl > 1 or bool(a.stages)
    free = [[torch.cuda.Event() for _ in range(nl)] for _ in range(NS)]
    for e in drained + scattered + [f for fs in free for f in fs]:
        e.record(s)
    total = a.warmup + a.steps
    t_in = [torch.cuda.Event(enable_timing=True) for _ in range(total + 1)]
    t_out = [torch.cuda.Event(enable_timing=True) for _ in range(total + 1)]

    # Software pipeline, one batch per step: while the graph of batch i runs on the
    # compute stream, batch i+depth is H2D'd (copy stream) and RCCL-scattered (comm
    # stream) and batch i-1's logits are gathered (comm) and copied out (egress).
    def ingress(i, timed=False):
        j = i % NS
        t0 = time.perf_counter()
        # slot j (and stage j) must no longer be read by the graph / scatter of batch
        # i-NS. Waited for on the HOST, not with cs.wait_event: an H2D issued behind a
        # device-side wait on a graph-launch event held the issuing thread until that
        # graph finished (~0.6 ms per step, the GPU then ran dry between batches). With
        # depth >= 3 these events completed long ago, so the host waits nothing.
        for f in free[j]:
            f.synchronize()
        scattered[j].synchronize()
        with torch.cuda.stream(cs):
            if timed:
                t_in[i].record(cs)
            if has_host:
                dst, host = (slots[j][:B] if direct else stage[j]), hosts[j]
                if a.copy == "raw":
                    C.memcpy_async(dst.data_ptr(), host.data_ptr(), host.numel(), 1, cs.cuda_stream)
                else:
                    dst.copy_(host, non_blocking=True)
            tt[0] += time.perf_counter() - t0
            ready[j].record(cs)
        if not direct:
            with torch.cuda.stream(ms):
                ms.wait_event(ready[j])
                dist.scatter(slots[j][:B], list(stage[j].chunk(world)) if rank == 0 else None, src=0)
                scattered[j].record(ms)

    def compute(i):
        j = i % NS
        inp = ready[j] if direct else scattered[j]
        if free_running:                    # lanes / stages replay free-running on their own streams
            eng.launch_async(B, [inp, drained[j]], free[j], capture=use_graph, slot=j)
            return
        with torch.cuda.stream(s):
            s.wait_event(inp)
            s.wait_event(drained[j])        # slot j's logits left (gather + D2H of batch i-NS)
            eng.launch(B, s, capture=use_graph, slot=j)
            free[j][0].record(s)            # input and logits of slot j are final

    def collect(i, timed=False):
        j = i % NS
        out = eng.slot_logits(j)[:B]
        if gather:
            # gather + D2H on the comm stream: one fewer stream, so compute, lanes, H2D
            # and comm each keep a hardware queue of their own (GPU_MAX_HW_QUEUES=4)
            with torch.cuda.stream(ms):
                for f in free[j]:
                    ms.wait_event(f)
                dist.gather(out, list(logits_all[j].chunk(world)) if rank == 0 else None, dst=0)
                if rank == 0:
                    d2h(out_host[j], logits_all[j], ms)
                drained[j].record(ms)
                if timed:
                    t_out[i].record(ms)
            return
        es = eng.out_stream if a.stages else ds     # stages: D2H behind the last stage on its stream
        with torch.cuda.stream(es):
            if es is ds:
                for f in free[j]:
                    ds.wait_event(f)
            d2h(out_host[j], out, es)
            drained[j].record(es)
            if timed:
                t_out[i].record(es)

    def d2h(dst, src, stream):
        if a.copy == "raw":
            n = min(dst.numel(), src.numel()) * src.element_size()
            C.memcpy_async(dst.data_ptr(), src.data_ptr(), n, 2, stream.cuda_stream)
        else:
            dst[:src.shape[0]].copy_(src, non_blocking=True)

    tt = [0.0, 0.0, 0.0]   # host seconds in ingress / compute / collect issue

    def step(i):
        # compute first: hipMemcpyAsync of the pinned ingress blocks the host until the
        # copy stream's event waits resolve (the graph that last read the slot), which
        # measured ~0.75 ms/step of host time; issued after batch i's graphs, that wait
        # overlaps a queued graph instead of draining the GPU at every step
        t1 = time.perf_counter()
        compute(i)
        t2 = time.perf_counter()
        collect(i)
        tt[1] += t2 - t1
        tt[2] += time.perf_counter() - t2
        ingress(i + a.depth)  # prefetch `depth` batches ahead (K timed steps = K ingresses + K forwards)

    # setup (not a warmup step): capture both slots' graphs and let the clocks ramp
    for j in range(NS):
        eng.program(B, use_graph, j)
    t_settle = time.perf_counter() + a.settle
    while time.perf_counter() < t_settle:
        for _ in range(10):
            eng.launch(B, s, capture=use_graph)
        torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    for i in range(a.depth):
        ingress(i)
    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()

    tt[:] = [0.0, 0.0, 0.0]
    t0 = time.perf_counter()
    for i in range(a.warmup, total):
        step(i)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # unloaded per-batch latency (same path, one batch in flight at a time), outside the timed region
    lat = []
    for k in range(min(20, total)):
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        ingress(k, timed=True)
        compute(k)
        collect(k, timed=True)
        torch.cuda.synchronize()
        lat.append(t_in[k].elapsed_time(t_out[k]))
    if dist_on:
        t = torch.tensor(lat, device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lat = t.tolist()

    if rank == 0:
        ms_step = elapsed * 1e3 / a.steps
        img_s = n_global * a.steps / elapsed
        res = {
            "metric": ("images/sec (whole node) + p50 latency, Xception 299x299 at 1/2/4/8 MI355X"
                       if a.model == "xception" else
                       f"images/sec (whole node) + p50 latency, {a.model} {S}x{S}"),
            "value": round(img_s, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "p50_latency_ms": round(statistics.median(lat), 4),
            "p99_latency_ms": round(sorted(lat)[min(len(lat) - 1, int(0.99 * len(lat)))], 4),
            "settle_s": a.settle,
            "latency_note": "p50/p99: one batch in flight (H2D start -> logits on host), measured "
                            "after the timed loop; the timed loop overlaps batch i+1's H2D with batch i",
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (None if BASELINE_IMG_S is None or a.model != "xception"
                            else round(img_s / BASELINE_IMG_S, 3)),
            "dtype": info.dtype,
            "data": f"synthetic uint8 {S}x{S}x3 images, random-init weights",
            "config": {"model": info.description,
                       "global_batch": n_global, "seq_len": None, "image_size": S,
                       "per_gpu_batch": B, "parallelism": f"dp{world}",
                       "ingress": a.ingress, "egress": a.egress if dist_on else "local", "hipgraph": use_graph, "lanes": a.lanes,
                       **({"stages": f"{len(eng.ranges)} (cut after {a.stages})"} if a.stages else {})},
        }
        print(json.dumps(res), flush=True)
        print(f"host issue time {t_issue * 1e3 / a.steps:.3f} ms/step (ingress {tt[0] * 1e3 / a.steps:.3f}, "
              f"compute {tt[1] * 1e3 / a.steps:.3f}, collect {tt[2] * 1e3 / a.steps:.3f})", file=sys.stderr)
        if a.profile_layers:
            for name, t in eng.profile(B, 10):
                print(f"{name:28s} {t * 1e3:9.1f} us", file=sys.stderr)
    if dist_on:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
