#!/usr/bin/env python
"""Headline benchmark: Xception 299x299 serving throughput (images/s, whole node)
and p50 batch latency on 1..8 MI355X (BASELINE.json metric/config).

One process per GPU, RCCL over xGMI. Two equivalent entry styles:

  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
  python bench.py --gpus N        # no launcher: bench.py spawns the N rank processes itself

(the self-launch parent never touches a GPU; it refuses N > visible GPUs unless
``--allow-shared``, which marks the JSON ``gpus_shared``). A timed step is one dynamic batch
of 32 images per GPU (weak scaling, global batch 32*N):

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
import socket
import statistics
import subprocess
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

BASELINE_IMG_S = None  # the reference publishes no throughput number


def _visible_gpus() -> int:
    """GPUs this process may use, counted WITHOUT touching HIP in this process: the visibility
    env vars if set, else ``torch.cuda.device_count()`` in a throwaway child (the launcher
    parent must stay GPU-free: it only spawns the ranks)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() != ""])
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def _free_port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(a, argv: list[str]) -> int:
    """``python bench.py --gpus N`` with no launcher: spawn the N ranks ourselves (one child
    process per GPU, the env torch.distributed.run would set, rendezvous on 127.0.0.1) and exit
    with the first failing child's status. Nothing here touches a GPU and nothing re-execs."""
    n = a.gpus
    if not a.dry_run:
        vis = _visible_gpus()
        if n > vis and not a.allow_shared:
            print(f"bench.py: --gpus {n} but only {vis} GPU(s) visible; refusing to pack ranks onto "
                  f"shared GPUs (pass --allow-shared to measure that anyway)", file=sys.stderr)
            return 2
    port = _free_port()
    kids = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        kids.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        live = list(kids)
        while live:
            for k in list(live):
                c = k.poll()
                if c is None:
                    continue
                live.remove(k)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    for o in live:                 # one rank died: the others would hang in a collective
                        o.terminate()
            time.sleep(0.05)
    finally:
        for k in kids:
            if k.poll() is None:
                k.kill()
                k.wait()
    return rc


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks) of this node to use. Without a launcher (no WORLD_SIZE in the env) "
                         "bench.py spawns the N ranks itself; under torch.distributed.run it must match "
                         "--nproc-per-node. Default: the launcher's world size, else 1")
    ap.add_argument("--allow-shared", action="store_true",
                    help="permit more ranks than visible GPUs (ranks share GPUs; the JSON says gpus_shared)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the launcher / rank wiring: gloo group, no GPU, one JSON line")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle", type=float, default=0.5,
                    help="minimum seconds of untimed pipelined steps before the warmup steps (GPU clock ramp)")
    ap.add_argument("--settle-max", type=float, default=3.0,
                    help="untimed steps continue past --settle until two consecutive 10-step chunks "
                         "agree within 1 %% (a stable replay time), for at most this many seconds")
    ap.add_argument("--batch", type=int, default=32, help="images per GPU per step")
    ap.add_argument("--model", default="xception",
                    help="xception (headline) | resnet50 | vit_b16 | vit_b16_fp8 | efficientnet_b7")
    ap.add_argument("--ingress", choices=["scatter", "local", "none"], default="local",
                    help="local: each rank H2Ds its own batch; scatter: rank 0 H2Ds all and RCCL-scatters; none: DIAGNOSTIC ONLY (no host->device copy; the graphs re-read stale "
                         "slots) to measure what ingress overlap costs; never a reported number")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--depth", type=int, default=3,
                    help="ingress prefetch distance in batches (input slots = depth + 1 + slack)")
    ap.add_argument("--settle-mode", choices=["pipe", "serial"], default="pipe",
                    help="DIAGNOSTIC: what the settle phase runs -- the pipelined step (default) or joined graph "
                         "replays (the pre-round-6 settle)")
    ap.add_argument("--touch", choices=["auto", "on", "off"], default="auto",
                    help="one joined replay before the inputs are primed, so the pipeline-stage streams submit before "
                         "the copy stream (hardware-queue mapping order); auto = on for 3+ stages")
    ap.add_argument("--timeline", action="store_true",
                    help="DIAGNOSTIC: timing events around every pipeline stage of the timed steps; prints per-stage "
                         "busy / overlap / idle to stderr (the events sit inside the timed window)")
    ap.add_argument("--slack", type=int, default=0,
                    help="extra input slots: the host's ingress of batch i+depth waits for batch i-1-slack "
                         "to finish instead of batch i-1, so the next batch is already queued on the GPU "
                         "when a batch retires (0: the pre-round-6 behaviour)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="split each GPU's batch into this many concurrent hipGraph lanes "
                         "(kdl/engine/lanes.py; default 2 when the batch is even)")
    ap.add_argument("--stages", default=None, metavar="STEP",
                    help="stage-pipeline the forward (kdl/engine/stages.py): cut after this step; stage 1 "
                         "of batch i+1 overlaps stage 2 of batch i. Default: the model's cut (Xception: "
                         "block8_sepconv3 since the fused entry blocks of round 4; stages measured +10 %% over 2 lanes); 'none' = lanes")
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
    # process-group backend. auto: gloo when the data path is all native RCCL (the group then only
    # carries host-side control: barriers, the comm id, the max-over-ranks of the clock), nccl when
    # torch collectives move data (--gather-impl torch, --ingress scatter). A second RCCL
    # communicator (torch's, beside the native one) cost 17 %% at world 1 (profiles/dist_path_r5.txt)
    ap.add_argument("--dist-backend", default="auto", help=argparse.SUPPRESS)
    ap.add_argument("--egress", choices=["gather", "local"], default="gather",
                    help="gather: RCCL-gather every step's logits to rank 0 (+ D2H there); local: each rank "
                         "D2Hs its own logits (what per-GPU serving executors do)")
    ap.add_argument("--gather-impl", choices=["native", "torch"], default="torch",
                    help="torch: torch.distributed.gather (its NCCL process group runs the collective on an "
                         "internal stream: a fifth stream beside 2 stages + H2D + comm; -1 %% vs no process group "
                         "at world 1); native: kdl._C.RcclComm.gather posted on the comm stream with a gloo control "
                         "group (-4 %%). profiles/dist_path_r5.txt")
    ap.add_argument("--force-dist", action="store_true",
                    help="take the multi-rank code path (process group, RCCL gather) even with one rank: "
                         "measures the collective overhead on a 1-GPU box")
    a = ap.parse_args(argv)

    launched = "WORLD_SIZE" in os.environ
    if not launched and a.gpus is not None and a.gpus > 1:
        return launch_ranks(a, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus is not None and a.gpus != world:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    if a.dry_run:
        return dry_run(a, rank, local, world)
    ndev = torch.cuda.device_count()
    shared = local >= ndev
    if shared and not a.allow_shared:
        print(f"bench.py: rank {rank} has LOCAL_RANK {local} but only {ndev} GPU(s) are visible; "
              f"refusing to share a GPU (--allow-shared)", file=sys.stderr)
        return 2
    local = local % max(1, ndev)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_on = world > 1 or a.force_dist
    if a.dist_backend == "auto":
        a.dist_backend = "gloo" if a.gather_impl == "native" and a.ingress != "scatter" else "nccl"
    cdev = dev if a.dist_backend == "nccl" else torch.device("cpu")    # where host-control collectives run
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
    NS = a.depth + 1 + a.slack
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
    # instead. Streams per rank at world > 1: 2 stages + H2D + the comm stream, plus the internal
    # stream torch.distributed's NCCL process group runs its collectives on: five streams on
    # GPU_MAX_HW_QUEUES = 4. Measured at world 1 under torchrun (profiles/dist_path_r5.txt): that
    # path costs 1 % against no process group at all; posting a native RCCL gather on the comm
    # stream (four streams) cost 4 %, and a second RCCL communicator beside torch's 17 %.
    ds = torch.cuda.Stream(device=dev) if not gather and not a.stages else None
    rcomm = None
    if gather and a.gather_impl == "native":
        ids = [C.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0)
        rcomm = C.RcclComm(ids[0], world, rank, local)
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
                if rcomm is not None:       # peers' blocks only; rank 0's own leaves from its slot
                    rcomm.gather(out.data_ptr(), logits_all[j].data_ptr(), out.numel() * out.element_size(),
                                 ms.cuda_stream)
                    if rank == 0:
                        d2h(out_host[j][:B], out, ms)
                        if world > 1:
                            d2h(out_host[j][B:], logits_all[j][B:], ms)
                else:
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
    # settle: run the pipelined step itself (untimed, before the warmup steps) until its time is
    # stable -- at least --settle and at most --settle-max seconds. Serial replays were used until
    # round 6, but the pipelined regime kept speeding up for ~60 steps after them (20 steps after
    # 5 warmup steps read 1.28 ms/step, after 60 warmup steps 1.254: profiles/bench_settle_r6.txt).
    # Ranks agree on every chunk (a step may hold collectives), so all run the same count.
    if a.settle_mode == "pipe":
        # one joined replay first, so every pipeline-stage stream submits work before the ingress copy
        # stream does: HIP binds streams to its GPU_MAX_HW_QUEUES (4 on the box) hardware queues in
        # first-use order. With the copies first, ResNet-50's three stages + the copy stream read 17 %
        # lower (32.5k vs 39.1k img/s); Xception's two stages read 0.4 % higher that way, so the touch
        # is on for 3+ stages only (profiles/bench_settle_r6.txt)
        touch = a.touch == "on" or (a.touch == "auto" and len(getattr(eng, "ranges", ())) >= 3)
        if touch:
            eng.launch(B, s, capture=use_graph)
            torch.cuda.synchronize()
        for i in range(a.depth):
            ingress(i)
    nxt = 0
    t_start = time.perf_counter()
    chunk_ms: list[float] = []
    while True:
        c0 = time.perf_counter()
        for _ in range(10):
            if a.settle_mode == "pipe":
                step(nxt)
                nxt += 1
            else:
                eng.launch(B, s, capture=use_graph)
        torch.cuda.synchronize()
        chunk_ms.append((time.perf_counter() - c0) * 1e3)
        spent = time.perf_counter() - t_start
        stable = len(chunk_ms) >= 3 and abs(chunk_ms[-1] - chunk_ms[-2]) <= 0.01 * chunk_ms[-2]
        more = not (spent >= a.settle_max or (spent >= a.settle and stable))
        if dist_on:
            t = torch.tensor([int(more)], device=cdev, dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            more = bool(t.item())
        if not more:
            break
    settle_s = time.perf_counter() - t_start
    if rank == 0:   # settle trajectory of the untimed pipelined steps (fresh-lease diagnosis, stderr only)
        print("settle chunks (10 pipelined steps, ms): " + " ".join(f"{c:.2f}" for c in chunk_ms), file=sys.stderr)
    if a.settle_mode != "pipe":
        for i in range(a.depth):
            ingress(i)
    if dist_on:
        dist.barrier()
    for i in range(nxt, nxt + a.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()

    tt[:] = [0.0, 0.0, 0.0]
    if a.timeline and a.stages:
        eng.trace = []
    t0 = time.perf_counter()
    for i in range(nxt + a.warmup, nxt + total):
        step(i)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if a.timeline and a.stages and rank == 0:
        _print_timeline(eng.trace, len(eng.ranges))
        eng.trace = None
    if dist_on:
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
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
        t = torch.tensor(lat, device=cdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lat = t.tolist()

    gpus_shared = shared
    if dist_on:
        t = torch.tensor([int(shared)], device=cdev, dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gpus_shared = bool(t.item())
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
            "settle_s": round(settle_s, 3),
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
                       "ingress": a.ingress, "egress": (f"{a.egress} ({a.gather_impl})" if a.egress == "gather" else a.egress) if dist_on else "local", "hipgraph": use_graph, "lanes": a.lanes,
                       **({"stages": f"{len(eng.ranges)} (cut after {a.stages})"} if a.stages else {})},
            **({"gpus_shared": True} if gpus_shared else {}),
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


def _print_timeline(trace: list, K: int) -> None:
    """--timeline: per-stage busy time, the time both stages ran at once and each stream's idle
    time between its consecutive stage runs, from the timing events around every stage launch."""
    ref = trace[0][2]
    iv = [(k, ref.elapsed_time(e0), ref.elapsed_time(e1)) for _, k, e0, e1 in trace]
    span = max(e for _, _, e in iv) - min(s for _, s, _ in iv)
    n = len(iv) // K
    out = [f"timeline: {n} batches, {span / n * 1e3:.1f} us per batch"]
    for k in range(K):
        mine = sorted((s, e) for kk, s, e in iv if kk == k)
        busy = sum(e - s for s, e in mine)
        idle = sum(max(0.0, b[0] - a[1]) for a, b in zip(mine, mine[1:]))
        out.append(f"  stage {k + 1}: run {busy / n * 1e3:7.1f} us/batch, idle between runs {idle / max(1, n - 1) * 1e3:7.1f} us")
    ev = sorted([(s, 1) for _, s, _ in iv] + [(e, -1) for _, _, e in iv])
    cnt, last, both = 0, None, 0.0
    for t, d in ev:
        if last is not None and cnt >= 2:
            both += t - last
        cnt += d
        last = t
    out.append(f"  two stages at once: {both / n * 1e3:.1f} us/batch")
    print("\n".join(out), file=sys.stderr)


def dry_run(a, rank: int, local: int, world: int) -> int:
    """--dry-run: the rank wiring without a GPU (tests/test_bench_launcher.py). Every rank joins
    a gloo group on the launcher's rendezvous, reports its env, and rank 0 prints one JSON line."""
    print(f"bench.py dry-run rank={rank} local_rank={local} world={world} "
          f"master={os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}", file=sys.stderr, flush=True)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        t = torch.tensor([rank + 1])
        dist.all_reduce(t)
        assert t.item() == world * (world + 1) // 2, t
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": 0.0, "unit": "images/s", "n_gpus": world,
                          "steps": a.steps, "warmup": a.warmup, "dry_run": True,
                          "config": {"parallelism": f"dp{world}"}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
