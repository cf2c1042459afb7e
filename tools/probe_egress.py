"""Egress-overlap probe: which part of bench.py's per-step pipeline (ingress H2D
on a copy stream, logits D2D on the compute stream, D2H on an egress stream) costs
time on top of back-to-back graph replays."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from kdl.engine import registry  # noqa: E402
from kdl.engine.tuning import tuning_path  # noqa: E402

info = registry.get("xception")
eng = info.engine(info.init_params(0), 32, torch.device("cuda", 0))
eng.load_tuning(tuning_path("xception", 32))
S = info.input_size
NS = 3
slots = eng.add_input_slots(NS)
for j in range(NS):
    eng.program(32, True, j)
host = torch.randint(0, 256, (32, S, S, 3), dtype=torch.uint8).pin_memory()
s, cs, ds = eng.stream, torch.cuda.Stream(), torch.cuda.Stream()
lbuf = [torch.zeros((32, 10), device="cuda") for _ in range(NS)]
out_host = [torch.zeros((32, 10)).pin_memory() for _ in range(NS)]
E = lambda: [torch.cuda.Event() for _ in range(NS)]  # noqa: E731
ready, free, done, drained = E(), E(), E(), E()
for e in free + done + drained:
    e.record(s)


outs = eng.slot_logits


def run_bench(depth, wait_before=True, n=100):
    """bench.py's step structure: ingress(i+depth), graph(i) into slot logits, D2H."""
    torch.cuda.synchronize()

    def ingress(i):
        j = i % NS
        with torch.cuda.stream(cs):
            cs.wait_event(free[j])
            slots[j].copy_(host, non_blocking=True)
            ready[j].record(cs)

    for i in range(depth):
        ingress(i)
    for i in range(n + 5):
        if i == 5:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        j = i % NS
        ingress(i + depth)
        s.wait_event(ready[j])
        if wait_before:
            s.wait_event(drained[j])
        eng.launch(32, s, slot=j)
        free[j].record(s)
        with torch.cuda.stream(ds):
            ds.wait_event(free[j])
            out_host[j].copy_(outs(j), non_blocking=True)
            drained[j].record(ds)
        if not wait_before:
            s.wait_event(drained[(j + 1) % NS])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def run(mode, n=100):
    torch.cuda.synchronize()
    for i in range(n + 5):
        if i == 5:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        j = i % NS
        if "h2d" in mode:
            with torch.cuda.stream(cs):
                cs.wait_event(free[j])
                slots[j].copy_(host, non_blocking=True)
                ready[j].record(cs)
            s.wait_event(ready[j])
        eng.launch(32, s, slot=j)
        free[j].record(s)
        if "lbuf" in mode:
            with torch.cuda.stream(s):
                s.wait_event(drained[j])
                lbuf[j].copy_(eng.logits[:32])
                done[j].record(s)
        if "d2h" in mode:
            with torch.cuda.stream(ds):
                ds.wait_event(done[j])
                out_host[j].copy_(lbuf[j], non_blocking=True)
                drained[j].record(ds)
        if "hostd2h" in mode:   # D2H on the compute stream itself
            with torch.cuda.stream(s):
                out_host[j].copy_(lbuf[j], non_blocking=True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for _ in range(2):
    for d in (1, 2):
        print(f"bench-like depth {d}     {run_bench(d):.3f} ms/step", flush=True)
        print(f"bench-like depth {d} late {run_bench(d, False):.3f} ms/step", flush=True)
    for m in ("graph", "h2d", "h2d+lbuf", "h2d+lbuf+d2h", "lbuf+d2h", "h2d+lbuf+hostd2h"):
        print(f"{m:20s} {run(m):.3f} ms/step", flush=True)
