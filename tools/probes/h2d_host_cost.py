#!/usr/bin/env python
"""Host-side cost of issuing the per-step ingress copy (8.6 MB pinned -> device,
32 uint8 299x299x3 images) and the egress copy (32x10 fp32 -> pinned), torch
copy_ vs raw hipMemcpyAsync through ctypes. bench.py's host issue time per step
jumps from 0.13 ms (no ingress) to 0.6-0.95 ms (with ingress)."""
import ctypes
import time

import torch

S = 299 * 299 * 3
h = torch.randint(0, 256, (32 * S,), dtype=torch.uint8).pin_memory()
d = torch.empty_like(h, device="cuda")
lo = torch.zeros(32 * 10, dtype=torch.float32, device="cuda")
lh = torch.zeros(32 * 10, dtype=torch.float32).pin_memory()
cs = torch.cuda.Stream()
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]


def bench(name, fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    t.sort()
    print(f"{name:34s} host us: median {t[n // 2] * 1e6:8.1f}  p90 {t[int(n * 0.9)] * 1e6:8.1f}", flush=True)


def torch_h2d():
    with torch.cuda.stream(cs):
        d.copy_(h, non_blocking=True)


def raw_h2d():
    hip.hipMemcpyAsync(d.data_ptr(), h.data_ptr(), h.numel(), 1, ctypes.c_void_p(cs.cuda_stream))


def torch_d2h():
    with torch.cuda.stream(cs):
        lh.copy_(lo, non_blocking=True)


def raw_d2h():
    hip.hipMemcpyAsync(lh.data_ptr(), lo.data_ptr(), lo.numel() * 4, 2, ctypes.c_void_p(cs.cuda_stream))


bench("torch copy_ H2D 8.6 MB", torch_h2d)
bench("hipMemcpyAsync H2D 8.6 MB", raw_h2d)
bench("torch copy_ D2H 1.3 KB", torch_d2h)
bench("hipMemcpyAsync D2H 1.3 KB", raw_d2h)
# GPU time of the H2D and whether it overlaps a busy compute stream
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(cs)
for _ in range(10):
    raw_h2d()
e1.record(cs)
e1.synchronize()
print(f"H2D GPU time {e0.elapsed_time(e1) / 10 * 1e3:.1f} us each")

# Does the async H2D block the host while its stream waits on an event of unfinished work?
busy = torch.cuda.Stream()
a_ = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
ev = torch.cuda.Event()
for label, wait in (("idle copy stream", False), ("copy stream waits on busy work", True)):
    ts = []
    for _ in range(10):
        with torch.cuda.stream(busy):
            for _ in range(20):
                a_ = (a_ @ a_).clamp_(-1, 1)      # ~2-4 ms of GPU work
            ev.record(busy)
        if wait:
            cs.wait_event(ev)
        t0 = time.perf_counter()
        raw_h2d()
        ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    ts.sort()
    print(f"{label:34s} host us: median {ts[5] * 1e6:8.1f}  max {ts[-1] * 1e6:8.1f}", flush=True)

# Same, but the event follows a hipGraph replay (what bench.py's slots wait on)
g_in = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
gs = torch.cuda.Stream()
graph = torch.cuda.CUDAGraph()
with torch.cuda.stream(gs):
    y_ = g_in @ g_in
    torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=gs):
        for _ in range(20):
            y_ = (y_ @ g_in).clamp_(-1, 1)
torch.cuda.synchronize()
big = torch.zeros(64 * 1024 // 4, dtype=torch.float32).pin_memory()
bigd = torch.zeros(64 * 1024 // 4, dtype=torch.float32, device="cuda")
cases = {
    "H2D 8.6 MB": lambda: hip.hipMemcpyAsync(d.data_ptr(), h.data_ptr(), h.numel(), 1, ctypes.c_void_p(cs.cuda_stream)),
    "D2H 1.3 KB": lambda: hip.hipMemcpyAsync(lh.data_ptr(), lo.data_ptr(), lo.numel() * 4, 2, ctypes.c_void_p(cs.cuda_stream)),
    "D2H 10 KB": lambda: hip.hipMemcpyAsync(big.data_ptr(), bigd.data_ptr(), 10240, 2, ctypes.c_void_p(cs.cuda_stream)),
    "D2H 64 KB": lambda: hip.hipMemcpyAsync(big.data_ptr(), bigd.data_ptr(), 65536, 2, ctypes.c_void_p(cs.cuda_stream)),
}
for label, fn in cases.items():
    for mode in ("idle", "wait-on-graph-event", "same-stream-after-graph"):
        ts = []
        for _ in range(8):
            graph.replay() if mode != "idle" else None
            if mode == "wait-on-graph-event":
                with torch.cuda.stream(gs):
                    graph.replay()
                    ev.record(gs)
                cs.wait_event(ev)
            elif mode == "same-stream-after-graph":
                with torch.cuda.stream(cs):
                    graph.replay()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        ts.sort()
        print(f"{label:12s} {mode:26s} host us: median {ts[4] * 1e6:8.1f}  max {ts[-1] * 1e6:8.1f}", flush=True)
