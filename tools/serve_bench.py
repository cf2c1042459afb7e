#!/usr/bin/env python
"""Closed-loop serving benchmark through the real gRPC server:
C concurrent clients each send Predict requests of `--images` images back to back;
reports throughput (images/s) and p50/p99 request latency. Starts an in-process
server on a synthetic model unless --target is given.

  python tools/serve_bench.py --clients 64 --images 1 --seconds 20 --signature serving_uint8
  python tools/serve_bench.py --client native --conns 8 --clients 64 --device null   # front-end ceiling

--client native drives the server with the C++ load generator (kdl._rt.grpc_load: HTTP/2
connections each keeping clients/conns calls in flight); Python clients top out near 1-2k
req/s per process at one image per request, below what the native front-end serves.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import grpc  # noqa: E402
import numpy as np  # noqa: E402


def _client_proc(conn, threads: int, req: bytes, seconds: float, warm_s: float) -> None:  # noqa: C901
    """Client worker process (spawned BEFORE the server initialises the GPU): receives
    the target, runs `threads` closed-loop clients, sends back the post-warm-up latencies."""
    target = conn.recv()
    lat, lock = [], threading.Lock()
    t_start = time.perf_counter()
    stop, warm = t_start + seconds, t_start + warm_s

    def client():
        ch = grpc.insecure_channel(target, options=[("grpc.max_send_message_length", -1),
                                                    ("grpc.use_local_subchannel_pool", 1)])
        call = ch.unary_unary("/tensorflow.serving.PredictionService/Predict")
        while time.perf_counter() < stop:
            t0 = time.perf_counter()
            call(req, timeout=30)
            t1 = time.perf_counter()
            if t0 > warm:
                with lock:
                    lat.append(t1 - t0)
    ths = [threading.Thread(target=client) for _ in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    conn.send(lat)


def _launch_procs(a):
    """`python -m kdl.serving --procs N` on a fixed port, waited until every process answers."""
    import socket
    import subprocess
    import tempfile
    base = os.path.join(tempfile.mkdtemp(), "clothing-model")
    os.makedirs(os.path.join(base, "1"))
    open(os.path.join(base, "1", "synthetic.json"), "w").write('{"seed": 0}')
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    sizes = ",".join(str(b) for b in (1, 2, 4, 8, 16, 32, 64) if b <= a.max_batch)
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    topo = ([f"--scatter=rccl", f"--dp_world={a.dp_world}"] if a.scatter == "rccl" else [f"--procs={a.procs}"])
    cmd = [sys.executable, "-m", "kdl.serving", *topo, f"--port={port}", "--rest_api_port=0",
           f"--model_base_path={base}", f"--device={a.device}", "--host=127.0.0.1", f"--allowed_batch_sizes={sizes}",
           f"--batch_timeout_micros={a.timeout_us}", f"--grpc_max_threads={max(64, a.clients * 2)}",
           f"--warm_signatures={a.signature}"]
    if a.executors_per_gpu:
        cmd.append(f"--executors_per_gpu={a.executors_per_gpu}")
    cmd.append(f"--grpc_frontend={a.frontend}")
    p = subprocess.Popen(cmd, cwd=root, env=dict(os.environ, PYTHONPATH=root), stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, start_new_session=True)
    target = f"127.0.0.1:{port}"
    seen, t_end = set(), time.time() + 600
    want = 1 if a.scatter == "rccl" else a.procs
    while len(seen) < want and time.time() < t_end and p.poll() is None:
        ch = grpc.insecure_channel(target, options=[("grpc.use_local_subchannel_pool", 1)])
        try:
            resp, call = ch.unary_unary("/grpc.health.v1.Health/Check").with_call(b"", timeout=5)
            if resp == b"\x08\x01":
                seen.add(dict(call.initial_metadata()).get("kdl-pid"))
        except grpc.RpcError:
            time.sleep(0.5)
        finally:
            ch.close()
    if len(seen) < want:
        raise SystemExit(f"only {len(seen)} of {want} server processes came up")
    return p, target


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", default=None)
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--images", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=15)
    ap.add_argument("--signature", default="serving_uint8", choices=["serving_uint8", "serving_default", "serving_image"])
    ap.add_argument("--image-size", default="534x400",
                    help="serving_image: HxW of the raw uint8 images the clients send (resized on the server)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--timeout-us", type=int, default=1000)
    ap.add_argument("--no-eager", action="store_true",
                    help="idle executors wait out the batch timeout (TF-Serving behaviour) instead of "
                         "dispatching whatever is queued")
    ap.add_argument("--device", default="auto", help="auto | cpu | gpu | null (zero-latency fake device: "
                                                    "the serving front-end's own ceiling)")
    ap.add_argument("--executors-per-gpu", type=int, default=0)
    ap.add_argument("--procs", type=int, default=0,
                    help="serve from `python -m kdl.serving --procs N` (N processes sharing the port via "
                         "SO_REUSEPORT, one per GPU mod the visible GPUs) instead of an in-process server; "
                         "every client opens its own connection")
    ap.add_argument("--scatter", choices=["host", "rccl"], default="host",
                    help="rccl: serve from `python -m kdl.serving --scatter rccl --dp_world W` (one front-end, "
                         "the native RCCL data-parallel executor, serving/dp.py)")
    ap.add_argument("--dp-world", type=int, default=1)
    ap.add_argument("--no-f32-exact", action="store_true",
                    help="in-process server: f32 requests that are exact 8-bit pixels are NOT moved to the uint8 path")
    ap.add_argument("--stages", action="store_true",
                    help="in-process server: print the native executor's mean per-stage times")
    ap.add_argument("--frontend", choices=["native", "python"], default="native",
                    help="server gRPC front-end: native (C++ HTTP/2, Predict fast path) or python (grpcio)")
    ap.add_argument("--client", choices=["python", "native"], default="python",
                    help="native: the C++ closed-loop load generator (--conns connections, clients/conns "
                         "calls in flight on each)")
    ap.add_argument("--conns", type=int, default=8, help="--client native: HTTP/2 connections")
    ap.add_argument("--client-procs", type=int, default=0,
                    help="run the clients in this many spawned processes (0: threads of the server "
                         "process, which then share its GIL with the server's handlers)")
    a = ap.parse_args(argv)
    rng = np.random.default_rng(0)
    H, W = (299, 299) if a.signature != "serving_image" else map(int, a.image_size.split("x"))
    u8 = rng.integers(0, 256, (a.images, H, W, 3), dtype=np.uint8)
    procs = []
    if a.client_procs and a.client == "python":
        import multiprocessing as mp
        from kdl.gateway.client import make_request as _mk
        if a.signature != "serving_default":
            req0 = _mk(u8, signature=a.signature, input_key="images").SerializeToString()
        else:
            req0 = _mk(u8.astype(np.float32) / 127.5 - 1).SerializeToString()
        ctx = mp.get_context("spawn")         # before any GPU initialisation in this process
        per = [a.clients // a.client_procs + (1 if i < a.clients % a.client_procs else 0)
               for i in range(a.client_procs)]
        for n in per:
            parent, child = ctx.Pipe()
            pr = ctx.Process(target=_client_proc, args=(child, n, req0, a.seconds, min(3.0, a.seconds / 4)),
                             daemon=True)
            pr.start()
            procs.append((pr, parent))
    from kdl.gateway.client import PredictionStub, make_request
    srv = None
    launcher = None
    target = a.target
    if target is None and (a.procs or a.scatter == "rccl"):
        launcher, target = _launch_procs(a)
    if target is None:
        import tempfile

        from kdl.serving.config import BatchingParams, ServerConfig
        from kdl.serving.server import ModelServer
        base = os.path.join(tempfile.mkdtemp(), "clothing-model")
        os.makedirs(os.path.join(base, "1"))
        open(os.path.join(base, "1", "synthetic.json"), "w").write('{"seed": 0}')
        sizes = [b for b in (1, 2, 4, 8, 16, 32, 64) if b <= a.max_batch]
        cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=base, device=a.device, gpus=a.gpus,
                           executors_per_gpu=a.executors_per_gpu,
                           host="127.0.0.1", file_system_poll_wait_seconds=0, grpc_max_threads=max(64, a.clients * 2),
                           f32_exact_u8=not a.no_f32_exact, grpc_frontend=a.frontend,
                           batching=BatchingParams(max_batch_size=a.max_batch, batch_timeout_micros=a.timeout_us,
                                                   allowed_batch_sizes=sizes, eager_when_idle=not a.no_eager))
        srv = ModelServer(cfg).start(block_until_loaded=True)
        if a.signature != "serving_default":
            srv.manager.get("clothing-model").runner(a.signature)
        target = f"127.0.0.1:{srv.grpc_port}"
    if a.signature != "serving_default":
        req = make_request(u8, signature=a.signature, input_key="images").SerializeToString()
    else:
        req = make_request(u8.astype(np.float32) / 127.5 - 1).SerializeToString()
    lat, lock = [], threading.Lock()
    native_load = None
    if a.client == "native":
        from kdl.ops import _lib
        host, port = target.rsplit(":", 1)
        warm_s = min(3.0, a.seconds / 4)
        native_load = _lib.rt().grpc_load(host, int(port), "/tensorflow.serving.PredictionService/Predict", req,
                                          conns=a.conns, streams=max(1, a.clients // a.conns),
                                          seconds=a.seconds - warm_s, warm_s=warm_s)
        if native_load["error"] or native_load["failed"]:
            print(f"native load: {native_load['failed']} failed, codes {native_load['codes']}, "
                  f"error {native_load['error']!r}", file=sys.stderr)
        lat = [x * 1e-3 for x in native_load["lat_ms"]]
    stop = time.perf_counter() + (0 if native_load is not None else a.seconds)
    warm = time.perf_counter() + min(3.0, a.seconds / 4)
    if procs:
        for _, conn in procs:
            conn.send(target)
        for pr, conn in procs:
            lat.extend(conn.recv())
            pr.join()

    def client():
        ch = grpc.insecure_channel(target, options=[("grpc.max_send_message_length", -1),
                                                    ("grpc.use_local_subchannel_pool", 1)])
        call = ch.unary_unary("/tensorflow.serving.PredictionService/Predict")
        while time.perf_counter() < stop:
            t0 = time.perf_counter()
            call(req, timeout=30)
            t1 = time.perf_counter()
            if t0 > warm:
                with lock:
                    lat.append(t1 - t0)
    ths = [threading.Thread(target=client) for _ in range(0 if procs or native_load is not None else a.clients)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    span = native_load["seconds"] if native_load is not None else stop - warm
    res = {"metric": "closed-loop gRPC serving", "device": a.device, "clients": a.clients,
           "client": a.client, "frontend": a.frontend,
           "client_procs": a.client_procs, **({"conns": a.conns} if native_load is not None else {}),
           "images_per_request": a.images,
           "signature": a.signature, "requests": len(lat), "images_per_s": round(len(lat) * a.images / span, 1),
           "p50_ms": round(statistics.median(lat) * 1e3, 2),
           "p99_ms": round(sorted(lat)[int(0.99 * (len(lat) - 1))] * 1e3, 2)}
    if srv is not None:
        res["f32_exact_u8"] = not a.no_f32_exact
        if srv.native is not None:
            ns = srv.native.stats()
            res["native_front"] = {k: ns[k] for k in ("fast_ok", "fast_err", "slow", "exact_u8")}
        run = srv.manager.get("clothing-model").runner(a.signature)
        if a.signature == "serving_image":
            res["image_size"] = a.image_size
            res["resize_into_device_slot"] = bool(getattr(run, "device_path", False))
        run = getattr(run, "inner", run)      # serving_image: the serving_uint8 runner behind the resize
        st = run.batcher.stats()
        res["mean_batch"] = round(st["items"] / max(1, st["batches"]), 2)
        if a.stages:
            for ex in run.executors:
                nat = getattr(ex, "native", None)
                if nat is not None:
                    sg = nat.stats()["stages"]
                    res.setdefault("stage_mean_ms", {})[ex.name] = {
                        k: round(v["sum_ms"] / max(1, v["count"]), 3) for k, v in sg.items()}
        srv.stop(0)
    if launcher is not None:
        import signal
        res["procs"] = a.procs
        if a.scatter == "rccl":
            res["topology"] = f"scatter rccl, dp_world {a.dp_world}"
        os.killpg(launcher.pid, signal.SIGTERM)
        launcher.wait(timeout=60)
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
