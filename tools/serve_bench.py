#!/usr/bin/env python
"""Closed-loop serving benchmark through the real gRPC server:
C concurrent clients each send Predict requests of `--images` images back to back;
reports throughput (images/s) and p50/p99 request latency. Starts an in-process
server on a synthetic model unless --target is given.

  python tools/serve_bench.py --clients 64 --images 1 --seconds 20 --signature serving_uint8
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


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", default=None)
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--images", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=15)
    ap.add_argument("--signature", default="serving_uint8", choices=["serving_uint8", "serving_default"])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--timeout-us", type=int, default=1000)
    ap.add_argument("--device", default="auto")
    a = ap.parse_args(argv)
    from kdl.gateway.client import PredictionStub, make_request
    srv = None
    target = a.target
    if target is None:
        import tempfile

        from kdl.serving.config import BatchingParams, ServerConfig
        from kdl.serving.server import ModelServer
        base = os.path.join(tempfile.mkdtemp(), "clothing-model")
        os.makedirs(os.path.join(base, "1"))
        open(os.path.join(base, "1", "synthetic.json"), "w").write('{"seed": 0}')
        sizes = [b for b in (1, 2, 4, 8, 16, 32, 64) if b <= a.max_batch]
        cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=base, device=a.device, gpus=a.gpus,
                           host="127.0.0.1", file_system_poll_wait_seconds=0, grpc_max_threads=max(64, a.clients * 2),
                           batching=BatchingParams(max_batch_size=a.max_batch, batch_timeout_micros=a.timeout_us,
                                                   allowed_batch_sizes=sizes))
        srv = ModelServer(cfg).start(block_until_loaded=True)
        if a.signature != "serving_default":
            srv.manager.get("clothing-model").runner(a.signature)
        target = f"127.0.0.1:{srv.grpc_port}"
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, (a.images, 299, 299, 3), dtype=np.uint8)
    if a.signature == "serving_uint8":
        req = make_request(u8, signature="serving_uint8", input_key="images").SerializeToString()
    else:
        req = make_request(u8.astype(np.float32) / 127.5 - 1).SerializeToString()
    lat, lock = [], threading.Lock()
    stop = time.perf_counter() + a.seconds
    warm = time.perf_counter() + min(3.0, a.seconds / 4)

    def client():
        ch = grpc.insecure_channel(target, options=[("grpc.max_send_message_length", -1)])
        call = ch.unary_unary("/tensorflow.serving.PredictionService/Predict")
        while time.perf_counter() < stop:
            t0 = time.perf_counter()
            call(req, timeout=30)
            t1 = time.perf_counter()
            if t0 > warm:
                with lock:
                    lat.append(t1 - t0)
    ths = [threading.Thread(target=client) for _ in range(a.clients)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    span = stop - warm
    res = {"metric": "closed-loop gRPC serving", "clients": a.clients, "images_per_request": a.images,
           "signature": a.signature, "requests": len(lat), "images_per_s": round(len(lat) * a.images / span, 1),
           "p50_ms": round(statistics.median(lat) * 1e3, 2),
           "p99_ms": round(sorted(lat)[int(0.99 * (len(lat) - 1))] * 1e3, 2)}
    if srv is not None:
        st = srv.manager.get("clothing-model").runner(a.signature).batcher.stats()
        res["mean_batch"] = round(st["items"] / max(1, st["batches"]), 2)
        srv.stop(0)
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
