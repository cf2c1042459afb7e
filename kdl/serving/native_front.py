"""Python side of the native gRPC front-end (kdl._rt.GrpcFront, csrc/runtime/grpc_front.h).

The C++ front-end owns the sockets, HTTP/2 and the Predict fast path (parse -> the signature's
C++ batcher -> response, no Python per request). Python keeps three jobs:

* the SLOW PATH: every request the fast path does not take (other methods, pinned versions or
  labels, requests it would reject, serving_image) runs the unchanged ``grpc_server.Servicer``
  method through ``_Context``, a stand-in for the slice of ``grpc.ServicerContext`` it uses --
  so status codes and messages are byte-for-byte the grpcio front-end's;
* ROUTES: after the slow path served a (model, signature) Predict of the latest version, its
  batcher (and, for the f32 signature, the uint8 one of the exact-u8 rule) is registered as a
  fast route; every version change drops them all (ModelManager.listeners);
* METRICS: the fast path's counters and latency histogram are merged into the Prometheus
  registry at scrape time (kdl_requests_total, kdl_request_latency_ms, kdl_f32_as_uint8_total).

Reference being replaced: TF-Serving's C++ gRPC server behind
/root/reference/tf-serving-clothing-model-deployment.yaml:20-27, driven by the gateway's
PredictionServiceStub (/root/reference/model_server.py:15-16,38-55).
"""
from __future__ import annotations

import logging
import threading

import grpc

from ..ops import _lib
from . import protos as P
from .backend import NATIVE_SIGNATURE, ServingError
from .metrics import METRICS

log = logging.getLogger("kdl.serving")

PREDICT = "/tensorflow.serving.PredictionService/Predict"
_CODE_NAMES = {sc.value[0]: sc.name for sc in grpc.StatusCode}


def available() -> tuple[bool, str]:
    """(True, "") when libnghttp2 loads (the front-end can start), else (False, why)."""
    return tuple(_lib.rt().http2_available())


class _Abort(Exception):
    pass


class _Context:
    """What ``Servicer`` uses of ``grpc.ServicerContext``: abort, time_remaining,
    send_initial_metadata."""

    def __init__(self, deadline_us: int):
        self.deadline_us = deadline_us
        self.code, self.details, self.meta = 0, "", []

    def time_remaining(self):
        if not self.deadline_us:
            return None
        return max(0.0, (self.deadline_us - _lib.rt().now_us()) * 1e-6)

    def abort(self, code, details):
        self.code, self.details = code.value[0], details
        raise _Abort()

    def send_initial_metadata(self, md):
        self.meta.extend((str(k), str(v)) for k, v in md)


class NativeFront:
    def __init__(self, manager, servicer, host: str, port: int, io_threads: int = 4, slow_threads: int = 64,
                 f32_exact_u8: bool = True, max_request_bytes: int = 64 << 20, reuse_port: bool = True):
        self.m, self.sv, self.f32_exact_u8 = manager, servicer, f32_exact_u8
        sp, ms = "/tensorflow.serving.PredictionService/", "/tensorflow.serving.ModelService/"
        self.methods = {
            PREDICT: servicer.predict,
            sp + "GetModelMetadata": servicer.get_model_metadata,
            sp + "Classify": servicer.unimplemented,
            sp + "Regress": servicer.unimplemented,
            sp + "MultiInference": servicer.unimplemented,
            ms + "GetModelStatus": servicer.get_model_status,
            ms + "HandleReloadConfigRequest": servicer.reload_config,
            "/grpc.health.v1.Health/Check": servicer.health_check,
        }
        self._lock = threading.Lock()
        self._learned: set[tuple] = set()
        self._gen = 0                    # bumped by every version change (_changed)
        self._last = {"by_code": {}, "lat_counts": None, "lat_sum_ms": 0.0, "exact_u8": 0}
        self.front = _lib.rt().GrpcFront(host, port, io_threads, slow_threads, self._slow,
                                         max_recv_bytes=max_request_bytes, reuse_port=reuse_port)
        self.port = self.front.port
        manager.listeners.append(self._changed)
        METRICS.poller(f"native_grpc:{id(self)}", self._poll)

    # ------------------------------------------------------------ slow path
    def _slow(self, path: str, msg: bytes, deadline_us: int):
        fn = self.methods.get(path)
        if fn is None:
            return 12, "Method not found!", b"", []           # grpcio's UNIMPLEMENTED text
        ctx = _Context(deadline_us)
        try:
            body = fn(msg, ctx)
        except _Abort:
            return ctx.code, ctx.details, b"", ctx.meta
        except Exception as e:  # noqa: BLE001 - grpcio's handler-exception answer
            log.exception("gRPC handler %s failed", path)
            return 2, f"Exception calling application: {e}", b"", ctx.meta
        if path == PREDICT:
            try:
                self._learn(msg)
            except Exception:  # noqa: BLE001 - the answer is already made; the route stays slow
                log.exception("native front-end: route registration failed")
        return 0, "", body, ctx.meta

    def _learn(self, msg: bytes) -> None:
        spec = _lib.rt().parse_model_spec_request(msg)        # PredictRequest field 1 = ModelSpec
        if spec["version"] >= 0 or spec["version_label"]:
            return
        sig_name = spec["signature_name"] or "serving_default"
        try:
            s = self.m.get(spec["name"])
        except ServingError:
            return
        key = (s.name, s.version, sig_name)
        with self._lock:
            if key in self._learned:
                return
            gen = self._gen
        runner = s.runner(sig_name)
        sig = runner.sig
        if sig.input_shape[1] <= 0 or not hasattr(runner, "batcher") or not runner.healthy():
            return                                             # serving_image: resize path, slow
        u8 = None
        if self.f32_exact_u8 and sig.input_dtype == P.DT_FLOAT and NATIVE_SIGNATURE in s.signatures:
            u8 = s.runner(NATIVE_SIGNATURE).batcher
        with self._lock:
            # a version change between the lookup above and here (advisor r5) already cleared the
            # routes: registering now would send unversioned requests to the retiring batcher
            if gen != self._gen:
                return
            self.front.set_route(model=s.name, signature=sig_name, version=s.version, input_key=sig.input_key,
                                 output_key=sig.output_key, dtype=sig.input_dtype, image=sig.input_shape[1],
                                 out_cols=s.source.classes, batcher=runner.batcher, u8=u8)
            self._learned.add(key)

    def _changed(self) -> None:
        with self._lock:
            self._gen += 1
            self._learned.clear()
            self.front.clear_routes()

    # ------------------------------------------------------------ metrics
    def _poll(self) -> None:
        st = self.front.stats()
        with self._lock:
            last = self._last
            for code, n in st["by_code"].items():
                d = n - last["by_code"].get(code, 0)
                if d:
                    METRICS.inc("kdl_requests_total", d, code=_CODE_NAMES.get(code, str(code)), method="Predict")
            prev = last["lat_counts"] or [0] * len(st["lat_counts"])
            delta = [a - b for a, b in zip(st["lat_counts"], prev)]
            if any(delta):
                METRICS.merge_hist("kdl_request_latency_ms", delta, st["lat_sum_ms"] - last["lat_sum_ms"],
                                   method="Predict")
            d = st["exact_u8"] - last["exact_u8"]
            if d:
                METRICS.inc("kdl_f32_as_uint8_total", d)
            self._last = {"by_code": dict(st["by_code"]), "lat_counts": list(st["lat_counts"]),
                          "lat_sum_ms": st["lat_sum_ms"], "exact_u8": st["exact_u8"]}

    def stats(self) -> dict:
        return self.front.stats()

    def stop(self) -> None:
        try:
            self.m.listeners.remove(self._changed)
        except ValueError:
            pass
        self._poll()
        METRICS.drop_poller(f"native_grpc:{id(self)}")
        self.front.stop()
