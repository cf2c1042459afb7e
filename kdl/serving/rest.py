"""TF-Serving REST API (:8501) + Prometheus metrics + k8s probes.

Routes (TF-Serving REST semantics):
  GET  /v1/models/<name>[/versions/<v>]            -> model_version_status
  GET  /v1/models/<name>[/versions/<v>]/metadata   -> signature_def
  POST /v1/models/<name>[/versions/<v>|/labels/<l>]:predict
       {"signature_name"?, "instances": [...]}  -> {"predictions": [...]}
       {"signature_name"?, "inputs": ...}       -> {"outputs": ...}
  GET  /monitoring/prometheus/metrics, /healthz (liveness), /readyz (readiness)
"""
from __future__ import annotations

import json
import time
import re
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np
from google.protobuf import json_format

from ..ops import _lib
from . import protos as P
from .backend import ServingError
from .grpc_server import route_exact_u8, signature_def_map
from .metrics import METRICS
from .model_repo import STATE_NAMES, ModelManager

_ROUTE = re.compile(r"^/v1/models/(?P<name>[^/:]+)(?:/versions/(?P<ver>\d+)|/labels/(?P<label>[^/:]+))?"
                    r"(?P<tail>:predict|/metadata)?/?$")
_HTTP = {"INVALID_ARGUMENT": 400, "NOT_FOUND": 404, "DEADLINE_EXCEEDED": 504, "UNAVAILABLE": 503,
         "RESOURCE_EXHAUSTED": 429, "UNIMPLEMENTED": 501, "INTERNAL": 500}


def make_handler(manager: ModelManager, f32_exact_u8: bool = True):
    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):  # quiet
            pass

        def _send(self, code: int, body, ctype="application/json"):
            data = body if isinstance(body, bytes) else (json.dumps(body) if not isinstance(body, str) else body).encode()
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def _err(self, e: ServingError):
            self._send(_HTTP.get(e.code, 500), {"error": str(e)})

        def do_GET(self):  # noqa: N802
            if self.path.startswith("/monitoring/prometheus/metrics"):
                return self._send(200, METRICS.render(), "text/plain; version=0.0.4")
            if self.path == "/healthz":
                return self._send(200, {"status": "alive"})
            if self.path == "/readyz":
                ok = manager.ready()
                return self._send(200 if ok else 503, {"ready": ok})
            m = _ROUTE.match(self.path)
            if not m or m.group("tail") == ":predict":
                return self._send(404, {"error": "not found"})
            try:
                ver = int(m.group("ver")) if m.group("ver") else None
                if m.group("tail") == "/metadata":
                    s = manager.get(m.group("name"), ver, m.group("label"))
                    sdm = json_format.MessageToDict(signature_def_map(s))
                    return self._send(200, {"model_spec": {"name": s.name, "signature_name": "",
                                                           "version": str(s.version)},
                                            "metadata": {"signature_def": sdm}})
                if m.group("name") != manager.name:
                    raise ServingError("NOT_FOUND", f"Could not find any versions of model {m.group('name')}")
                st = [{"version": str(v), "state": STATE_NAMES.get(state, "UNKNOWN"),
                       "status": {"error_code": "OK" if not msg else "UNKNOWN", "error_message": msg}}
                      for v, state, msg in manager.status(ver)]
                return self._send(200, {"model_version_status": st})
            except ServingError as e:
                return self._err(e)

        def do_POST(self):  # noqa: N802
            m = _ROUTE.match(self.path)
            if not m or m.group("tail") != ":predict":
                return self._send(404, {"error": "not found"})
            t0 = time.perf_counter()
            try:
                n = int(self.headers.get("Content-Length", "0"))
                body = json.loads(self.rfile.read(n) or b"{}")
                ver = int(m.group("ver")) if m.group("ver") else None
                s = manager.get(m.group("name"), ver, m.group("label"))
                runner = s.runner(body.get("signature_name") or "serving_default")
                sig = runner.sig
                dt = np.uint8 if sig.input_dtype == P.DT_UINT8 else np.float32
                if "instances" in body:
                    inst = body["instances"]
                    if inst and isinstance(inst[0], dict):
                        inst = [i[sig.input_key] for i in inst]
                    x, rows = np.asarray(inst, dtype=dt), True
                elif "inputs" in body:
                    inp = body["inputs"]
                    if isinstance(inp, dict):
                        inp = inp[sig.input_key]
                    x, rows = np.asarray(inp, dtype=dt), False
                else:
                    raise ServingError("INVALID_ARGUMENT", "request must contain 'instances' or 'inputs'")
                S = sig.input_shape[1]
                if S == -1:          # serving_image: any size
                    if x.ndim != 4 or x.shape[3] != 3 or min(x.shape) < 1:
                        raise ServingError("INVALID_ARGUMENT", f"expected images [-1,-1,-1,3], got {list(x.shape)}")
                elif x.ndim != 4 or x.shape[1:] != (S, S, 3):
                    raise ServingError("INVALID_ARGUMENT", f"expected images [-1,{S},{S},3], got {list(x.shape)}")
                x = np.ascontiguousarray(x)
                dl = self.headers.get("X-Deadline-Ms")
                deadline = int(_lib.rt().now_us() + float(dl) * 1e3) if dl else 0
                n_img = x.shape[0]
                if f32_exact_u8:     # same routing as gRPC (--scatter rccl serves serving_uint8 over the node)
                    runner, x = route_exact_u8(s, runner, x, n_img)
                t1 = time.perf_counter()
                out = runner.predict(x, n_img, deadline).tolist()
                t2 = time.perf_counter()
                r = self._send(200, {"predictions": out} if rows else {"outputs": out})
                # same per-request stage trace as the gRPC path (SURVEY.md §5 tracing)
                METRICS.observe("kdl_stage_ms", (t1 - t0) * 1e3, stage="parse")
                METRICS.observe("kdl_stage_ms", (t2 - t1) * 1e3, stage="batch_and_run")
                METRICS.observe("kdl_stage_ms", (time.perf_counter() - t2) * 1e3, stage="respond")
                METRICS.inc("kdl_requests_total", code="OK", method="RestPredict")
                METRICS.observe("kdl_request_latency_ms", (time.perf_counter() - t0) * 1e3, method="RestPredict")
                return r
            except ServingError as e:
                METRICS.inc("kdl_requests_total", code=e.code, method="RestPredict")
                return self._err(e)
            except (ValueError, KeyError, TypeError) as e:
                return self._err(ServingError("INVALID_ARGUMENT", str(e)))

    return H


class _ReusePortHTTPServer(ThreadingHTTPServer):
    """SO_REUSEPORT listener: the per-GPU server processes of one node (``--procs``) all bind
    the same REST port and the kernel spreads connections over them."""

    def server_bind(self):
        import socket
        if hasattr(socket, "SO_REUSEPORT"):
            self.socket.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
        super().server_bind()


def start_rest_server(manager: ModelManager, host: str, port: int, reuse_port: bool = False,
                      f32_exact_u8: bool = True):
    srv = (_ReusePortHTTPServer if reuse_port else ThreadingHTTPServer)((host, port), make_handler(manager, f32_exact_u8))
    srv.daemon_threads = True
    t = threading.Thread(target=srv.serve_forever, name="rest", daemon=True)
    t.start()
    return srv
