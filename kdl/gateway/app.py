"""Serving gateway: ``POST /predict {"url": ...}`` -> ``{label: logit}``.

Same contract as the reference Flask gateway (`model_server.py:59-70`, SURVEY.md
§2.9.1): Flask app named 'clothing-model', backend address from
``TF_SERVING_HOST`` (default ``localhost:8500``), Xception preprocessing, gRPC
Predict with a 20 s deadline, ten labels in model output order. Improvements
the reference lacks (§8.1): JSON errors (400 bad body, 502 fetch/backend errors,
504 deadline) instead of bare 500s, a batch route, health probes, and a native
mode that ships uint8 pixels to the ``serving_uint8`` signature (4x fewer bytes).

Env: TF_SERVING_HOST, MODEL_NAME, SIGNATURE, INPUT_KEY, OUTPUT_KEY, LABELS,
GATEWAY_MODE=compat|uint8|raw (raw: decoded pixels at their own size to ``serving_image``,
resized on the model server's GPU -- no resize here), PREDICT_TIMEOUT, GATEWAY_CHANNELS (gRPC connections to open:
each gets its own subchannel, so a node running one model-server process per GPU on a
shared SO_REUSEPORT port -- ``--procs`` -- sees the gateway's requests spread over all
of them instead of pinned to whichever process accepted a single connection).
"""
from __future__ import annotations

import itertools
import os
import threading
import urllib.error

import grpc
import numpy as np
from flask import Flask, jsonify, request

from ..labels import LABELS as DEFAULT_LABELS
from . import preprocess as pp
from .client import PredictionStub, make_request, process_batch_response, process_response


class GatewayConfig:
    def __init__(self, env=None):
        env = os.environ if env is None else env
        self.server = env.get("TF_SERVING_HOST", "localhost:8500")
        self.model_name = env.get("MODEL_NAME", "clothing-model")
        self.mode = env.get("GATEWAY_MODE", "compat")
        if self.mode not in ("compat", "uint8", "raw"):
            raise ValueError(f"GATEWAY_MODE must be compat, uint8 or raw, got {self.mode!r}")
        self.signature = env.get("SIGNATURE", {"compat": "serving_default", "uint8": "serving_uint8",
                                               "raw": "serving_image"}[self.mode])
        self.input_key = env.get("INPUT_KEY", "input_8" if self.mode == "compat" else "images")
        self.output_key = env.get("OUTPUT_KEY", "dense_7")
        labels = env.get("LABELS", "")
        self.labels = [s for s in labels.split(",") if s] or list(DEFAULT_LABELS)
        self.timeout = float(env.get("PREDICT_TIMEOUT", "20.0"))
        self.channels = max(1, int(env.get("GATEWAY_CHANNELS", "1")))


def create_app(cfg: GatewayConfig | None = None, channel: grpc.Channel | None = None) -> Flask:
    cfg = cfg or GatewayConfig()
    opts = [("grpc.max_send_message_length", -1), ("grpc.max_receive_message_length", -1)]
    if channel is not None:
        stubs = [PredictionStub(channel)]
    else:
        # one connection per channel (a local subchannel pool each), round-robin per request
        extra = [("grpc.use_local_subchannel_pool", 1)] if cfg.channels > 1 else []
        stubs = [PredictionStub(grpc.insecure_channel(cfg.server, options=opts + extra)) for _ in range(cfg.channels)]
    rr, rr_lock = itertools.cycle(stubs), threading.Lock()

    def next_stub():
        with rr_lock:
            return next(rr)
    preprocessor = pp.create_preprocessor("xception", target_size=(299, 299))
    app = Flask("clothing-model")
    app.config["kdl_gateway"] = cfg

    def tensor_from_image(img):
        if cfg.mode == "uint8":
            return pp.to_uint8(img)[None]
        if cfg.mode == "raw":
            return np.asarray(img, dtype=np.uint8)[None]
        return pp.image_to_tensor(img)

    def run(X: np.ndarray):
        req = make_request(X, cfg.model_name, cfg.signature, cfg.input_key)
        return next_stub().Predict(req, timeout=cfg.timeout)

    def fail(code: int, msg: str):
        return jsonify({"error": msg}), code

    def grpc_fail(e: grpc.RpcError):
        code = e.code() if hasattr(e, "code") else None
        http = {grpc.StatusCode.DEADLINE_EXCEEDED: 504, grpc.StatusCode.INVALID_ARGUMENT: 400,
                grpc.StatusCode.NOT_FOUND: 404, grpc.StatusCode.UNAVAILABLE: 503,
                grpc.StatusCode.RESOURCE_EXHAUSTED: 429}.get(code, 502)
        details = e.details() if hasattr(e, "details") else str(e)
        return fail(http, f"model server error ({code.name if code else 'UNKNOWN'}): {details}")

    def load(url: str):
        try:
            return pp.load_image(pp.fetch(url))
        except (urllib.error.URLError, ValueError, OSError) as e:
            raise LookupError(f"could not fetch/decode image from {url!r}: {e}") from e

    @app.route("/predict", methods=["POST"])
    def predict():
        body = request.get_json(silent=True)
        if not isinstance(body, dict) or not isinstance(body.get("url"), str):
            return fail(400, 'request body must be JSON {"url": "<image url>"}')
        try:
            img = load(body["url"])
        except LookupError as e:
            return fail(502, str(e))
        try:
            pb_result = run(tensor_from_image(img))
        except grpc.RpcError as e:
            return grpc_fail(e)
        return jsonify(process_response(pb_result, cfg.labels, cfg.output_key))

    @app.route("/predict_batch", methods=["POST"])
    def predict_batch():
        body = request.get_json(silent=True)
        urls = body.get("urls") if isinstance(body, dict) else None
        if not isinstance(urls, list) or not urls or not all(isinstance(u, str) for u in urls):
            return fail(400, 'request body must be JSON {"urls": ["<image url>", ...]}')
        try:
            Xs = [tensor_from_image(load(u)) for u in urls]
        except LookupError as e:
            return fail(502, str(e))
        try:
            if cfg.mode == "raw" and len({x.shape for x in Xs}) > 1:
                # raw pixels of different sizes cannot share one dense tensor: one request each
                return jsonify([process_response(run(x), cfg.labels, cfg.output_key) for x in Xs])
            pb_result = run(np.concatenate(Xs))
        except grpc.RpcError as e:
            return grpc_fail(e)
        return jsonify(process_batch_response(pb_result, cfg.labels, cfg.output_key))

    @app.route("/healthz", methods=["GET"])
    def healthz():
        return jsonify({"status": "alive", "backend": cfg.server})

    return app


def main():  # dev entry like the reference's app.run (model_server.py:69-70), without debug=True
    create_app().run(host="0.0.0.0", port=int(os.environ.get("PORT", "9696")))


if __name__ == "__main__":
    main()
