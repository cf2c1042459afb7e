"""gRPC front-end: tensorflow.serving.PredictionService / ModelService + health.

Wire-compatible with the reference client (`model_server.py:15-16,38-55`):
method ``/tensorflow.serving.PredictionService/Predict``, request inputs as
``tensor_content``, outputs as ``float_val``. Handlers receive the *raw*
request bytes (no Python protobuf decode of the ~1 MB image): the native codec
in ``kdl._rt`` returns (offset, size) views and the payload goes straight into
the batcher. Max message size is unlimited like TF-Serving's INT32_MAX.
"""
from __future__ import annotations

import logging
import os
import time
from concurrent import futures

import grpc
import numpy as np

from ..ops import _lib
from . import protos as P
from .backend import NATIVE_SIGNATURE, ServingError
from .metrics import METRICS
from .model_repo import ModelManager

log = logging.getLogger("kdl.serving")

_ITEMSIZE = {P.DT_FLOAT: 4, P.DT_UINT8: 1}


def _deadline_us(context) -> int:
    rem = context.time_remaining() if context is not None else None
    if rem is None or rem > 1e8:
        return 0
    return int(_lib.rt().now_us() + rem * 1e6)


def _abort(context, err: ServingError):
    code = getattr(grpc.StatusCode, err.code, grpc.StatusCode.INTERNAL)
    context.abort(code, str(err))


def _payload(raw: bytes, td: dict, sig) -> tuple[object, int]:
    """Return (buffer of n images in the signature's dtype, n) from a parsed input."""
    dims = list(td["dims"])
    IMG = sig.input_shape[1]
    if IMG == -1:           # serving_image: uint8 [n, H, W, 3] of any size
        return _image_payload(raw, td, sig, dims)
    if td["dtype"] != sig.input_dtype:
        raise ServingError("INVALID_ARGUMENT",
                           f"Expects arg[0] to be {P.DTYPE_NAMES.get(sig.input_dtype)} but "
                           f"{P.DTYPE_NAMES.get(td['dtype'], td['dtype'])} is provided")
    if len(dims) != 4 or dims[1:] != [IMG, IMG, 3] or dims[0] < 1:
        raise ServingError("INVALID_ARGUMENT", f"input '{sig.input_key}' must have shape [-1,{IMG},{IMG},3], got {dims}")
    n = dims[0]
    item = _ITEMSIZE[sig.input_dtype]
    need = n * IMG * IMG * 3 * item
    vf = td["values_field"]
    if td["has_content"] or (vf == 5 and sig.input_dtype == P.DT_FLOAT):
        if td["size"] != need:
            if vf == 5 and td["size"] == item:   # single value broadcast (TF semantics)
                v = np.frombuffer(raw, dtype=np.float32, count=1, offset=td["offset"])[0]
                return np.full((n, IMG, IMG, 3), v, dtype=np.float32), n
            raise ServingError("INVALID_ARGUMENT", f"tensor content has {td['size']} bytes, expected {need}")
        return memoryview(raw)[td["offset"]:td["offset"] + need], n
    try:
        if td["unpacked"]:
            arr = np.frombuffer(td["unpacked"], dtype=np.float32)
        else:  # typed *_val that needs protobuf decoding (e.g. packed varint int_val for uint8)
            req = P.PredictRequest.FromString(raw)
            arr = P.tensor_proto_to_np(req.inputs[td["key"]])
    except (ValueError, KeyError, TypeError) as e:
        raise ServingError("INVALID_ARGUMENT", f"cannot decode input '{sig.input_key}': {e}") from e
    if arr.size != n * IMG * IMG * 3:
        # TF-Serving: "Input to reshape is a tensor with X values, but the requested shape has Y"
        raise ServingError("INVALID_ARGUMENT", f"input '{sig.input_key}' has {arr.size} values, but its "
                           f"shape {dims} needs {n * IMG * IMG * 3}")
    arr = np.ascontiguousarray(arr.reshape(n, IMG, IMG, 3),
                               dtype=np.uint8 if sig.input_dtype == P.DT_UINT8 else np.float32)
    return arr, n


def _image_payload(raw: bytes, td: dict, sig, dims: list) -> tuple[np.ndarray, int]:
    if td["dtype"] != P.DT_UINT8:
        raise ServingError("INVALID_ARGUMENT", f"Expects arg[0] to be uint8 but "
                           f"{P.DTYPE_NAMES.get(td['dtype'], td['dtype'])} is provided")
    if len(dims) != 4 or dims[3] != 3 or min(dims[:3]) < 1:
        raise ServingError("INVALID_ARGUMENT", f"input '{sig.input_key}' must have shape [-1,-1,-1,3], got {dims}")
    n, H, W = dims[:3]
    need = n * H * W * 3
    if td["has_content"]:
        if td["size"] != need:
            raise ServingError("INVALID_ARGUMENT", f"tensor content has {td['size']} bytes, expected {need}")
        arr = np.frombuffer(raw, dtype=np.uint8, count=need, offset=td["offset"])
    else:
        try:
            arr = P.tensor_proto_to_np(P.PredictRequest.FromString(raw).inputs[td["key"]]).astype(np.uint8)
        except (ValueError, KeyError, TypeError) as e:
            raise ServingError("INVALID_ARGUMENT", f"cannot decode input '{sig.input_key}': {e}") from e
        if arr.size != need:
            raise ServingError("INVALID_ARGUMENT", f"input '{sig.input_key}' has {arr.size} values, but its "
                               f"shape {dims} needs {need}")
    return arr.reshape(n, H, W, 3), n


def route_exact_u8(s, runner, buf, n: int):
    """The reference gateway's f32 request is exactly x / 127.5 - 1 of 8-bit pixels
    (keras_image_helper's Xception preprocessing, /root/reference/model_server.py:18,53): serve
    it on the uint8 signature (4x fewer bytes to stage and copy; the same logits up to the stem's
    rounding of bf16(x) vs u8) -- and, under ``--scatter rccl``, data parallel over the node,
    since that is the signature the DP group serves. Shared by gRPC and REST. Returns
    (runner, payload): unchanged when the signature or the values do not qualify."""
    sig = runner.sig
    if sig.input_dtype != P.DT_FLOAT or sig.input_shape[1] <= 0 or NATIVE_SIGNATURE not in s.signatures:
        return runner, buf
    u8 = np.empty(n * sig.input_shape[1] * sig.input_shape[2] * 3, dtype=np.uint8)
    if not _lib.rt().f32_to_u8_exact(buf, u8):
        return runner, buf
    METRICS.inc("kdl_f32_as_uint8_total")
    return s.runner(NATIVE_SIGNATURE), u8


class Servicer:
    def __init__(self, manager: ModelManager, f32_exact_u8: bool = True):
        self.m = manager
        self.f32_exact_u8 = f32_exact_u8

    # ---------------------------------------------------------------- Predict
    def predict(self, raw: bytes, context) -> bytes:
        t0 = time.perf_counter()
        rt = _lib.rt()
        try:
            try:
                req = rt.parse_predict_request(raw)
            except ValueError as e:
                raise ServingError("INVALID_ARGUMENT", f"malformed PredictRequest: {e}") from e
            spec = req["model_spec"]
            version = spec["version"] if spec["version"] >= 0 else None
            s = self.m.get(spec["name"], version, spec["version_label"] or None)
            sig_name = spec["signature_name"] or "serving_default"
            runner = s.runner(sig_name)
            sig = runner.sig
            inputs = {td["key"]: td for td in req["inputs"]}
            if sig.input_key not in inputs:
                raise ServingError("INVALID_ARGUMENT", f"input tensor alias not found in signature: "
                                   f"{', '.join(inputs) or '<none>'}. Inputs expected to be in the set "
                                   f"{{{sig.input_key}}}.")
            if len(inputs) != 1:
                raise ServingError("INVALID_ARGUMENT", f"expected exactly one input ({sig.input_key})")
            for f in req["output_filter"]:
                if f != sig.output_key:
                    raise ServingError("INVALID_ARGUMENT", f"output tensor alias not found in signature: {f}")
            buf, n = _payload(raw, inputs[sig.input_key], sig)
            if self.f32_exact_u8:
                runner, buf = route_exact_u8(s, runner, buf, n)
            t1 = time.perf_counter()
            logits = runner.predict(buf, n, _deadline_us(context))
            t2 = time.perf_counter()
            out = rt.build_predict_response([(sig.output_key, logits)], s.name, s.version, sig_name)
            # per-request stage trace (SURVEY.md §5 tracing): parse+validate, batcher wait+run, respond
            METRICS.observe("kdl_stage_ms", (t1 - t0) * 1e3, stage="parse")
            METRICS.observe("kdl_stage_ms", (t2 - t1) * 1e3, stage="batch_and_run")
            METRICS.observe("kdl_stage_ms", (time.perf_counter() - t2) * 1e3, stage="respond")
        except ServingError as e:
            METRICS.inc("kdl_requests_total", code=e.code, method="Predict")
            _abort(context, e)
            return b""
        ms = (time.perf_counter() - t0) * 1e3
        METRICS.inc("kdl_requests_total", code="OK", method="Predict")
        METRICS.observe("kdl_request_latency_ms", ms, method="Predict")
        return out

    # ---------------------------------------------------------------- metadata / status
    def get_model_metadata(self, raw: bytes, context) -> bytes:
        try:
            req = P.GetModelMetadataRequest.FromString(raw)
            if list(req.metadata_field) != ["signature_def"]:
                raise ServingError("INVALID_ARGUMENT", "Metadata field signature_def is the only supported field")
            ver = req.model_spec.version.value if req.model_spec.HasField("version") else None
            s = self.m.get(req.model_spec.name, ver)
            resp = P.GetModelMetadataResponse()
            resp.model_spec.name = s.name
            resp.model_spec.version.value = s.version
            resp.metadata["signature_def"].Pack(signature_def_map(s))
            METRICS.inc("kdl_requests_total", code="OK", method="GetModelMetadata")
            return resp.SerializeToString()
        except ServingError as e:
            _abort(context, e)
            return b""

    def get_model_status(self, raw: bytes, context) -> bytes:
        try:
            req = P.GetModelStatusRequest.FromString(raw)
            if req.model_spec.name != self.m.name:
                raise ServingError("NOT_FOUND", f"Could not find any versions of model {req.model_spec.name}")
            ver = req.model_spec.version.value if req.model_spec.HasField("version") else None
            resp = P.GetModelStatusResponse()
            for v, state, msg in self.m.status(ver):
                st = resp.model_version_status.add(version=v, state=state)
                st.status.error_code = 0 if not msg else 13
                st.status.error_message = msg
            return resp.SerializeToString()
        except ServingError as e:
            _abort(context, e)
            return b""

    def reload_config(self, raw: bytes, context) -> bytes:
        try:
            self.m.reload()
            return P.ReloadConfigResponse().SerializeToString()
        except Exception as e:  # noqa: BLE001
            resp = P.ReloadConfigResponse()
            resp.status.error_code = 13
            resp.status.error_message = str(e)
            return resp.SerializeToString()

    def unimplemented(self, raw: bytes, context) -> bytes:
        context.abort(grpc.StatusCode.UNIMPLEMENTED,
                      "only Predict is supported for tensorflow/serving/predict signatures")
        return b""

    # ---------------------------------------------------------------- grpc.health.v1
    def health_check(self, raw: bytes, context) -> bytes:
        # HealthCheckResponse{status=1 SERVING | 2 NOT_SERVING}; the serving process's pid rides in
        # the initial metadata (which of a node's SO_REUSEPORT processes answered: --procs)
        if context is not None:
            context.send_initial_metadata((("kdl-pid", str(os.getpid())),))
        return b"\x08\x01" if self.m.ready() else b"\x08\x02"


def signature_def_map(s) -> "P.SignatureDefMap":
    m = P.SignatureDefMap()
    for name, sig in s.signatures.items():
        sd = m.signature_def[name]
        sd.method_name = sig.method_name
        ti = sd.inputs[sig.input_key]
        ti.name = f"{name}_{sig.input_key}:0"
        ti.dtype = sig.input_dtype
        for d in sig.input_shape:
            ti.tensor_shape.dim.add(size=d)
        to = sd.outputs[sig.output_key]
        to.name = "StatefulPartitionedCall:0"
        to.dtype = P.DT_FLOAT
        for d in sig.output_shape:
            to.tensor_shape.dim.add(size=d)
    return m


def build_grpc_server(manager: ModelManager, host: str, port: int, max_workers: int = 64, reuse_port: bool = False,
                      f32_exact_u8: bool = True, max_request_bytes: int = 64 << 20):
    sv = Servicer(manager, f32_exact_u8)
    raw = dict(request_deserializer=None, response_serializer=None)
    pred = grpc.method_handlers_generic_handler("tensorflow.serving.PredictionService", {
        "Predict": grpc.unary_unary_rpc_method_handler(sv.predict, **raw),
        "GetModelMetadata": grpc.unary_unary_rpc_method_handler(sv.get_model_metadata, **raw),
        "Classify": grpc.unary_unary_rpc_method_handler(sv.unimplemented, **raw),
        "Regress": grpc.unary_unary_rpc_method_handler(sv.unimplemented, **raw),
        "MultiInference": grpc.unary_unary_rpc_method_handler(sv.unimplemented, **raw),
    })
    model = grpc.method_handlers_generic_handler("tensorflow.serving.ModelService", {
        "GetModelStatus": grpc.unary_unary_rpc_method_handler(sv.get_model_status, **raw),
        "HandleReloadConfigRequest": grpc.unary_unary_rpc_method_handler(sv.reload_config, **raw),
    })
    health = grpc.method_handlers_generic_handler("grpc.health.v1.Health", {
        "Check": grpc.unary_unary_rpc_method_handler(sv.health_check, **raw),
    })
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                         options=[("grpc.max_receive_message_length", int(max_request_bytes)),
                                  ("grpc.max_send_message_length", -1),
                                  # --procs: every per-GPU process of the node binds the same port
                                  ("grpc.so_reuseport", 1 if reuse_port else 0)])
    server.add_generic_rpc_handlers((pred, model, health))
    bound = server.add_insecure_port(f"{host}:{port}")
    return server, bound, sv
