"""Reference-compatible TF-Serving gRPC client (`model_server.py:13-56`).

Builds the request exactly like the reference gateway (model_spec name,
signature_name, inputs[<input key>] = make_tensor_proto(X)) and reads
``outputs[<output key>].float_val``, using the runtime-built protos instead of
``tensorflow_serving.apis`` (not installable offline).
"""
from __future__ import annotations

import grpc
import numpy as np

from ..serving import protos as P


class PredictionStub:
    """Equivalent of prediction_service_pb2_grpc.PredictionServiceStub."""

    def __init__(self, channel: grpc.Channel):
        self.Predict = channel.unary_unary(P.PREDICT_METHOD, request_serializer=P.PredictRequest.SerializeToString,
                                           response_deserializer=P.PredictResponse.FromString)
        self.GetModelMetadata = channel.unary_unary(
            P.METADATA_METHOD, request_serializer=P.GetModelMetadataRequest.SerializeToString,
            response_deserializer=P.GetModelMetadataResponse.FromString)


class ModelStub:
    def __init__(self, channel: grpc.Channel):
        self.GetModelStatus = channel.unary_unary(
            P.STATUS_METHOD, request_serializer=P.GetModelStatusRequest.SerializeToString,
            response_deserializer=P.GetModelStatusResponse.FromString)


def np_to_protobuf(data: np.ndarray):
    return P.np_to_tensor_proto(data)


def make_request(X: np.ndarray, model_name="clothing-model", signature="serving_default", input_key="input_8"):
    pb_request = P.PredictRequest()
    pb_request.model_spec.name = model_name
    pb_request.model_spec.signature_name = signature
    pb_request.inputs[input_key].CopyFrom(np_to_protobuf(X))
    return pb_request


def process_response(pb_result, labels, output_key="dense_7") -> dict:
    pred = pb_result.outputs[output_key].float_val
    return {c: p for c, p in zip(labels, pred)}


def process_batch_response(pb_result, labels, output_key="dense_7") -> list[dict]:
    """Batched variant (the reference's process_response only handles batch=1,
    SURVEY.md §8.1)."""
    t = pb_result.outputs[output_key]
    vals = np.asarray(t.float_val, dtype=np.float32).reshape([d.size for d in t.tensor_shape.dim])
    return [{c: float(p) for c, p in zip(labels, row)} for row in vals]
