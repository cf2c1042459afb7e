"""End-to-end serving on CPU ("config #1: plumbing, no GPU").

A real gRPC server on 127.0.0.1 (ephemeral port) with a SavedModel fixture in a
versioned repo, queried by a client that builds requests exactly like the
reference gateway (`model_server.py:38-55`); the Flask gateway is exercised
with an image served by a local http.server (stand-in for bit.ly).
"""
import http.server
import json
import threading
import urllib.request
from pathlib import Path

import grpc
import numpy as np
import pytest
import torch

from kdl.gateway import preprocess as pp
from kdl.gateway.app import GatewayConfig, create_app
from kdl.gateway.client import ModelStub, PredictionStub, make_request, process_response
from kdl.ingest.keras_map import to_keras_variables
from kdl.ingest.savedmodel import write_savedmodel
from kdl.models import xception as X
from kdl.serving import protos as P
from kdl.serving.config import BatchingParams, ServerConfig
from kdl.serving.server import ModelServer

pytest.importorskip("kdl._rt")
DATA = Path(__file__).parent / "data"


@pytest.fixture(scope="module")
def params():
    return X.init_params(seed=5)


@pytest.fixture(scope="module")
def server(tmp_path_factory, params):
    repo = tmp_path_factory.mktemp("models") / "clothing-model"
    write_savedmodel(repo / "1", to_keras_variables(params, residual_offset=2))
    import socket
    with socket.socket() as so:          # rest_api_port=0 means "disabled" (TF-Serving)
        so.bind(("127.0.0.1", 0))
        rest_port = so.getsockname()[1]
    cfg = ServerConfig(port=0, rest_api_port=rest_port, model_name="clothing-model", model_base_path=str(repo),
                       device="cpu", host="127.0.0.1", file_system_poll_wait_seconds=0,
                       batching=BatchingParams(max_batch_size=4, batch_timeout_micros=2000,
                                               allowed_batch_sizes=[1, 2, 4]))
    srv = ModelServer(cfg).start(block_until_loaded=True)
    yield srv
    srv.stop(0)


@pytest.fixture(scope="module")
def channel(server):
    ch = grpc.insecure_channel(f"127.0.0.1:{server.grpc_port}")
    yield ch
    ch.close()


@pytest.fixture(scope="module")
def image_server():
    class H(http.server.SimpleHTTPRequestHandler):
        def __init__(self, *a, **k):
            super().__init__(*a, directory=str(DATA), **k)

        def log_message(self, *a):
            pass
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    yield f"http://127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()


def test_reference_style_predict(channel, params):
    img = pp.load_image((DATA / "pants.png").read_bytes())
    X_ = pp.image_to_tensor(img)                                   # f32 [1,299,299,3]
    stub = PredictionStub(channel)
    res = stub.Predict(make_request(X_), timeout=20.0)             # model_server.py:55
    got = process_response(res, X.LABELS)
    assert list(got) == X.LABELS
    ref = X.xception_forward(params, torch.from_numpy(X_))[0]
    assert np.allclose([got[k] for k in X.LABELS], ref.numpy(), atol=1e-3)


def test_batched_request_and_native_uint8_signature(channel, params):
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, (3, 299, 299, 3), dtype=np.uint8)
    stub = PredictionStub(channel)
    r1 = stub.Predict(make_request(pp.xception_preprocess(u8)), timeout=20.0)
    r2 = stub.Predict(make_request(u8, signature="serving_uint8", input_key="images"), timeout=20.0)
    a = np.asarray(r1.outputs["dense_7"].float_val).reshape(3, 10)
    b = np.asarray(r2.outputs["dense_7"].float_val).reshape(3, 10)
    assert np.allclose(a, b, atol=1e-4)
    ref = X.xception_forward(params, torch.from_numpy(pp.xception_preprocess(u8)))
    assert np.allclose(a, ref.numpy(), atol=1e-3)


def test_errors_map_to_grpc_codes(channel):
    stub = PredictionStub(channel)
    x = np.zeros((1, 299, 299, 3), np.float32)
    with pytest.raises(grpc.RpcError) as e:
        stub.Predict(make_request(x, model_name="nope"), timeout=5)
    assert e.value.code() == grpc.StatusCode.NOT_FOUND
    with pytest.raises(grpc.RpcError) as e:
        stub.Predict(make_request(x, input_key="wrong"), timeout=5)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    with pytest.raises(grpc.RpcError) as e:
        stub.Predict(make_request(np.zeros((1, 32, 32, 3), np.float32)), timeout=5)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    with pytest.raises(grpc.RpcError) as e:
        stub.Predict(make_request(x, signature="nope"), timeout=5)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    # typed float_val whose value count does not match the declared shape (neither
    # the full count nor a single broadcast value) -> INVALID_ARGUMENT, not UNKNOWN
    bad = P.PredictRequest()
    bad.model_spec.name = "clothing-model"
    t = bad.inputs["input_8"]
    t.dtype = P.DT_FLOAT
    for d in (1, 299, 299, 3):
        t.tensor_shape.dim.add(size=d)
    t.float_val.extend([0.5] * 7)
    with pytest.raises(grpc.RpcError) as e:
        stub.Predict(bad, timeout=5)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    req = make_request(x)
    req.model_spec.version.value = 42
    with pytest.raises(grpc.RpcError) as e:
        stub.Predict(req, timeout=5)
    assert e.value.code() == grpc.StatusCode.NOT_FOUND


def test_metadata_status_health(channel):
    stub = PredictionStub(channel)
    req = P.GetModelMetadataRequest()
    req.model_spec.name = "clothing-model"
    req.metadata_field.append("signature_def")
    resp = stub.GetModelMetadata(req, timeout=5)
    sdm = P.SignatureDefMap()
    resp.metadata["signature_def"].Unpack(sdm)
    sd = sdm.signature_def["serving_default"]
    assert list(sd.inputs) == ["input_8"] and list(sd.outputs) == ["dense_7"]
    assert [d.size for d in sd.inputs["input_8"].tensor_shape.dim] == [-1, 299, 299, 3]
    st = ModelStub(channel).GetModelStatus(P.GetModelStatusRequest(model_spec=P.ModelSpec(name="clothing-model")),
                                          timeout=5)
    assert [(s.version, s.state) for s in st.model_version_status] == [(1, 30)]  # AVAILABLE
    health = channel.unary_unary("/grpc.health.v1.Health/Check")(b"", timeout=5)
    assert health == b"\x08\x01"


def test_rest_api(server):
    base = f"http://127.0.0.1:{server.rest_port}"
    st = json.load(urllib.request.urlopen(f"{base}/v1/models/clothing-model"))
    assert st["model_version_status"][0]["state"] == "AVAILABLE"
    md = json.load(urllib.request.urlopen(f"{base}/v1/models/clothing-model/metadata"))
    assert "serving_default" in md["metadata"]["signature_def"]["signatureDef"]
    x = np.zeros((1, 299, 299, 3), np.float32).tolist()
    req = urllib.request.Request(f"{base}/v1/models/clothing-model:predict",
                                 data=json.dumps({"instances": x}).encode(), method="POST")
    out = json.load(urllib.request.urlopen(req))
    assert len(out["predictions"]) == 1 and len(out["predictions"][0]) == 10
    text = urllib.request.urlopen(f"{base}/monitoring/prometheus/metrics").read().decode()
    assert "kdl_requests_total" in text
    for stage in ("parse", "queue_wait", "batch_and_run", "respond"):   # per-request stage trace
        assert f'stage="{stage}"' in text, stage
    assert urllib.request.urlopen(f"{base}/readyz").status == 200


def test_gateway_predict(server, image_server, params):
    cfg = GatewayConfig({"TF_SERVING_HOST": f"127.0.0.1:{server.grpc_port}"})
    app = create_app(cfg)
    c = app.test_client()
    r = c.post("/predict", json={"url": f"{image_server}/pants.png"})
    assert r.status_code == 200, r.data
    got = r.get_json()
    assert set(got) == set(X.LABELS)
    img = pp.load_image((DATA / "pants.png").read_bytes())
    ref = X.xception_forward(params, torch.from_numpy(pp.image_to_tensor(img)))[0]
    assert np.allclose([got[k] for k in X.LABELS], ref.numpy(), atol=1e-3)
    # error handling the reference lacks
    assert c.post("/predict", json={"nourl": 1}).status_code == 400
    assert c.post("/predict", json={"url": f"{image_server}/missing.png"}).status_code == 502
    rb = c.post("/predict_batch", json={"urls": [f"{image_server}/pants.png"] * 2})
    assert rb.status_code == 200 and len(rb.get_json()) == 2


def test_gateway_uint8_mode_matches_compat(server, image_server):
    base = {"TF_SERVING_HOST": f"127.0.0.1:{server.grpc_port}"}
    a = create_app(GatewayConfig(base)).test_client().post("/predict", json={"url": f"{image_server}/pants.png"})
    b = create_app(GatewayConfig({**base, "GATEWAY_MODE": "uint8"})).test_client().post(
        "/predict", json={"url": f"{image_server}/pants.png"})
    ga, gb = a.get_json(), b.get_json()
    assert all(abs(ga[k] - gb[k]) < 1e-3 for k in ga)


def test_gateway_raw_mode_resizes_on_the_server(server, image_server):
    """GATEWAY_MODE=raw ships the decoded pixels at their own size to serving_image; the server's
    resize (PIL NEAREST tables) makes it exactly the uint8 mode's prediction."""
    base = {"TF_SERVING_HOST": f"127.0.0.1:{server.grpc_port}"}
    a = create_app(GatewayConfig({**base, "GATEWAY_MODE": "uint8"})).test_client().post(
        "/predict", json={"url": f"{image_server}/pants.png"})
    b = create_app(GatewayConfig({**base, "GATEWAY_MODE": "raw"})).test_client().post(
        "/predict", json={"url": f"{image_server}/pants.png"})
    assert a.status_code == b.status_code == 200, b.data
    assert a.get_json() == b.get_json()
    with pytest.raises(ValueError):
        GatewayConfig({**base, "GATEWAY_MODE": "bogus"})


@pytest.mark.parametrize("shape", [(1, 534, 400), (2, 1, 1), (1, 2200, 300), (1, 299, 299)])
def test_serving_image_any_size_equals_pil_resize(channel, shape):
    n, H, W = shape
    rng = np.random.default_rng(H * 7 + W)
    raw = rng.integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    from PIL import Image
    pil = np.stack([np.asarray(Image.fromarray(im).resize((299, 299), Image.NEAREST)) for im in raw])
    stub = PredictionStub(channel)
    r1 = stub.Predict(make_request(raw, signature="serving_image", input_key="images"), timeout=30.0)
    r2 = stub.Predict(make_request(pil, signature="serving_uint8", input_key="images"), timeout=30.0)
    a = np.asarray(r1.outputs["dense_7"].float_val)
    assert a.size == n * 10 and np.array_equal(a, np.asarray(r2.outputs["dense_7"].float_val))


def test_serving_image_rejects_bad_shapes(channel):
    stub = PredictionStub(channel)
    for bad in (np.zeros((1, 5, 5, 4), np.uint8), np.zeros((1, 5, 5, 3), np.float32)):
        with pytest.raises(grpc.RpcError) as e:
            stub.Predict(make_request(bad, signature="serving_image", input_key="images"), timeout=5)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_deadline_exceeded(channel):
    stub = PredictionStub(channel)
    x = np.zeros((4, 299, 299, 3), np.float32)
    with pytest.raises(grpc.RpcError) as e:
        stub.Predict(make_request(x), timeout=0.001)
    assert e.value.code() == grpc.StatusCode.DEADLINE_EXCEEDED


def test_reference_f32_request_rides_the_uint8_path(channel, server):
    """The reference gateway's f32 request (x / 127.5 - 1 of 8-bit pixels, model_server.py:36-42) is
    recognised as exact 8-bit pixels and served by the serving_uint8 runner: same logits as sending
    the pixels, the f32 runner not involved; a non-pixel f32 request keeps the f32 path."""
    from kdl.serving.metrics import METRICS
    stub = PredictionStub(channel)
    u8 = np.random.default_rng(9).integers(0, 256, (2, 299, 299, 3), dtype=np.uint8)
    key = "kdl_f32_as_uint8_total"
    n0 = METRICS.snapshot()["counters"].get(key, 0)
    r1 = stub.Predict(make_request(u8.astype(np.float32) / 127.5 - 1), timeout=20.0)
    r2 = stub.Predict(make_request(u8, signature="serving_uint8", input_key="images"), timeout=20.0)
    a1 = np.asarray(r1.outputs["dense_7"].float_val, np.float32)
    assert np.array_equal(a1, np.asarray(r2.outputs["dense_7"].float_val, np.float32))
    assert METRICS.snapshot()["counters"].get(key, 0) == n0 + 1
    x = u8.astype(np.float32) / 127.5 - 1 + 1e-3          # not pixels: f32 path
    stub.Predict(make_request(x), timeout=20.0)
    assert METRICS.snapshot()["counters"].get(key, 0) == n0 + 1
