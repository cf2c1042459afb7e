"""Native gRPC front-end (kdl._rt.GrpcFront, csrc/runtime/grpc_front.h; serving/native_front.py).

The same model repo is served twice, by the native front-end and by the grpcio one, on the
zero-latency null device (logits = first input byte + class index): responses must be byte
for byte the same, every error the same (code, message), and after the first Predict of a
signature the native one must serve it on its fast path (no Python per request). Also: the
grpc-timeout deadline on the fast path, routes dropped on a version change, a stop with calls
in flight, and the native load generator (tools/serve_bench.py --client native).
Reference surface: /root/reference/model_server.py:15-16,38-55 (PredictionServiceStub.Predict).
"""
import time

import grpc
import numpy as np
import pytest

from kdl.gateway.client import make_request
from kdl.serving import protos as P
from kdl.serving.config import BatchingParams, ServerConfig
from kdl.serving.server import ModelServer

rt = pytest.importorskip("kdl._rt")
pytestmark = pytest.mark.skipif(not rt.http2_available()[0], reason="libnghttp2 not loadable")

PREDICT = "/tensorflow.serving.PredictionService/Predict"


def _repo(tmp_path, versions=(1,)):
    base = tmp_path / "clothing-model"
    for v in versions:
        (base / str(v)).mkdir(parents=True)
        (base / str(v) / "synthetic.json").write_text('{"seed": 0}')
    return base


def _server(base, frontend, **kw):
    cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=str(base), device="null", host="127.0.0.1",
                       file_system_poll_wait_seconds=kw.pop("poll", 0), grpc_frontend=frontend, grpc_io_threads=2,
                       batching=BatchingParams(max_batch_size=8, batch_timeout_micros=500,
                                               allowed_batch_sizes=[1, 2, 4, 8]), **kw)
    return ModelServer(cfg).start(block_until_loaded=True)


@pytest.fixture(scope="module")
def pair(tmp_path_factory):
    base = _repo(tmp_path_factory.mktemp("front"))
    nat, py = _server(base, "native"), _server(base, "python")
    assert nat.native is not None and py.native is None
    yield nat, py
    nat.stop(0)
    py.stop(0)


def _call(port, path, req: bytes, timeout=10.0):
    with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
        try:
            return 0, "", ch.unary_unary(path)(req, timeout=timeout)
        except grpc.RpcError as e:
            return e.code().value[0], e.details(), b""


def _u8_req(n=2, seed=0, **kw):
    u8 = np.random.default_rng(seed).integers(0, 256, (n, 299, 299, 3), dtype=np.uint8)
    return make_request(u8, signature="serving_uint8", input_key="images", **kw).SerializeToString(), u8


def test_fast_path_engages_and_answers_byte_for_byte_like_grpcio(pair):
    nat, py = pair
    s0 = nat.native.stats()
    for seed in range(4):
        req, u8 = _u8_req(n=1 + seed % 3, seed=seed)
        a, b = _call(nat.grpc_port, PREDICT, req), _call(py.grpc_port, PREDICT, req)
        assert a[0] == 0 and a == b
        out = np.asarray(P.PredictResponse.FromString(a[2]).outputs["dense_7"].float_val).reshape(-1, 10)
        assert np.array_equal(out, u8.reshape(len(u8), -1)[:, :1] + np.arange(10))   # null device rows
    s1 = nat.native.stats()
    assert s1["slow"] - s0["slow"] <= 1 and s1["fast_ok"] - s0["fast_ok"] >= 3   # learned after one request
    # the reference gateway's f32 request: fast path, exact-u8 rule, same bytes as grpcio
    u8 = np.random.default_rng(7).integers(0, 256, (1, 299, 299, 3), dtype=np.uint8)
    req = make_request(u8.astype(np.float32) / 127.5 - 1).SerializeToString()
    for _ in range(2):
        a, b = _call(nat.grpc_port, PREDICT, req), _call(py.grpc_port, PREDICT, req)
        assert a[0] == 0 and a == b
    assert nat.native.stats()["exact_u8"] >= 1


def _bad_requests():
    x = np.zeros((1, 299, 299, 3), np.float32)
    yield "unknown model", make_request(x, model_name="nope")
    yield "wrong input key", make_request(x, input_key="wrong")
    yield "wrong size", make_request(np.zeros((1, 32, 32, 3), np.float32))
    yield "unknown signature", make_request(x, signature="nope")
    yield "dtype mismatch", make_request(x, signature="serving_uint8", input_key="images")
    r = make_request(x)
    r.model_spec.version.value = 42
    yield "missing version", r
    bad = P.PredictRequest()
    bad.model_spec.name = "clothing-model"
    t = bad.inputs["input_8"]
    t.dtype = P.DT_FLOAT
    for d in (1, 299, 299, 3):
        t.tensor_shape.dim.add(size=d)
    t.float_val.extend([0.5] * 7)
    yield "value count", bad
    r = make_request(x)
    r.output_filter.append("nope")
    yield "output filter", r


@pytest.mark.parametrize("name,req", list(_bad_requests()), ids=[n for n, _ in _bad_requests()])
def test_errors_match_grpcio(pair, name, req):
    nat, py = pair
    raw = req.SerializeToString()
    _call(nat.grpc_port, PREDICT, _u8_req()[0])        # routes learned: the fast path must still refuse these
    a, b = _call(nat.grpc_port, PREDICT, raw), _call(py.grpc_port, PREDICT, raw)
    assert a[0] != 0 and a == b, name


def test_other_methods_and_unknown_method_match_grpcio(pair):
    nat, py = pair
    md = P.GetModelMetadataRequest()
    md.model_spec.name = "clothing-model"
    md.metadata_field.append("signature_def")
    st = P.GetModelStatusRequest(model_spec=P.ModelSpec(name="clothing-model"))
    for path, req in (("/tensorflow.serving.PredictionService/GetModelMetadata", md.SerializeToString()),
                      ("/tensorflow.serving.ModelService/GetModelStatus", st.SerializeToString()),
                      ("/tensorflow.serving.PredictionService/Classify", b""),
                      ("/grpc.health.v1.Health/Check", b""),
                      ("/no.such.Service/Method", b"")):
        assert _call(nat.grpc_port, path, req) == _call(py.grpc_port, path, req), path
    with grpc.insecure_channel(f"127.0.0.1:{nat.grpc_port}") as ch:   # the answering process in metadata
        _, call = ch.unary_unary("/grpc.health.v1.Health/Check").with_call(b"", timeout=5)
        assert "kdl-pid" in dict(call.initial_metadata())


def test_a_label_takes_the_slow_path_the_live_version_pinned_does_not(pair):
    nat, _ = pair
    req, _ = _u8_req(n=1)
    _call(nat.grpc_port, PREDICT, req)
    s0 = nat.native.stats()
    r = P.PredictRequest.FromString(req)
    r.model_spec.version.value = 1
    assert _call(nat.grpc_port, PREDICT, r.SerializeToString())[0] == 0
    r = P.PredictRequest.FromString(req)
    r.model_spec.version_label = "stable"
    assert _call(nat.grpc_port, PREDICT, r.SerializeToString())[0] == 0
    st = nat.native.stats()
    assert st["slow"] == s0["slow"] + 1 and st["fast_ok"] == s0["fast_ok"] + 1


def test_prometheus_counts_fast_path_requests(pair):
    from kdl.serving.metrics import METRICS
    nat, _ = pair
    req, _ = _u8_req(n=1)
    _call(nat.grpc_port, PREDICT, req)
    k = "kdl_requests_total{code=OK,method=Predict}"
    n0 = METRICS.snapshot()["counters"].get(k, 0)
    for _ in range(5):
        _call(nat.grpc_port, PREDICT, req)
    assert METRICS.snapshot()["counters"].get(k, 0) >= n0 + 5
    assert 'kdl_request_latency_ms_bucket{method="Predict",le="+Inf"}' in METRICS.render()


def test_fast_path_deadline_expires_in_the_batcher(tmp_path, monkeypatch):
    """A fast-path request queued behind a busy executor past its grpc-timeout is dropped by the
    batcher (submit_async's ST_DEADLINE callback), never run."""
    import threading
    monkeypatch.setenv("KDL_FAULT_INJECT", "delay=null:300")       # every batch holds the executor 300 ms
    srv = _server(_repo(tmp_path), "native")
    try:
        req, _ = _u8_req(n=1)
        assert _call(srv.grpc_port, PREDICT, req)[0] == 0          # slow path, learns the route
        batcher = srv.manager.get("clothing-model").runner("serving_uint8").batcher
        e0, f0 = batcher.stats()["expired"], srv.native.stats()["fast_ok"]
        n0 = batcher.stats()["submitted"]
        busy = threading.Thread(target=_call, args=(srv.grpc_port, PREDICT, req))
        busy.start()
        t_end = time.time() + 10
        while batcher.stats()["submitted"] == n0 and time.time() < t_end:   # the busy call holds the executor
            time.sleep(0.005)
        time.sleep(0.02)
        code, _, _ = _call(srv.grpc_port, PREDICT, req, timeout=0.1)
        assert code == grpc.StatusCode.DEADLINE_EXCEEDED.value[0]
        busy.join(10)
        t_end = time.time() + 5
        while batcher.stats()["expired"] == e0 and time.time() < t_end:
            time.sleep(0.05)
        assert batcher.stats()["expired"] == e0 + 1
        assert srv.native.stats()["fast_ok"] == f0 + 1             # the busy call, on the fast path
    finally:
        srv.stop(0)


def test_version_change_drops_routes(tmp_path):
    base = _repo(tmp_path)
    srv = _server(base, "native", poll=1)
    try:
        req, _ = _u8_req(n=1)
        for _ in range(2):
            code, _, out = _call(srv.grpc_port, PREDICT, req)
            assert code == 0 and P.PredictResponse.FromString(out).model_spec.version.value == 1
        (base / "2").mkdir()
        (base / "2" / "synthetic.json").write_text('{"seed": 0}')
        t_end = time.time() + 60
        while time.time() < t_end:
            code, _, out = _call(srv.grpc_port, PREDICT, req)
            if code == 0 and P.PredictResponse.FromString(out).model_spec.version.value == 2:
                break
            time.sleep(0.2)
        else:
            raise AssertionError("version 2 never answered")
        s0 = srv.native.stats()
        for _ in range(3):
            code, _, out = _call(srv.grpc_port, PREDICT, req)
            assert code == 0 and P.PredictResponse.FromString(out).model_spec.version.value == 2
        assert srv.native.stats()["fast_ok"] >= s0["fast_ok"] + 2        # re-learned for version 2
    finally:
        srv.stop(0)


def test_native_load_generator_and_stop_with_calls_in_flight(tmp_path, monkeypatch):
    monkeypatch.setenv("KDL_FAULT_INJECT", "delay=null:20")
    srv = _server(_repo(tmp_path), "native")
    req, _ = _u8_req(n=1)
    assert _call(srv.grpc_port, PREDICT, req)[0] == 0
    r = rt.grpc_load("127.0.0.1", srv.grpc_port, PREDICT, req, conns=2, streams=4, seconds=1.0, warm_s=0.2)
    assert r["error"] == "" and r["failed"] == 0 and r["ok"] > 10 and set(r["codes"]) == {0}
    import threading
    th = threading.Thread(target=rt.grpc_load, args=("127.0.0.1", srv.grpc_port, PREDICT, req),
                          kwargs=dict(conns=2, streams=8, seconds=3.0, warm_s=0.0, timeout_s=5.0))
    th.start()
    time.sleep(0.5)
    srv.stop(0)                                   # calls in flight in the batcher: dropped, no crash
    th.join(30)
    assert not th.is_alive()


def test_connections_spread_over_the_io_workers(tmp_path):
    """One process, K epoll workers each with its own SO_REUSEPORT listener: the kernel spreads
    connections over them (VERDICT r4 item 7's several-ingress goal, as threads of one process
    feeding the same C++ batcher instead of K processes and a shared-memory ring)."""
    base = _repo(tmp_path)
    cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=str(base), device="null", host="127.0.0.1",
                       file_system_poll_wait_seconds=0, grpc_frontend="native", grpc_io_threads=2)
    srv = ModelServer(cfg).start(block_until_loaded=True)
    try:
        req, _ = _u8_req(n=1)
        r = rt.grpc_load("127.0.0.1", srv.grpc_port, PREDICT, req, conns=16, streams=2, seconds=0.5, warm_s=0.1)
        assert r["failed"] == 0 and r["ok"] > 0
        wc = srv.native.stats()["worker_calls"]
        assert len(wc) == 2 and min(wc) > 0, wc
    finally:
        srv.stop(0)


def test_grpc_message_percent_encoding():
    assert rt.grpc_percent_encode("a b%\né") == "a b%25%0A%C3%A9"


def test_oversized_request_resource_exhausted_like_grpcio(tmp_path):
    """Both front-ends cap the request message (--grpc_max_request_bytes):
    a larger one is answered RESOURCE_EXHAUSTED with grpcio's wording, and a request within the
    cap still works. A prefix that lies about its length is covered at the C++ level
    (csrc/tests/front_stress.cpp oversize phase, under TSAN and ASan in test_sanitizers.py)."""
    base = _repo(tmp_path)
    cap = 1 << 20
    nat = _server(base, "native", grpc_max_request_bytes=cap)
    py = _server(base, "python", grpc_max_request_bytes=cap)
    try:
        big = make_request(np.zeros((4, 299, 299, 3), np.float32)).SerializeToString()   # 4.3 MB > 1 MiB
        a, b = _call(nat.grpc_port, PREDICT, big), _call(py.grpc_port, PREDICT, big)
        assert a[0] == b[0] == grpc.StatusCode.RESOURCE_EXHAUSTED.value[0], (a[:2], b[:2])
        assert a[1] == b[1], (a[1], b[1])
        small = _u8_req(n=1)[0]                                                        # 268 KB
        a, b = _call(nat.grpc_port, PREDICT, small), _call(py.grpc_port, PREDICT, small)
        assert a[0] == 0 and a == b
        # the native load generator with a raw prefix announcing 2 GiB - 1: refused, nothing buffered
        liar = b"\0\x7f\xff\xff\xff" + b"x" * 4096
        r = rt.grpc_load("127.0.0.1", nat.grpc_port, PREDICT, liar, conns=2, streams=64, seconds=0.5,
                         warm_s=0.0, timeout_s=10.0, raw_frame=True)
        assert r["error"] == "" and set(r["codes"]) == {8} and r["failed"] > 0, r
    finally:
        nat.stop(0)
        py.stop(0)


def test_second_server_on_the_port_fails_unless_shared(tmp_path):
    """Outside --procs (gpu_index < 0) the native front-end must not silently share a port that
    another server holds (advisor r5): SO_REUSEPORT stays among its own listeners."""
    base = _repo(tmp_path)
    first = _server(base, "native")
    try:
        with pytest.raises(Exception):
            ModelServer(ServerConfig(port=first.grpc_port, rest_api_port=0, model_base_path=str(base),
                                     device="null", host="127.0.0.1", grpc_frontend="native",
                                     grpc_io_threads=2)).start(block_until_loaded=True)
        # a --procs child shares it on purpose
        shared = rt.GrpcFront("127.0.0.1", first.grpc_port, 1, 1, lambda p, m, d: (12, "x", b"", []),
                              reuse_port=True)
        shared.stop()
    finally:
        first.stop(0)
