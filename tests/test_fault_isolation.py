"""Per-device fault isolation + fault injection (SURVEY.md §5 failure detection):
an executor whose batches keep failing is marked unhealthy and leaves the shared
batcher to the healthy ones; readiness drops only when no healthy device is left."""
import grpc
import numpy as np
import pytest

from kdl.gateway.client import PredictionStub, make_request
from kdl.serving.backend import FaultInjector
from kdl.serving.config import BatchingParams, ServerConfig
from kdl.serving.metrics import METRICS
from kdl.serving.server import ModelServer

pytest.importorskip("kdl._rt")


def test_fault_injector_rules():
    f = FaultInjector("fail=gpu1:2,delay=cpu:0")
    f.before_batch("gpu0/serving_default")
    for _ in range(2):
        with pytest.raises(RuntimeError):
            f.before_batch("gpu1/serving_default")
    f.before_batch("gpu1/serving_default")      # budget of 2 failures spent
    with pytest.raises(ValueError):
        FaultInjector("explode=gpu0")


def _server(tmp_path, monkeypatch, spec):
    monkeypatch.setenv("KDL_FAULT_INJECT", spec)
    base = tmp_path / "m"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 0, "model": "resnet50"}')
    cfg = ServerConfig(port=0, rest_api_port=0, model_name="m", model_base_path=str(base), device="cpu",
                       host="127.0.0.1", file_system_poll_wait_seconds=0, executors_per_gpu=2,
                       batching=BatchingParams(max_batch_size=1, batch_timeout_micros=0, allowed_batch_sizes=[1]))
    return ModelServer(cfg).start(block_until_loaded=True)


def test_failing_executor_is_isolated(tmp_path, monkeypatch):
    srv = _server(tmp_path, monkeypatch, "fail=cpu0:-1")
    try:
        stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{srv.grpc_port}"))
        x = np.zeros((1, 224, 224, 3), np.uint8)
        codes = []
        for _ in range(12):
            try:
                stub.Predict(make_request(x, model_name="m", input_key="images"), timeout=60)
                codes.append("OK")
            except grpc.RpcError as e:
                codes.append(e.code().name)
        runner = srv.manager.get("m").runner("serving_default")
        ex = {e.name.split("/")[0]: e for e in runner.executors}
        assert not ex["cpu0"].healthy and ex["cpu1"].healthy
        assert codes.count("INTERNAL") <= 3 and codes[-4:] == ["OK"] * 4
        assert srv.manager.ready()
        assert "kdl_executor_healthy" in METRICS.render()
    finally:
        srv.stop(0)


def test_not_ready_when_every_device_failed(tmp_path, monkeypatch):
    srv = _server(tmp_path, monkeypatch, "fail=cpu:-1")
    try:
        stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{srv.grpc_port}"))
        x = np.zeros((1, 224, 224, 3), np.uint8)
        for _ in range(6):
            with pytest.raises(grpc.RpcError):
                stub.Predict(make_request(x, model_name="m", input_key="images"), timeout=5)
        assert not srv.manager.ready()
        with pytest.raises(grpc.RpcError) as e:     # fails fast instead of waiting for the deadline
            stub.Predict(make_request(x, model_name="m", input_key="images"), timeout=30)
        assert e.value.code() == grpc.StatusCode.UNAVAILABLE
    finally:
        srv.stop(0)


def test_no_deadline_requests_fail_when_last_executor_leaves(tmp_path, monkeypatch):
    """Requests without a deadline (REST without X-Deadline-Ms, gRPC without a timeout)
    that are queued when the last healthy executor leaves must fail, not block forever."""
    import threading

    from kdl.serving.backend import ServingError
    srv = _server(tmp_path, monkeypatch, "fail=cpu:-1,delay=cpu:20")
    try:
        runner = srv.manager.get("m").runner("serving_default")
        x = np.zeros((1, 224, 224, 3), np.uint8)
        codes, lock = [], threading.Lock()

        def call():
            try:
                runner.predict(x, 1, 0)        # deadline 0 = none
                code = "OK"
            except ServingError as e:
                code = e.code
            with lock:
                codes.append(code)

        ths = [threading.Thread(target=call, daemon=True) for _ in range(16)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=60)
        assert not any(t.is_alive() for t in ths), "a no-deadline request hung after every executor failed"
        assert len(codes) == 16 and "OK" not in codes
        assert set(codes) <= {"INTERNAL", "UNAVAILABLE"}
        assert not runner.healthy()
    finally:
        srv.stop(0)
