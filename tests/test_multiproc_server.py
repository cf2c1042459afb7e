"""One server process per GPU (``python -m kdl.serving --procs N``), CPU rehearsal.

Two server processes (null device: the real gRPC front-end, request codec, batcher and
native executor over a zero-latency fake device) bind the same gRPC port through
SO_REUSEPORT; independent client connections are spread over both processes by the
kernel, every Predict answers correctly whichever process took it, and SIGTERM to the
launcher stops the whole group. This is the scale-out that replaces the reference's
Deployment replicas behind a ClusterIP Service (tf-serving-clothing-model-deployment.yaml:8,
tf-serving-clothing-model-service.yaml:1-14) inside one pod.
"""
import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

import grpc
import numpy as np
import pytest

from kdl.gateway.client import PredictionStub, make_request

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _health(target):
    ch = grpc.insecure_channel(target, options=[("grpc.use_local_subchannel_pool", 1)])
    call = ch.unary_unary("/grpc.health.v1.Health/Check")
    try:
        resp, c = call.with_call(b"", timeout=5)
        md = dict(c.initial_metadata())
        return resp, md.get("kdl-pid")
    finally:
        ch.close()


@pytest.fixture()
def two_procs(tmp_path):
    base = tmp_path / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 0}')
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    # space-separated "--procs 2", the form README / docs/guide.md document (the
    # launcher used to forward the stray "2" to every child, which then refused its argv)
    p = subprocess.Popen([sys.executable, "-m", "kdl.serving", "--procs", "2", f"--port={port}", "--rest_api_port=0",
                          f"--model_base_path={base}", "--device=null", "--host=127.0.0.1",
                          "--allowed_batch_sizes=1,2,4,8"], cwd=str(ROOT), env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)
    target = f"127.0.0.1:{port}"
    try:
        deadline = time.time() + 240
        pids = set()
        while time.time() < deadline and len(pids) < 2:     # both processes up and SERVING
            try:
                resp, pid = _health(target)
                if resp == b"\x08\x01":
                    pids.add(pid)
            except grpc.RpcError:
                pass
            time.sleep(0.2)
        assert p.poll() is None, "launcher exited"
        yield p, target
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)


def test_connections_spread_over_both_processes_and_predict_is_right(two_procs):
    p, target = two_procs
    pids = {_health(target)[1] for _ in range(40)}
    assert len(pids) == 2, pids
    rng = np.random.default_rng(0)
    for k in range(12):
        ch = grpc.insecure_channel(target, options=[("grpc.use_local_subchannel_pool", 1),
                                                    ("grpc.max_send_message_length", -1)])
        u8 = rng.integers(0, 200, (3, 299, 299, 3), dtype=np.uint8)
        r = PredictionStub(ch).Predict(make_request(u8, signature="serving_uint8", input_key="images"), timeout=30)
        got = np.asarray(r.outputs["dense_7"].float_val, np.float32).reshape(3, 10)
        # the null device answers {first byte of the image + class index}
        want = u8[:, 0, 0, 0:1].astype(np.float32) + np.arange(10, dtype=np.float32)[None]
        assert np.array_equal(got, want)
        ch.close()


def test_sigterm_stops_every_process(two_procs):
    p, target = two_procs
    os.kill(p.pid, signal.SIGTERM)
    assert p.wait(timeout=60) == 0
    with pytest.raises(grpc.RpcError):
        _health(target)


# ---------------------------------------------------------------- per-GPU fault isolation
def test_supervisor_replaces_a_dead_slot_and_gives_up_on_a_crash_loop():
    """ProcsSupervisor with stub children: slot 1 dies -> a FRESH process replaces it (slot 0
    untouched); a slot that dies every time trips the crash-loop limit -> the launcher exits."""
    from kdl.serving.server import ProcsSupervisor
    spawned = []

    def cmd_for(i, restarts):
        spawned.append((i, restarts))
        code = "import time; time.sleep(30)" if (i == 0 or restarts > 0) else "raise SystemExit(4)"
        return [sys.executable, "-c", code], dict(os.environ)
    sup = ProcsSupervisor(cmd_for, 2, max_restarts=3, window_s=60, backoff_s=0.05)
    sup.spawn(0)
    sup.spawn(1)
    first0 = sup.kids[0].pid
    t0 = time.monotonic()
    while time.monotonic() - t0 < 20 and (1, 1) not in spawned:
        assert sup.step(time.monotonic()) is None
        time.sleep(0.05)
    assert (1, 1) in spawned and sup.kids[0].pid == first0 and sup.kids[0].poll() is None
    assert sup.kids[1].poll() is None                   # the replacement serves
    for k in sup.kids:
        k.kill()
        k.wait()

    def always_dies(i, restarts):
        return [sys.executable, "-c", "raise SystemExit(4)"], dict(os.environ)
    sup = ProcsSupervisor(always_dies, 1, max_restarts=2, window_s=60, backoff_s=0.01)
    sup.spawn(0)
    t0, rc = time.monotonic(), None
    while rc is None and time.monotonic() - t0 < 20:
        rc = sup.step(time.monotonic())
        time.sleep(0.02)
    assert rc == 4 and len(sup.restarts[0]) == 2


def test_failed_gpu_slot_is_replaced_while_the_other_keeps_serving(tmp_path):
    """--procs 2 on the null device, KDL_FAULT_INJECT fails every batch of GPU slot 1: its
    executor goes unhealthy, the child closes its listeners and exits 4, the launcher starts a
    fresh child for slot 1, every client request succeeds (retrying a broken connection, as
    the gateway's gRPC client does), and the launcher never exits."""
    base = tmp_path / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 0}')
    port = _free_port()
    logf = tmp_path / "launcher.log"
    env = dict(os.environ, PYTHONPATH=str(ROOT), KDL_FAULT_INJECT="fail=gpu1:-1", KDL_RESTART_BACKOFF_S="0.5")
    with open(logf, "w") as lf:
        p = subprocess.Popen([sys.executable, "-m", "kdl.serving", "--procs=2", f"--port={port}", "--rest_api_port=0",
                              f"--model_base_path={base}", "--device=null", "--host=127.0.0.1",
                              "--allowed_batch_sizes=1,2,4,8"], cwd=str(ROOT), env=env,
                             stdout=lf, stderr=subprocess.STDOUT, start_new_session=True)
    target = f"127.0.0.1:{port}"
    try:
        deadline, pids = time.time() + 240, set()
        while time.time() < deadline and len(pids) < 2:
            try:
                resp, pid = _health(target)
                if resp == b"\x08\x01":
                    pids.add(pid)
            except grpc.RpcError:
                pass
            time.sleep(0.2)
        assert len(pids) == 2
        rng = np.random.default_rng(1)
        ok = failed_attempts = 0
        for k in range(40):
            u8 = rng.integers(0, 200, (2, 299, 299, 3), dtype=np.uint8)
            for attempt in range(20):
                ch = grpc.insecure_channel(target, options=[("grpc.use_local_subchannel_pool", 1),
                                                            ("grpc.max_send_message_length", -1)])
                try:
                    r = PredictionStub(ch).Predict(make_request(u8, signature="serving_uint8", input_key="images"),
                                                   timeout=30)
                    got = np.asarray(r.outputs["dense_7"].float_val, np.float32).reshape(2, 10)
                    want = u8[:, 0, 0, 0:1].astype(np.float32) + np.arange(10, dtype=np.float32)[None]
                    assert np.array_equal(got, want)
                    ok += 1
                    break
                except grpc.RpcError:
                    failed_attempts += 1
                    time.sleep(0.1)
                finally:
                    ch.close()
        assert ok == 40 and failed_attempts > 0      # slot 1 did fail requests before it left
        # the replacement for slot 1 comes up as a new process; the launcher stays up
        deadline, seen = time.time() + 120, set()
        while time.time() < deadline and not (seen - pids):
            try:
                resp, pid = _health(target)
                if resp == b"\x08\x01":
                    seen.add(pid)
            except grpc.RpcError:
                pass
            time.sleep(0.2)
        assert seen - pids, "no replacement child answered"
        assert p.poll() is None
        text = logf.read_text()
        assert "GPU slot 1" in text and "restarted" in text
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)


def test_one_failing_signature_does_not_count_as_a_dead_device(tmp_path, monkeypatch):
    """Advisor r5: the --procs device watch (server._watch_devices) recycles a child only when no
    signature of any loaded version has a healthy executor left; one signature failing every
    batch (KDL_FAULT_INJECT on its executors only) leaves the device alive while readiness drops."""
    from kdl.serving.config import BatchingParams, ServerConfig
    from kdl.serving.model_repo import ModelManager

    monkeypatch.setenv("KDL_FAULT_INJECT", "fail=/serving_default:-1")
    base = tmp_path / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 0}')
    cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=str(base), device="null", host="127.0.0.1",
                       batching=BatchingParams(max_batch_size=4, batch_timeout_micros=200, allowed_batch_sizes=[1, 4]),
                       warm_signatures=["serving_uint8"])
    m = ModelManager(cfg)
    m.load_initial()
    try:
        s = m.servables[max(m.servables)]
        assert m.ready() and m.device_alive() and {"serving_default", "serving_uint8"} <= set(s.runners)
        bad, good = s.runners["serving_default"], s.runners["serving_uint8"]
        x = np.zeros((1, 299, 299, 3), np.float32)
        for _ in range(10):                          # every batch fails: its executors give up
            if not bad.healthy():
                break
            with pytest.raises(Exception):
                bad.predict(x.tobytes(), 1, 0)
        assert not bad.healthy() and not m.ready()
        # only the failing signature has been used: that is all the evidence, the device is dead
        assert not m.device_alive()
        out = good.predict(np.full((1, 299, 299, 3), 5, np.uint8).tobytes(), 1, 0)
        assert np.array_equal(out[0], 5 + np.arange(10, dtype=np.float32))
        assert not m.ready() and m.device_alive()   # another signature serves on the same device
    finally:
        for sv in m.servables.values():
            sv.close()
