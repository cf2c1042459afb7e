"""``--scatter rccl``: one front-end, batches scattered / logits gathered over the group.

CPU rehearsal on gloo with two ranks (the GPU path is the same code on the "nccl" = RCCL
backend, one process per GPU): the launcher starts rank 0 (gRPC front-end + batcher) and a
follower; the follower gets the model by broadcast (C1), every Predict batch is split over
both ranks (C2), each rank runs its fp32 CPU oracle on its shard, the logits come back by
gather (C3) and match the single-process oracle; SIGTERM to the launcher stops rank 0,
whose stop broadcast ends the follower.
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
import torch

from kdl.gateway.client import PredictionStub, make_request
from kdl.models import xception as X

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture()
def dp_group(tmp_path):
    base = tmp_path / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 3}')
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2")
    log = open(tmp_path / "server.log", "w")
    p = subprocess.Popen([sys.executable, "-m", "kdl.serving", "--scatter=rccl", "--dp_world=2", f"--port={port}",
                          "--rest_api_port=0", f"--model_base_path={base}", "--device=cpu", "--host=127.0.0.1",
                          "--allowed_batch_sizes=1,2", "--batch_timeout_micros=20000", "--dp_signature=serving_uint8"],
                         cwd=str(ROOT), env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    target = f"127.0.0.1:{port}"
    try:
        deadline = time.time() + 300
        ok = False
        while time.time() < deadline and not ok and p.poll() is None:
            try:
                ch = grpc.insecure_channel(target)
                ok = ch.unary_unary("/grpc.health.v1.Health/Check")(b"", timeout=5) == b"\x08\x01"
                ch.close()
            except grpc.RpcError:
                time.sleep(0.5)
        assert ok, (tmp_path / "server.log").read_text()[-3000:]
        yield p, target, tmp_path / "server.log"
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
            try:
                p.wait(timeout=90)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        log.close()


def test_rccl_group_scatters_batches_and_matches_the_oracle(dp_group):
    p, target, logf = dp_group
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, (3, 299, 299, 3), dtype=np.uint8)    # 3 images -> 2 per rank, one padded
    ch = grpc.insecure_channel(target, options=[("grpc.max_send_message_length", -1)])
    r = PredictionStub(ch).Predict(make_request(u8, signature="serving_uint8", input_key="images"), timeout=240)
    got = np.asarray(r.outputs["dense_7"].float_val, np.float32).reshape(3, 10)
    ref = X.xception_forward(X.init_params(seed=3), torch.from_numpy(u8).float() / 127.5 - 1.0).numpy()
    assert np.allclose(got, ref, atol=1e-3, rtol=1e-3), np.abs(got - ref).max()
    ch.close()
    text = logf.read_text()
    assert "rccl data-parallel group of 2" in text and "dp rank 1/2" in text, text[-2000:]


def test_sigterm_stops_rank0_and_the_follower(dp_group):
    p, target, logf = dp_group
    os.kill(p.pid, signal.SIGTERM)
    assert p.wait(timeout=120) == 0, logf.read_text()[-3000:]
    assert "dp rank 1: stop after" in logf.read_text()
