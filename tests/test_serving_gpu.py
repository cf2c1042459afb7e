"""Model server on the MI355X: gRPC Predict through the native batcher into the
hipGraph-captured HIP engine, vs the fp32 oracle; plus RCCL world-size-1 DP."""
import os
import socket

import grpc
import numpy as np
import pytest
import torch

from kdl.gateway.client import PredictionStub, make_request
from kdl.models import xception as X
from kdl.serving.config import BatchingParams, ServerConfig
from kdl.serving.server import ModelServer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_server(tmp_path_factory):
    base = tmp_path_factory.mktemp("m") / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 0}')
    cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=str(base), device="gpu", gpus=1,
                       host="127.0.0.1", file_system_poll_wait_seconds=0,
                       batching=BatchingParams(max_batch_size=8, batch_timeout_micros=1000,
                                               allowed_batch_sizes=[1, 2, 4, 8]))
    srv = ModelServer(cfg).start(block_until_loaded=True)
    yield srv
    srv.stop(0)


def test_gpu_predict_matches_oracle(gpu_server):
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, (5, 299, 299, 3), dtype=np.uint8)
    x = u8.astype(np.float32) / 127.5 - 1.0
    stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{gpu_server.grpc_port}"))
    r = stub.Predict(make_request(x), timeout=60)
    got = np.asarray(r.outputs["dense_7"].float_val, np.float32).reshape(5, 10)
    r8 = stub.Predict(make_request(u8, signature="serving_uint8", input_key="images"), timeout=60)
    got8 = np.asarray(r8.outputs["dense_7"].float_val, np.float32).reshape(5, 10)
    ref = X.xception_forward(X.init_params(seed=0), torch.from_numpy(x)).numpy()
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() < 0.05 * scale
    assert np.abs(got8 - ref).max() < 0.05 * scale


def test_gpu_serving_image_resizes_on_device_exactly(gpu_server):
    """serving_image: any-size uint8 images, resized by the HIP kernel on the server's GPU,
    give bit-for-bit the logits of serving_uint8 fed with PIL-NEAREST-resized images."""
    from PIL import Image
    from kdl.serving.resize import Resizer
    stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{gpu_server.grpc_port}"))
    for n, H, W in [(1, 534, 400), (2, 1, 1), (1, 2200, 2200)]:
        raw = np.random.default_rng(H).integers(0, 256, (n, H, W, 3), dtype=np.uint8)
        pil = np.stack([np.asarray(Image.fromarray(im).resize((299, 299), Image.NEAREST)) for im in raw])
        r1 = stub.Predict(make_request(raw, signature="serving_image", input_key="images"), timeout=60)
        r2 = stub.Predict(make_request(pil, signature="serving_uint8", input_key="images"), timeout=60)
        a = np.asarray(r1.outputs["dense_7"].float_val, np.float32)
        assert a.size == 10 * n and np.array_equal(a, np.asarray(r2.outputs["dense_7"].float_val, np.float32))
    s = gpu_server.manager.get("clothing-model", None, None)
    assert s.runner("serving_image").resizer.device is not None, "resize ran on the CPU"
    assert s.runner("serving_image").device_path, "resized images round-tripped through the host"


def test_gpu_serving_image_device_rows_share_batches_with_host_rows(gpu_server):
    """Concurrent serving_image (device-resident rows, D2D into the engine slot) and
    serving_uint8 (pinned staging, H2D) requests land in the same batches; every request
    gets the logits of its own PIL-resized images (up to the bucket graphs' bf16 rounding:
    a batch of another size runs another captured graph)."""
    import threading
    from PIL import Image
    s = gpu_server.manager.get("clothing-model", None, None)
    img, u8 = s.runner("serving_image"), s.runner("serving_uint8")
    rng = np.random.default_rng(3)
    raws = [rng.integers(0, 256, (1 + i % 2, 300 + 37 * i, 400 - 23 * i, 3), dtype=np.uint8) for i in range(6)]
    pils = [np.stack([np.asarray(Image.fromarray(im).resize((299, 299), Image.NEAREST)) for im in r]) for r in raws]
    want = [u8.predict(p, p.shape[0], 0) for p in pils]
    got, errs = {}, []

    def worker(i):
        try:
            for _ in range(4):
                got.setdefault(i, []).append(img.predict(raws[i], raws[i].shape[0], 0) if i % 2 == 0
                                             else u8.predict(pils[i], pils[i].shape[0], 0))
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ths = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not errs, errs
    for i in range(6):
        scale = np.abs(want[i]).max()
        assert all(np.abs(g - want[i]).max() <= 0.02 * scale for g in got[i]), i


def test_rccl_world1_dp_runner():
    import torch.distributed as dist

    from kdl.parallel.dp import DPRunner
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        inp = torch.zeros((4, 8, 8, 3), dtype=torch.uint8, device="cuda")
        out = torch.zeros((4, 10), device="cuda")

        def fwd(k):
            out[:k, 0] = inp[:k].float().mean(dim=(1, 2, 3))
            return out
        r = DPRunner(inp, fwd, [1, 2, 4], torch.device("cuda", 0))
        batch = torch.stack([torch.full((8, 8, 3), i, dtype=torch.uint8) for i in range(3)]).cuda()
        stopped, logits = r.step(batch)
        assert not stopped and logits[:, 0].tolist() == [0.0, 1.0, 2.0]
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("family", ["resnet50", "vit_b16"])
def test_gpu_serving_other_families(tmp_path, family):
    from kdl.engine import registry
    info = registry.get(family)
    base = tmp_path / family
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 2, "model": "%s"}' % family)
    cfg = ServerConfig(port=0, rest_api_port=0, model_name=family, model_base_path=str(base), device="gpu", gpus=1,
                       host="127.0.0.1", file_system_poll_wait_seconds=0,
                       batching=BatchingParams(max_batch_size=4, batch_timeout_micros=1000, allowed_batch_sizes=[2, 4]))
    srv = ModelServer(cfg).start(block_until_loaded=True)
    try:
        S = info.input_size
        x = np.random.default_rng(1).integers(0, 256, (3, S, S, 3), dtype=np.uint8)
        stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{srv.grpc_port}"))
        r = stub.Predict(make_request(x, model_name=family, input_key="images"), timeout=120)
        got = torch.from_numpy(np.asarray(r.outputs["logits"].float_val, np.float32).reshape(3, info.classes))
        ref = info.oracle(info.init_params(2), torch.from_numpy(x))
        assert torch.nn.functional.cosine_similarity(got, ref, dim=1).min() > 0.98
    finally:
        srv.stop(0)



def test_gpu_server_lanes_path_matches_oracle(tmp_path, monkeypatch):
    """KDL_LANES=2: a full top-bucket batch (16) runs on the executor's LaneGroup
    (two 8-image hipGraph lanes, kdl/engine/lanes.py) and still matches the oracle."""
    monkeypatch.setenv("KDL_LANES", "2")
    base = tmp_path / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 0}')
    cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=str(base), device="gpu", gpus=1,
                       host="127.0.0.1", file_system_poll_wait_seconds=0,
                       batching=BatchingParams(max_batch_size=16, batch_timeout_micros=1000,
                                               allowed_batch_sizes=[4, 16]))
    srv = ModelServer(cfg).start(block_until_loaded=True)
    try:
        rng = np.random.default_rng(3)
        u8 = rng.integers(0, 256, (16, 299, 299, 3), dtype=np.uint8)
        stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{srv.grpc_port}"))
        r = stub.Predict(make_request(u8, signature="serving_uint8", input_key="images"), timeout=60)
        got = np.asarray(r.outputs["dense_7"].float_val, np.float32).reshape(16, 10)
    finally:
        srv.stop(0)
    x = torch.from_numpy(u8.astype(np.float32) / 127.5 - 1.0)
    ref = X.xception_forward(X.init_params(seed=0), x).numpy()
    assert np.abs(got - ref).max() < 0.05 * np.abs(ref).max()


def test_native_executors_two_per_gpu_concurrent_clients(tmp_path):
    """executors_per_gpu=2: two native C++ executors (kdl._rt.Executor over
    kdl._C.HipExecBackend, each with its own engine, stage pipe and hipGraphs) share one GPU and
    one batcher; 8 concurrent clients get their own, oracle-exact logits; both executors take
    batches; the C++ stage trace reaches the Prometheus endpoint."""
    import threading

    from kdl.serving.metrics import METRICS
    base = tmp_path / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 0}')
    cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=str(base), device="gpu", gpus=1,
                       host="127.0.0.1", file_system_poll_wait_seconds=0, executors_per_gpu=2,
                       batching=BatchingParams(max_batch_size=8, batch_timeout_micros=500,
                                               allowed_batch_sizes=[2, 4, 8]))
    srv = ModelServer(cfg).start(block_until_loaded=True)
    rng = np.random.default_rng(7)
    imgs = rng.integers(0, 256, (24, 299, 299, 3), dtype=np.uint8)
    got = np.zeros((24, 10), np.float32)
    errs = []
    try:
        runner = srv.manager.get("clothing-model").runner("serving_uint8")
        assert len(runner.executors) == 2 and all(ex.native is not None for ex in runner.executors)

        def client(k):
            stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{srv.grpc_port}"))
            try:
                for rep in range(3):
                    sl = slice(3 * k, 3 * k + 3)
                    r = stub.Predict(make_request(imgs[sl], signature="serving_uint8", input_key="images"), timeout=60)
                    got[sl] = np.asarray(r.outputs["dense_7"].float_val, np.float32).reshape(3, 10)
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        ths = [threading.Thread(target=client, args=(k,)) for k in range(8)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(120)
        stats = [ex.native.stats() for ex in runner.executors]
        text = METRICS.render()          # what /monitoring/prometheus/metrics serves
    finally:
        srv.stop(0)
    assert not errs, errs
    p = {k: v.cuda() for k, v in X.init_params(seed=0).items()}
    ref = X.xception_forward(p, torch.from_numpy(imgs).cuda().float() / 127.5 - 1.0).cpu().numpy()
    assert np.abs(got - ref).max() < 0.05 * np.abs(ref).max()
    assert all(s["batches"] > 0 for s in stats), stats
    assert sum(s["items"] for s in stats) == 72
    fw = [s["stages"]["device_forward"] for s in stats]
    assert all(h["count"] > 0 and h["sum_ms"] > 0 for h in fw)
    assert 'kdl_exec_stage_ms_count{executor="gpu0/serving_uint8",stage="device_forward"}' in text
    assert "kdl_gpu_busy_ratio" in text


def test_native_and_python_executors_agree_bit_for_bit(tmp_path, monkeypatch):
    """The native executor replays the very same captured graphs as the Python loop it replaced:
    identical logits for an identical request."""
    rng = np.random.default_rng(11)
    u8 = rng.integers(0, 256, (4, 299, 299, 3), dtype=np.uint8)
    outs = []
    for native in ("1", "0"):
        monkeypatch.setenv("KDL_NATIVE_EXEC", native)
        base = tmp_path / native / "clothing-model"
        (base / "1").mkdir(parents=True)
        (base / "1" / "synthetic.json").write_text('{"seed": 0}')
        cfg = ServerConfig(port=0, rest_api_port=0, model_base_path=str(base), device="gpu", gpus=1,
                           host="127.0.0.1", file_system_poll_wait_seconds=0,
                           batching=BatchingParams(max_batch_size=4, batch_timeout_micros=500, allowed_batch_sizes=[4]))
        srv = ModelServer(cfg).start(block_until_loaded=True)
        try:
            ex = srv.manager.get("clothing-model").runner("serving_uint8").executors[0]
            assert (ex.native is not None) == (native == "1")
            stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{srv.grpc_port}"))
            r = stub.Predict(make_request(u8, signature="serving_uint8", input_key="images"), timeout=60)
            outs.append(np.asarray(r.outputs["dense_7"].float_val, np.float32))
        finally:
            srv.stop(0)
    assert np.array_equal(outs[0], outs[1])


def test_rccl_scatter_server_world1(tmp_path):
    """``--scatter rccl`` on the GPU: the launcher, rank 0's front-end, the model handed over by
    broadcast (C1), every batch scattered (C2) into the engine's static input and the logits
    gathered (C3) over RCCL -- world size 1 on this one-GPU box (the 8-GPU group is the same
    code; tests/test_dp_serving.py runs two ranks over gloo)."""
    import signal
    import subprocess
    import sys
    import time
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    base = tmp_path / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text('{"seed": 0}')
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    logf = open(tmp_path / "srv.log", "w")
    p = subprocess.Popen([sys.executable, "-m", "kdl.serving", "--scatter=rccl", "--dp_world=1", f"--port={port}",
                          "--rest_api_port=0", f"--model_base_path={base}", "--host=127.0.0.1",
                          "--allowed_batch_sizes=1,2,4,8"], cwd=str(root), stdout=logf, stderr=subprocess.STDOUT,
                         env=dict(os.environ, PYTHONPATH=str(root)), start_new_session=True)
    try:
        deadline, ok = time.time() + 100, False
        while time.time() < deadline and not ok and p.poll() is None:
            try:
                ch = grpc.insecure_channel(f"127.0.0.1:{port}")
                ok = ch.unary_unary("/grpc.health.v1.Health/Check")(b"", timeout=5) == b"\x08\x01"
                ch.close()
            except grpc.RpcError:
                time.sleep(0.5)
        assert ok, (tmp_path / "srv.log").read_text()[-3000:]
        rng = np.random.default_rng(1)
        u8 = rng.integers(0, 256, (3, 299, 299, 3), dtype=np.uint8)
        x = u8.astype(np.float32) / 127.5 - 1.0
        stub = PredictionStub(grpc.insecure_channel(f"127.0.0.1:{port}", options=[("grpc.max_send_message_length", -1)]))
        ref = X.xception_forward(X.init_params(seed=0), torch.from_numpy(x)).numpy()
        # the data-parallel signature (default serving_uint8): native DpLeader + RCCL comms
        for n in (3, 8, 1):
            r = stub.Predict(make_request(u8[:n] if n <= 3 else np.concatenate([u8] * 3)[:n],
                                          signature="serving_uint8", input_key="images"), timeout=60)
            got = np.asarray(r.outputs["dense_7"].float_val, np.float32).reshape(n, 10)
            want = ref[:n] if n <= 3 else np.concatenate([ref] * 3)[:n]
            assert np.abs(got - want).max() < 0.05 * np.abs(ref).max(), n
        # the reference client's f32 serving_default request: rank 0's own executor
        r = stub.Predict(make_request(x), timeout=60)
        got = np.asarray(r.outputs["dense_7"].float_val, np.float32).reshape(3, 10)
        assert np.abs(got - ref).max() < 0.05 * np.abs(ref).max()
        text = (tmp_path / "srv.log").read_text()
        assert "rccl data-parallel group of 1" in text
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        logf.close()


def test_native_dp_leader_world1_matches_local_backend(tmp_path):
    """comm.cpp at world size 1 (one GPU on this box): two RCCL communicators, DpLeader wrapping
    the same captured graphs as the single-GPU HipExecBackend; a batch through the leader gives
    exactly the local backend's logits, and the stop control word goes out cleanly."""
    import torch.distributed as dist

    from kdl.engine.xception import XceptionEngine
    from kdl.ops import _lib
    C = _lib.lib()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        p = X.init_params(seed=0)
        eng = XceptionEngine(p, max_batch=4, buckets=[2, 4])
        eng.add_input_slots(2)
        item = 299 * 299 * 3
        be = C.HipExecBackend(0, 2, item, 4, 10)
        progs = {b: [[[eng.program(b, True, s)]] * 2 for s in range(2)] for b in (2, 4)}
        for b in (2, 4):
            be.add_recipe(b, [eng.stream.cuda_stream], [0], progs[b], [eng.inputs[s].data_ptr() for s in range(2)],
                          [eng.slot_logits(s).data_ptr() for s in range(2)])
        ids = [C.rccl_unique_id(), C.rccl_unique_id()]
        comms = [C.RcclComm(i, 1, 0, 0) for i in ids]
        lead = C.DpLeader(be, *comms, [2, 4], 30.0)
        rng = np.random.default_rng(3)
        u8 = rng.integers(0, 256, (4, 299, 299, 3), dtype=np.uint8)
        outs = []
        for run in (be.run, lead.run):
            st = np.frombuffer((ctypes_buffer(be.staging_ptr(0), 4 * item)), dtype=np.uint8)
            st[:] = u8.reshape(-1)
            res = run(0, 4, 4)
            ptr = res[0] if isinstance(res, tuple) else res
            outs.append(np.frombuffer(ctypes_buffer(ptr, 4 * 10 * 4), dtype=np.float32).copy().reshape(4, 10))
        assert np.array_equal(outs[0], outs[1])
        ref = X.xception_forward(p, torch.from_numpy(u8).float() / 127.5 - 1.0).numpy()
        assert np.abs(outs[1] - ref).max() < 0.05 * np.abs(ref).max()
        assert lead.send_ctrl(C.DP_STOP, 0) == 0 and lead.steps == 1
        del lead, comms, be
    finally:
        dist.destroy_process_group()


def ctypes_buffer(ptr: int, n: int):
    import ctypes
    return (ctypes.c_uint8 * n).from_address(ptr)
