"""The native data-parallel protocol at WORLD 2 on ONE MI355X.

RCCL refuses two ranks on one device (tools/probes/rccl_dup_probe.py), so the RCCL instance of
dp_core.h can only run at world 1 on a one-GPU box. Here the same DpLeaderT / DpFollowerT run
over the HIP loopback platform (kdl/csrc/runtime/dp_hiploop.h): two real Xception engines with
captured hipGraphs (HipExecBackend), real HIP streams / events, hipMalloc'd control words and
send buffers, the follower's real HipExecBackend::launch keyed by the device-side control word's
per-rank bucket -- only the byte mover is a device-to-device copy instead of ncclSend / ncclRecv.
Rank 0's leader sits under the native DynamicBatcher + Executor exactly as in --scatter rccl;
rank 1 runs DpFollower.run() in a thread of this process.

Checked: every row of every request (1..8 images, so padded world x bucket batches) against the
fp32 oracle; DP_RELOAD mid-stream to a new model version (new weights on both ranks, rows then
match the new version's oracle); a follower that dies fails the leader within timeout_s (the
executor goes unhealthy, no row is mis-delivered). Reference scale-out being replaced:
/root/reference/tf-serving-clothing-model-deployment.yaml:8.
"""
import threading
import time

import numpy as np
import pytest
import torch

from kdl.engine.xception import XceptionEngine
from kdl.models import xception as X
from kdl.ops import _lib

pytestmark = pytest.mark.gpu
ITEM = 299 * 299 * 3
BUCKETS = [1, 2, 4]                 # per-rank buckets; the batcher forms 2 x these


def _engine_backend(C, params, max_batch):
    eng = XceptionEngine(params, max_batch=max(BUCKETS), buckets=BUCKETS)
    eng.add_input_slots(2)
    be = C.HipExecBackend(0, 2, ITEM, max_batch, 10)
    for b in BUCKETS:
        progs = [[[eng.program(b, True, s)]] * 2 for s in range(2)]
        be.add_recipe(b, [eng.stream.cuda_stream], [0], progs, [eng.inputs[s].data_ptr() for s in range(2)],
                      [eng.slot_logits(s).data_ptr() for s in range(2)])
    return eng, be


class World2:
    """Rank 0 (leader under the native executor) + rank 1 (follower thread) of one version."""

    def __init__(self, C, rt, params, version, timeout_s=10.0, liveness_s=8.0):
        self.C, self.rt, self.params, self.version = C, rt, params, version
        ids = (C.hiploop_unique_id(), C.hiploop_unique_id())
        self.eng0, self.be0 = _engine_backend(C, params, 2 * max(BUCKETS))
        self.eng1, self.be1 = _engine_backend(C, params, max(BUCKETS))
        self.c1 = (C.HipLoopComm(ids[0], 2, 1), C.HipLoopComm(ids[1], 2, 1))
        self.c0 = (C.HipLoopComm(ids[0], 2, 0), C.HipLoopComm(ids[1], 2, 0))
        self.result = None
        self.follower = C.HipLoopDpFollower(self.be1, *self.c1)

        def follow():
            try:
                self.result = ("ok",) + tuple(self.follower.run(liveness_s))
            except RuntimeError as e:
                self.result = ("error", str(e))
        self.th = threading.Thread(target=follow, daemon=True)
        self.th.start()
        self.lead = C.HipLoopDpLeader(self.be0, *self.c0, BUCKETS, timeout_s, 0.2)
        self.batcher = rt.DynamicBatcher(max_batch_size=2 * max(BUCKETS), batch_timeout_us=500,
                                         max_enqueued_batches=64, allowed_batch_sizes=[2 * b for b in BUCKETS],
                                         item_bytes=ITEM, out_cols=10)
        self.group = rt.ExecGroup()
        self.ex = rt.Executor(self.batcher, self.lead, self.group, name="hiploop-dp2", max_failures=2, poll_us=2000)
        self.ex.start()

    def close(self, cmd, version=0):
        self.ex.stop()
        rc = self.lead.send_ctrl(cmd, version)
        self.batcher.shutdown()
        self.th.join(60)
        return rc


def _oracle(params, u8):
    p = {k: v.cuda() for k, v in params.items()}
    with torch.no_grad():
        return X.xception_forward(p, torch.from_numpy(u8).cuda().float() / 127.5 - 1.0).float().cpu().numpy()


def _clients(w, n_threads=3, n_req=6, seed=0):
    rng = np.random.default_rng(seed)
    reqs = [rng.integers(0, 256, (int(rng.integers(1, 2 * max(BUCKETS) + 1)), 299, 299, 3), dtype=np.uint8)
            for _ in range(n_threads * n_req)]
    outs = [None] * len(reqs)

    def client(t):
        for i in range(t, len(reqs), n_threads):
            u8 = reqs[i]
            tk = w.batcher.submit(u8.reshape(-1), len(u8), 0)
            out = np.zeros((len(u8), 10), np.float32)
            st = w.batcher.wait(tk, out) if tk >= 0 else -tk
            outs[i] = (st, out)

    ths = [threading.Thread(target=client, args=(t,)) for t in range(n_threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(300)
    return reqs, outs


def _check_rows(w, reqs, outs):
    ok = 0
    for u8, (st, out) in zip(reqs, outs):
        assert st == w.rt.ST_OK, st
        ref = _oracle(w.params, u8)
        err = np.abs(out - ref).max() / np.abs(ref).max()
        cos = (out * ref).sum(1) / (np.linalg.norm(out, axis=1) * np.linalg.norm(ref, axis=1))
        assert err < 0.05 and cos.min() > 0.995, (len(u8), err, cos.min())
        ok += len(u8)
    return ok


def test_hip_loopback_dp_world2_rows_reload_and_dead_follower():
    C, rt = _lib.lib(), _lib.rt()
    p1 = X.init_params(seed=0)
    w = World2(C, rt, p1, version=1)
    try:
        reqs, outs = _clients(w, seed=1)
        rows = _check_rows(w, reqs, outs)
        assert rows > 20 and w.lead.steps > 0 and w.follower.steps == w.lead.steps
        # DP_RELOAD mid-stream: the follower leaves its loop with the new version; both ranks then
        # serve version 2's weights on new communicators
        assert w.close(C.DP_RELOAD, 2) == 0
        assert w.result == ("ok", C.DP_RELOAD, 2, w.result[3]), w.result
    except BaseException:
        w.close(C.DP_STOP)
        raise
    p2 = X.init_params(seed=5)
    w2 = World2(C, rt, p2, version=2, timeout_s=3.0, liveness_s=3.0)
    try:
        reqs, outs = _clients(w2, seed=2)
        _check_rows(w2, reqs, outs)
        # rank 1 dies: nothing of it matches any more; rank 0's next batches fail within timeout_s
        w2.c1[0].kill()
        w2.c1[1].kill()
        t0 = time.monotonic()
        u8 = np.zeros((3, 299, 299, 3), np.uint8)
        st = []
        for _ in range(3):
            tk = w2.batcher.submit(u8.reshape(-1), 3, 0)
            st.append(w2.batcher.wait(tk, np.zeros((3, 10), np.float32)) if tk >= 0 else -tk)
        dt = time.monotonic() - t0
        assert all(s != rt.ST_OK for s in st), st      # failed, never mis-delivered
        assert w2.lead.broken and not w2.ex.healthy()
        assert dt < 3 * 3.0 + 10, dt                   # bounded by the leader's timeout, not a hang
        w2.ex.stop()
        w2.th.join(30)
        assert not w2.th.is_alive() and w2.result[0] == "error", w2.result
    finally:
        w2.ex.stop()
        w2.batcher.shutdown()
