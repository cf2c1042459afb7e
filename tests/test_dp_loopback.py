"""The native data-parallel protocol EXECUTED at world 2/4/8 on the CPU.

kdl/csrc/runtime/dp_core.h holds the leader / follower state machine once, templated on a
platform; kdl._C instantiates it over HIP + RCCL, kdl._rt over the loopback platform of
dp_loop.h (stream threads, host memory, rendezvous send/recv queues per (channel, peer)). Here
rank 0's DpLeader sits under the real native DynamicBatcher + Executor, N-1 DpFollowers run in
threads, and every request's rows must come back with ITS logits: the fake forward of every
rank maps input row i (its first 4 bytes = a unique id) to f(id, column, model version).

Covers VERDICT r4 "next" item 1: random batch sizes (padded buckets), DP_RELOAD mid-stream
then more batches under the new version, a dead follower failing the leader within timeout_s
(executor unhealthy), a dead leader ending the followers within their liveness window, and
idle keep-alive pings. Reference scale-out being replaced: Deployment replicas behind a Service
(/root/reference/tf-serving-clothing-model-deployment.yaml:8)."""
import threading
import time

import numpy as np
import pytest

from kdl.ops import _lib

pytestmark = pytest.mark.skipif(not _lib.rt_available(), reason="kdl._rt not built")
ITEM, COLS = 64, 4


class Group:
    """One DP group of `world` loopback ranks; followers in threads, rebuilt on DP_RELOAD."""

    def __init__(self, world, buckets, nslots=2, latency_us=150, timeout_s=5.0, ping_s=0.0, liveness_s=5.0,
                 epochs=3):
        self.rt = _lib.rt()
        self.world, self.buckets, self.nslots = world, buckets, nslots
        self.latency_us, self.timeout_s, self.ping_s, self.liveness_s = latency_us, timeout_s, ping_s, liveness_s
        self.ids = [(self.rt.loop_unique_id(), self.rt.loop_unique_id()) for _ in range(epochs)]
        self.comms = {}                  # (epoch, rank) -> (scatter, gather)
        self.result = {}                 # rank -> ("stop"|"error", t, detail)
        self.forwards = {}
        self.threads = [threading.Thread(target=self._follow, args=(r,), daemon=True) for r in range(1, world)]
        for t in self.threads:
            t.start()
        self.epoch = 0
        self._lead(0)

    def _comm(self, epoch, rank):
        key = (epoch, rank)
        if key not in self.comms:
            s, g = self.ids[epoch]
            self.comms[key] = (self.rt.LoopComm(s, self.world, rank), self.rt.LoopComm(g, self.world, rank))
        return self.comms[key]

    def _follow(self, rank):
        rt, epoch, version = self.rt, 0, 0
        while True:
            dev = rt.LoopDevice(rank, self.nslots, ITEM, max(self.buckets), COLS, self.buckets, version,
                                self.latency_us)
            f = rt.LoopDpFollower(dev, *self._comm(epoch, rank))
            try:
                cmd, ver, _seq = f.run(self.liveness_s)
            except RuntimeError as e:
                self.result[rank] = ("error", time.monotonic(), str(e))
                return
            finally:
                self.forwards[rank] = self.forwards.get(rank, 0) + dev.forwards
            if cmd == rt.DP_RELOAD:
                epoch, version = epoch + 1, ver
                continue
            self.result[rank] = ("stop", time.monotonic(), cmd)
            return

    def _lead(self, version):
        rt = self.rt
        mb = self.world * max(self.buckets)
        self.version = version
        self.dev0 = rt.LoopDevice(0, self.nslots, ITEM, mb, COLS, self.buckets, version, self.latency_us)
        self.leader = rt.LoopDpLeader(self.dev0, *self._comm(self.epoch, 0), self.buckets, self.timeout_s, self.ping_s)
        self.batcher = rt.DynamicBatcher(max_batch_size=mb, batch_timeout_us=400, max_enqueued_batches=256,
                                         allowed_batch_sizes=[self.world * b for b in self.buckets], item_bytes=ITEM,
                                         out_cols=COLS)
        self.xgroup = rt.ExecGroup()
        self.ex = rt.Executor(self.batcher, self.leader, self.xgroup, name=f"dp{self.world}", max_failures=2,
                              poll_us=2000)
        self.ex.start()

    def reload(self, version):
        """Mid-stream hot reload: drain rank 0's executor, DP_RELOAD(version) to every follower
        (they leave their loop and rebuild), new communicators + leader + executor."""
        self.ex.stop()
        assert self.leader.send_ctrl(self.rt.DP_RELOAD, version) == 0
        self.batcher.shutdown()
        self.epoch += 1
        self._lead(version)

    def stop(self):
        self.ex.stop()
        rc = self.leader.send_ctrl(self.rt.DP_STOP, 0)
        self.batcher.shutdown()
        for t in self.threads:
            t.join(30)
        return rc


def _clients(g, n_threads=4, n_req=25, seed=0, max_items=None):
    rt = g.rt
    mb = max_items or g.world * max(g.buckets)
    ok, bad, err = [], [], []
    lock = threading.Lock()

    def client(s):
        rng = np.random.default_rng(seed * 1000 + s)
        for r in range(n_req):
            n = int(rng.integers(1, mb + 1))
            ids = (s * 100000 + r * 100 + np.arange(n)).astype(np.uint32) + seed * 10000000 % 1000
            data = rng.integers(0, 256, size=(n, ITEM), dtype=np.uint8)
            data[:, :4] = ids.view(np.uint8).reshape(n, 4)
            t = g.batcher.submit(data.reshape(-1), n, 0)
            out = np.zeros((n, COLS), np.float32)
            st = g.batcher.wait(t, out) if t >= 0 else -t
            with lock:
                if st != rt.ST_OK:
                    err.append(st)
                    continue
                want = np.array([[rt.LoopDevice.logit(int(i), k, g.version) for k in range(COLS)] for i in ids],
                                np.float32)
                (ok if np.array_equal(out, want) else bad).append((s, r, n))

    ths = [threading.Thread(target=client, args=(s,)) for s in range(n_threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    return ok, bad, err


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_world_serves_every_row_then_reloads_mid_stream(world):
    g = Group(world, buckets=[1, 2, 4, 8], nslots=2 if world < 8 else 3)
    ok, bad, err = _clients(g, seed=1)
    assert not bad and not err and len(ok) == 4 * 25
    steps0 = g.leader.steps
    assert steps0 > 0 and g.ex.stats()["batches"] == steps0
    g.reload(version=3)                  # followers rebuild at version 3 on new communicators
    ok2, bad2, err2 = _clients(g, seed=2)
    assert not bad2 and not err2 and len(ok2) == 4 * 25
    assert g.stop() == 0
    assert all(g.result[r][0] == "stop" for r in range(1, world)), g.result
    # every follower computed shards in both versions
    assert all(g.forwards[r] >= 2 for r in range(1, world))


def test_world1_leader_is_the_local_backend():
    g = Group(1, buckets=[1, 4, 16])
    ok, bad, err = _clients(g, seed=3)
    assert not bad and not err and len(ok) == 100
    assert g.stop() == 0


def test_dead_follower_fails_the_leader_within_timeout_and_executor_goes_unhealthy():
    g = Group(4, buckets=[1, 2, 4], timeout_s=1.0, liveness_s=2.0)
    ok, bad, err = _clients(g, n_threads=2, n_req=10, seed=4)
    assert not bad and not err
    s, ga = g.comms[(0, 2)]
    s.kill()                             # rank 2's process "dies": nothing of it matches any more
    ga.kill()
    t0 = time.monotonic()
    ok2, bad2, err2 = _clients(g, n_threads=2, n_req=5, seed=5)
    dt = time.monotonic() - t0
    assert not bad2 and err2                  # its batches failed (ST_ERROR), none mis-delivered
    assert not g.ex.healthy() and g.leader.broken
    assert dt < 1.0 * 2 + 5, dt               # bounded by the leader's timeout, not a hang
    g.ex.stop()
    # the live followers notice the silence (no pings from a broken leader) and exit
    for t in g.threads:
        t.join(10)
    assert all(not t.is_alive() for t in g.threads)
    assert g.result[1][0] == "error" and g.result[3][0] == "error"


def test_dead_leader_ends_followers_within_liveness_and_pings_keep_idle_ones_alive():
    g = Group(3, buckets=[1, 2], ping_s=0.1, liveness_s=1.0)
    ok, bad, err = _clients(g, n_threads=2, n_req=5, seed=6)
    assert not bad and not err
    time.sleep(2.5)                      # idle > liveness: the heartbeat keeps followers alive
    assert all(t.is_alive() for t in g.threads) and not g.result
    ok, bad, err = _clients(g, n_threads=1, n_req=3, seed=7)
    assert not bad and not err and len(ok) == 3
    g.ex.stop()
    t0 = time.monotonic()
    for c in g.comms[(0, 0)]:
        c.kill()                         # rank 0 dies: no more control words of any kind
    for t in g.threads:
        t.join(10)
    assert all(not t.is_alive() for t in g.threads)
    for r in (1, 2):
        kind, t_end, detail = g.result[r]
        assert kind == "error" and "liveness" in detail
        assert t_end - t0 < 1.0 + 1.5, t_end - t0


def test_one_local_issue_failure_fails_one_batch_not_the_group():
    """Advisor r5: a failure of rank 0's own engine issue must fail that batch only. The
    leader used to spend a sequence number before the local issue, so the next control word
    (batch or heartbeat) reached every follower out of sequence and the whole group died."""
    g = Group(2, buckets=[1, 2, 4], ping_s=0.1, liveness_s=2.0)
    ok, bad, err = _clients(g, n_threads=1, n_req=5, seed=8)
    assert not bad and not err
    g.dev0.fail_issues(1)                # the next local issue fails before touching anything
    ok1, bad1, err1 = _clients(g, n_threads=1, n_req=3, seed=9)
    assert not bad1 and len(err1) == 1 and len(ok1) == 2, (ok1, err1)
    time.sleep(0.5)                      # heartbeats after the failure keep the follower in sequence
    ok2, bad2, err2 = _clients(g, n_threads=2, n_req=10, seed=10)
    assert not bad2 and not err2 and len(ok2) == 20
    assert not g.leader.broken and g.ex.healthy()
    assert g.stop() == 0
    assert g.result[1][0] == "stop", g.result
