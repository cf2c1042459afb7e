"""The native batch executor (kdl/csrc/runtime/executor.cpp) against the fake device backend.

CPU only: the C++ executor threads pull batches from the C++ batcher into the fake
backend's staging, "run" them (result row = first byte of the item, +k per column) with a
simulated device latency and several batches in flight, and scatter results back -- the
same code path the HIP backend (kdl/csrc/runtime/hip_backend.cpp) plugs into on a GPU.
"""
import threading
import time

import numpy as np
import pytest

from kdl.ops import _lib

rt = _lib.rt()
ITEM, COLS, MAXB = 96, 4, 8


def _batcher(**kw):
    return rt.DynamicBatcher(max_batch_size=MAXB, batch_timeout_us=500, max_enqueued_batches=64,
                             allowed_batch_sizes=[1, 2, 4, 8], item_bytes=ITEM, out_cols=COLS, **kw)


def _client(b, seed, n_req, errors, results, deadline_us=0):
    rng = np.random.default_rng(seed)
    for r in range(n_req):
        n = int(rng.integers(1, 5))
        vals = rng.integers(0, 200, size=n).astype(np.uint8)
        data = np.repeat(vals, ITEM).astype(np.uint8)
        t = b.submit(data, n, rt.now_us() + deadline_us if deadline_us else 0)
        if t < 0:
            errors.append(("submit", -t))
            continue
        out = np.zeros((n, COLS), np.float32)
        st = b.wait(t, out)
        if st != rt.ST_OK:
            errors.append(("wait", st))
            continue
        want = vals[:, None].astype(np.float32) + np.arange(COLS, dtype=np.float32)[None]
        results.append(bool(np.array_equal(out, want)))


def _run_clients(b, n_threads=6, n_req=80, **kw):
    errors, results = [], []
    ths = [threading.Thread(target=_client, args=(b, s, n_req, errors, results), kwargs=kw) for s in range(n_threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    return errors, results


def test_two_executors_serve_every_request_with_batches_in_flight():
    b = _batcher()
    g = rt.ExecGroup()
    fakes = [rt.FakeBackend(nslots=2, item_bytes=ITEM, max_batch=MAXB, out_cols=COLS, latency_us=300) for _ in range(2)]
    exs = [rt.Executor(b, f, g, name=f"fake{i}") for i, f in enumerate(fakes)]
    for e in exs:
        e.start()
    errors, results = _run_clients(b)
    for e in exs:
        e.stop()
    b.shutdown()
    assert not errors and len(results) == 6 * 80 and all(results)
    st = [e.stats() for e in exs]
    assert sum(s["items"] for s in st) == b.stats()["items"] > 0
    assert all(s["batches"] > 0 for s in st), "both executors pulled batches"
    for s in st:
        lat = s["stages"]["batch_latency"]
        assert lat["count"] == s["batches"] and sum(lat["buckets"]) == lat["count"]
        fw = s["stages"]["device_forward"]
        assert fw["count"] == s["batches"] and abs(fw["sum_ms"] / fw["count"] - 0.3) < 1e-3
        assert s["stages"]["in_flight"]["sum_ms"] / s["batches"] >= 0.25   # waited for the device
    tr = exs[0].recent(5)
    assert tr and all(t["oldest_enqueue_us"] <= t["formed_us"] <= t["copied_us"] <= t["issued_us"]
                      <= t["completed_us"] <= t["finished_us"] for t in tr)
    assert g.healthy() == 2


def test_failing_device_is_isolated_and_the_other_serves_everything():
    b = _batcher()
    g = rt.ExecGroup()
    good = rt.FakeBackend(nslots=2, item_bytes=ITEM, max_batch=MAXB, out_cols=COLS, latency_us=100)
    bad = rt.FakeBackend(nslots=2, item_bytes=ITEM, max_batch=MAXB, out_cols=COLS, latency_us=100, fail_every=1)
    e_bad = rt.Executor(b, bad, g, name="bad", max_failures=2)
    e_good = rt.Executor(b, good, g, name="good")
    e_bad.start()
    time.sleep(0.05)
    e_good.start()
    errors, results = _run_clients(b, n_threads=4, n_req=40)
    e_good.stop()
    e_bad.stop()
    b.shutdown()
    # the bad device failed at most its 2 batches (their requests see an error), then left
    assert not e_bad.healthy() and e_good.healthy() and g.healthy() == 1
    assert e_bad.stats()["failed_batches"] == 2
    assert len(errors) <= 2 * MAXB and all(err == ("wait", rt.ST_ERROR) for err in errors)
    assert len(results) + len(errors) == 4 * 40 and all(results)


def test_last_executor_giving_up_shuts_the_batcher_so_waiters_do_not_hang():
    b = _batcher()
    g = rt.ExecGroup()
    bad = rt.FakeBackend(nslots=2, item_bytes=ITEM, max_batch=MAXB, out_cols=COLS, fail_every=1)
    e = rt.Executor(b, bad, g, name="bad", max_failures=1)
    e.start()
    errors, results = _run_clients(b, n_threads=3, n_req=10)
    e.stop()
    assert not results and len(errors) == 30
    assert g.healthy() == 0
    assert {k for k, _ in errors} <= {"wait", "submit"}


def test_injected_fault_then_recovery_and_trace_statuses():
    b = _batcher()
    g = rt.ExecGroup()
    f = rt.FakeBackend(nslots=3, item_bytes=ITEM, max_batch=MAXB, out_cols=COLS, latency_us=50)
    e = rt.Executor(b, f, g, name="inj", fail_batches=1, delay_us=100)
    e.start()
    errors, results = _run_clients(b, n_threads=2, n_req=20)
    e.stop()
    b.shutdown()
    assert e.healthy() and e.stats()["failed_batches"] == 1
    assert len(errors) >= 1 and len(results) + len(errors) == 40 and all(results)
    assert [t["status"] for t in e.recent(1000)].count(rt.ST_ERROR) == 1


@pytest.mark.parametrize("nslots", [1, 4])
def test_stop_drains_in_flight_batches(nslots):
    b = _batcher()
    g = rt.ExecGroup()
    f = rt.FakeBackend(nslots=nslots, item_bytes=ITEM, max_batch=MAXB, out_cols=COLS, latency_us=2000)
    e = rt.Executor(b, f, g, name="drain")
    e.start()
    errors, results = [], []
    th = threading.Thread(target=_client, args=(b, 1, 10, errors, results))
    th.start()
    time.sleep(0.02)
    e.stop()                     # joins after completing what was issued
    b.shutdown()
    th.join(30)
    assert not th.is_alive()
    assert all(results) and len(results) + len(errors) == 10
    assert all(err[1] in (rt.ST_SHUTDOWN, rt.ST_ERROR) for err in errors)


def test_device_resident_items_ride_issue_dev_beside_host_rows():
    """submit_device (serving_image rows the GPU resized) and host submits share batches: the
    executor hands the device rows to the backend's issue_dev as pieces (the fake backend's
    "device" memory is host memory) and every request still gets its own rows back."""
    b = _batcher()
    g = rt.ExecGroup()
    f = rt.FakeBackend(nslots=2, item_bytes=ITEM, max_batch=MAXB, out_cols=COLS, latency_us=200)
    ex = rt.Executor(b, f, g, name="fake-dev")
    ex.start()
    errors, results, keep = [], [], []

    def client(seed, device):
        rng = np.random.default_rng(seed)
        for _ in range(40):
            n = int(rng.integers(1, 4))
            vals = rng.integers(0, 200, size=n).astype(np.uint8)
            data = np.repeat(vals, ITEM).astype(np.uint8)
            keep.append(data)
            t = b.submit_device(data.ctypes.data, n, 0) if device else b.submit(data, n, 0)
            out = np.zeros((n, COLS), np.float32)
            if t < 0 or b.wait(t, out) != rt.ST_OK:
                errors.append(seed)
                continue
            want = vals[:, None].astype(np.float32) + np.arange(COLS, dtype=np.float32)[None]
            results.append(bool(np.array_equal(out, want)))

    ths = [threading.Thread(target=client, args=(s, s % 2 == 0)) for s in range(6)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    ex.stop()
    b.shutdown()
    assert not errors and len(results) == 240 and all(results)
    assert f.dev_pieces > 0


def test_batch_lists_device_items_for_the_backend():
    """Only native executors take device-resident rows; the batch fails instead of running on
    whatever the staging held."""
    b = _batcher()
    data = np.full(ITEM, 7, np.uint8)
    t = b.submit_device(data.ctypes.data, 1, 0)
    batch = b.next_batch(0, 1000, True)
    assert batch is not None and batch.dev_src == [data.ctypes.data]
    b.finish(batch, 0, rt.ST_ERROR)
    assert b.wait(t, np.zeros((1, COLS), np.float32)) == rt.ST_ERROR
