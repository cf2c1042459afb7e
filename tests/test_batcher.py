"""Native dynamic batcher (TF-Serving BasicBatchScheduler semantics)."""
import threading
import time

import numpy as np
import pytest

rt = pytest.importorskip("kdl._rt")

ITEM = 16  # bytes per item in these tests


def _mk(max_bs=8, timeout_us=2000, sizes=(1, 2, 4, 8), cols=2, max_enq=100):
    return rt.DynamicBatcher(max_batch_size=max_bs, batch_timeout_us=timeout_us, max_enqueued_batches=max_enq,
                             allowed_batch_sizes=list(sizes), item_bytes=ITEM, out_cols=cols)


def _consumer(b, stop, seen, fn=lambda x: x):
    staging = np.zeros(8 * ITEM, np.uint8)
    out = np.zeros((8, 2), np.float32)
    while not stop.is_set():
        batch = b.next_batch(staging.ctypes.data, 20_000)
        if batch is None:
            continue
        seen.append((batch.n_real, batch.bucket, list(batch.n_items)))
        items = staging.reshape(8, ITEM)[:batch.bucket]
        out[:batch.bucket, 0] = items[:, 0]          # echo first byte of each item
        out[:batch.bucket, 1] = batch.id
        b.finish(batch, out.ctypes.data, rt.ST_OK)


def test_full_batches_and_results_routed_back():
    b = _mk(timeout_us=200_000)
    stop, seen = threading.Event(), []
    th = threading.Thread(target=_consumer, args=(b, stop, seen))
    th.start()
    results = {}

    def client(i, n):
        data = np.full(n * ITEM, i, np.uint8)
        t = b.submit(data, n, 0)
        out = np.zeros((n, 2), np.float32)
        assert b.wait(t, out) == rt.ST_OK
        results[i] = out.copy()

    ths = [threading.Thread(target=client, args=(i, 2)) for i in range(1, 9)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    stop.set()
    th.join()
    for i, out in results.items():
        assert (out[:, 0] == i).all(), (i, out)       # each request got its own rows back
    assert sum(n for n, _, _ in seen) == 16
    assert all(n <= 8 for n, _, _ in seen)
    st = b.stats()
    assert st["completed"] == 8 and st["items"] == 16


def test_timeout_flushes_partial_batch_into_bucket():
    b = _mk(timeout_us=1000)
    stop, seen = threading.Event(), []
    th = threading.Thread(target=_consumer, args=(b, stop, seen))
    th.start()
    data = np.full(3 * ITEM, 5, np.uint8)
    t0 = time.perf_counter()
    t = b.submit(data, 3, 0)
    out = np.zeros((3, 2), np.float32)
    assert b.wait(t, out) == rt.ST_OK
    assert time.perf_counter() - t0 < 1.0
    stop.set()
    th.join()
    assert seen[0] == (3, 4, [3])          # 3 real items padded to the 4-bucket
    assert b.bucket_for(5) == 8 and b.bucket_for(1) == 1


def test_eager_dispatch_skips_the_timeout_when_idle():
    """eager next_batch (the executor's device is idle) returns a partial batch at once;
    the non-eager call waits the batch timeout out first."""
    b = _mk(timeout_us=500_000)
    data = np.full(3 * ITEM, 7, np.uint8)
    staging = np.zeros(8 * ITEM, np.uint8)
    t = b.submit(data, 3, 0)
    t0 = time.perf_counter()
    assert b.next_batch(staging.ctypes.data, 0) is None          # not full, not timed out
    batch = b.next_batch(staging.ctypes.data, 0, True)
    assert time.perf_counter() - t0 < 0.25
    assert batch is not None and batch.n_real == 3 and batch.bucket == 4
    assert (staging[:3 * ITEM] == 7).all()
    b.finish(batch, np.zeros((4, 2), np.float32).ctypes.data, rt.ST_OK)
    assert b.wait(t, np.zeros((3, 2), np.float32)) == rt.ST_OK


def test_deadline_expires_queued_request():
    b = _mk(timeout_us=10_000_000)          # never flushes by timeout
    data = np.zeros(ITEM, np.uint8)
    t = b.submit(data, 1, rt.now_us() + 20_000)
    out = np.zeros((1, 2), np.float32)
    t0 = time.perf_counter()
    assert b.wait(t, out) == rt.ST_DEADLINE
    assert time.perf_counter() - t0 < 1.0
    assert b.stats()["expired"] == 1
    assert b.stats()["queue_items"] == 0


def test_rejects_oversize_and_queue_full():
    b = _mk(max_bs=4, sizes=(4,), max_enq=1)
    assert b.submit(np.zeros(8 * ITEM, np.uint8), 8, 0) == -rt.ST_ERROR
    ok = b.submit(np.zeros(4 * ITEM, np.uint8), 4, 0)
    assert ok > 0
    assert b.submit(np.zeros(ITEM, np.uint8), 1, 0) == -rt.ST_QUEUE_FULL
    b.shutdown()
    assert b.wait(ok, np.zeros((4, 2), np.float32)) == rt.ST_SHUTDOWN


def test_many_concurrent_clients_two_consumers():
    b = _mk(timeout_us=500)
    stop, seen = threading.Event(), []
    cons = [threading.Thread(target=_consumer, args=(b, stop, seen)) for _ in range(2)]
    for c in cons:
        c.start()
    errors = []

    def client(i):
        n = 1 + i % 4
        data = np.full(n * ITEM, i % 251, np.uint8)
        out = np.zeros((n, 2), np.float32)
        st = b.wait(b.submit(data, n, 0), out)
        if st != rt.ST_OK or not (out[:, 0] == i % 251).all():
            errors.append(i)

    ths = [threading.Thread(target=client, args=(i,)) for i in range(200)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    stop.set()
    for c in cons:
        c.join()
    assert not errors
    assert b.stats()["completed"] == 200


@pytest.mark.parametrize("threads", [1, 4])
def test_large_payloads_copied_in_parallel_pieces(threads):
    """Batches of several MB are copied into staging in 1 MiB pieces by up to copy_threads
    threads: every byte must land at its request's item offset (299x299x3 items)."""
    item = 299 * 299 * 3
    b = rt.DynamicBatcher(max_batch_size=8, batch_timeout_us=1_000_000, max_enqueued_batches=10,
                          allowed_batch_sizes=[8], item_bytes=item, out_cols=1, copy_threads=threads)
    rng = np.random.default_rng(threads)
    reqs = [rng.integers(0, 256, n * item, dtype=np.uint8) for n in (3, 1, 4)]
    tickets = [b.submit(r, len(r) // item, 0) for r in reqs]
    staging = np.zeros(8 * item, np.uint8)
    batch = b.next_batch(staging.ctypes.data, 1_000_000)
    assert batch is not None and batch.n_real == 8
    assert np.array_equal(staging, np.concatenate(reqs))
    out = np.zeros((8, 1), np.float32)
    b.finish(batch, out.ctypes.data, rt.ST_OK)
    for t, r in zip(tickets, reqs):
        assert b.wait(t, np.zeros((len(r) // item, 1), np.float32)) == rt.ST_OK
