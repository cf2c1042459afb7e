"""Prometheus-text metrics for the model server (SURVEY.md §5 observability).

TF-Serving exposes ``/monitoring/prometheus/metrics`` on its REST port when
monitoring is configured; the same path is served here with request counts,
latency and batch-size histograms, queue depth and per-stage executor timings.
The reference itself has no metrics (`model_server.py:1-70`).
"""
from __future__ import annotations

import bisect
import threading
from collections import defaultdict

LAT_BUCKETS_MS = [0.5, 1, 2, 3, 5, 7.5, 10, 15, 20, 30, 50, 75, 100, 200, 500, 1000, 2000, 5000, 20000]
BATCH_BUCKETS = [1, 2, 4, 8, 16, 32, 64, 128, 256]


class Histogram:
    def __init__(self, buckets):
        self.buckets = list(buckets)
        self.counts = [0] * (len(self.buckets) + 1)
        self.sum = 0.0
        self.n = 0
        self.samples: list[float] = []

    def observe(self, v: float) -> None:
        self.counts[bisect.bisect_left(self.buckets, v)] += 1
        self.sum += v
        self.n += 1
        if len(self.samples) < 100_000:
            self.samples.append(v)

    def quantile(self, q: float) -> float:
        if self.n and len(self.samples) < min(self.n, 100_000):
            # counts merged from native histograms (merge) carry no samples: the upper bound of
            # the bucket holding the q-th observation
            acc, want = 0, q * self.n
            for b, c in zip(self.buckets + [float("inf")], self.counts):
                acc += c
                if acc >= want and c:
                    return float(b)
        if not self.samples:
            return 0.0
        s = sorted(self.samples)
        return s[min(len(s) - 1, int(q * len(s)))]

    def merge(self, counts, total: float) -> None:
        """Add a native histogram's per-bucket counts (same buckets, +Inf last) and sum."""
        for i, c in enumerate(counts):
            self.counts[i] += c
        self.n += sum(counts)
        self.sum += total


class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.counters: dict[tuple, float] = defaultdict(float)
        self.hists: dict[tuple, Histogram] = {}
        self.gauges: dict[tuple, callable] = {}
        self.collectors: dict[str, callable] = {}     # key -> fn() -> list of exposition lines
        self.pollers: dict[str, callable] = {}        # key -> fn(): folds native counters in (inc / merge_hist)

    def inc(self, name: str, value: float = 1.0, **labels) -> None:
        with self._lock:
            self.counters[(name, tuple(sorted(labels.items())))] += value

    def observe(self, name: str, value: float, buckets=LAT_BUCKETS_MS, **labels) -> None:
        key = (name, tuple(sorted(labels.items())))
        with self._lock:
            h = self.hists.get(key)
            if h is None:
                h = self.hists[key] = Histogram(buckets)
            h.observe(value)

    def merge_hist(self, name: str, counts, total: float, buckets=LAT_BUCKETS_MS, **labels) -> None:
        key = (name, tuple(sorted(labels.items())))
        with self._lock:
            h = self.hists.get(key)
            if h is None:
                h = self.hists[key] = Histogram(buckets)
            h.merge(counts, total)

    def poller(self, key: str, fn) -> None:
        """Register fn(), run before every render / snapshot (native front-end counters)."""
        self.pollers[key] = fn

    def drop_poller(self, key: str) -> None:
        self.pollers.pop(key, None)

    def _poll(self) -> None:
        for fn in list(self.pollers.values()):
            try:
                fn()
            except Exception:  # noqa: BLE001 - a broken poller must not break scraping
                pass

    def gauge(self, name: str, fn, **labels) -> None:
        self.gauges[(name, tuple(sorted(labels.items())))] = fn

    def collector(self, key: str, fn) -> None:
        """Register fn() -> [exposition lines] (native executor histograms), replacing ``key``'s."""
        self.collectors[key] = fn

    def drop_collector(self, key: str) -> None:
        self.collectors.pop(key, None)

    def hist(self, name: str, **labels) -> Histogram | None:
        return self.hists.get((name, tuple(sorted(labels.items()))))

    @staticmethod
    def _lbl(labels, extra=()) -> str:
        items = list(labels) + list(extra)
        if not items:
            return ""
        return "{" + ",".join(f'{k}="{v}"' for k, v in items) + "}"

    def render(self) -> str:
        self._poll()
        out = []
        with self._lock:
            for (name, labels), v in sorted(self.counters.items()):
                out.append(f"{name}{self._lbl(labels)} {v:g}")
            for (name, labels), h in sorted(self.hists.items()):
                acc = 0
                for b, c in zip(h.buckets + ["+Inf"], h.counts):
                    acc += c
                    out.append(f"{name}_bucket{self._lbl(labels, [('le', b)])} {acc}")
                out.append(f"{name}_sum{self._lbl(labels)} {h.sum:g}")
                out.append(f"{name}_count{self._lbl(labels)} {h.n}")
            gauges = list(self.gauges.items())
            collectors = list(self.collectors.values())
        for (name, labels), fn in sorted(gauges, key=lambda kv: kv[0]):
            try:
                out.append(f"{name}{self._lbl(labels)} {float(fn()):g}")
            except Exception:  # noqa: BLE001 - a broken gauge must not break scraping
                pass
        for fn in collectors:
            try:
                out.extend(fn())
            except Exception:  # noqa: BLE001
                pass
        return "\n".join(out) + "\n"

    def snapshot(self) -> dict:
        """Counters, histogram summaries (count, mean, p50, p99) and gauges as one JSON-able
        dict (the periodic "stats" log record). Reading a rate gauge here starts its next
        window, like a scrape does."""
        def key(name, labels):
            return name + ("{" + ",".join(f"{k}={v}" for k, v in labels) + "}" if labels else "")
        self._poll()
        out: dict = {"counters": {}, "histograms": {}, "gauges": {}}
        with self._lock:
            for (name, labels), v in sorted(self.counters.items()):
                out["counters"][key(name, labels)] = v
            for (name, labels), h in sorted(self.hists.items()):
                out["histograms"][key(name, labels)] = {
                    "count": h.n, "mean": h.sum / h.n if h.n else 0.0, "p50": h.quantile(0.5), "p99": h.quantile(0.99)}
            gauges = list(self.gauges.items())
        for (name, labels), fn in sorted(gauges, key=lambda kv: kv[0]):
            try:
                out["gauges"][key(name, labels)] = float(fn())
            except Exception:  # noqa: BLE001 - a broken gauge must not break the record
                pass
        return out


METRICS = Metrics()
