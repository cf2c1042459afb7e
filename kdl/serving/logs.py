"""Structured logs for the model server (SURVEY.md §5 observability).

``--log_format json`` turns every log line into one JSON object (time, level, logger,
message, pid, and the record's ``extra`` fields), the shape log shippers on a
Kubernetes node ingest without parsing rules; ``--stats_log_interval_s N`` adds a
``"event": "stats"`` record every N seconds with the metrics snapshot (request
counts by code, latency p50 / p99, batch sizes, queue depth, per-GPU busy ratio).
The reference's only logging is Flask's debug server (`model_server.py:69-70`).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import threading
import time

from .metrics import METRICS

_STD = set(vars(logging.makeLogRecord({})).keys()) | {"message", "asctime"}


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": round(record.created, 6), "level": record.levelname, "logger": record.name,
             "msg": record.getMessage(), "pid": os.getpid()}
        for k, v in vars(record).items():
            if k not in _STD and not k.startswith("_"):
                d[k] = v
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d, default=str)


def setup_logging(fmt: str = "text", stream=None) -> None:
    h = logging.StreamHandler(stream or sys.stdout)
    if fmt == "json":
        h.setFormatter(JsonFormatter())
    else:
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(logging.INFO)


class StatsLogger(threading.Thread):
    """Logs ``METRICS.snapshot()`` every ``interval`` seconds as an ``event=stats`` record."""

    def __init__(self, interval: float, logger: logging.Logger | None = None):
        super().__init__(name="kdl-stats-log", daemon=True)
        self.interval = interval
        self.log = logger or logging.getLogger("kdl.serving.stats")
        self.stop = threading.Event()

    def run(self) -> None:
        while not self.stop.wait(self.interval):
            self.log.info("stats", extra={"event": "stats", "t": time.time(), **METRICS.snapshot()})
