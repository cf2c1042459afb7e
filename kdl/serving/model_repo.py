"""Versioned model repository: ``<model_base_path>/<int version>/``.

TF-Serving's FileSystemStoragePathSource polls the base path and serves the
highest numeric version ("latest" policy); the reference copies its SavedModel
to ``/models/clothing-model/1`` (`tf-serving.dockerfile:4-5`). This manager does
the same: initial load, optional polling (``--file_system_poll_wait_seconds``),
load-new-then-retire-old so there is never a gap, and per-version status for
``ModelService/GetModelStatus``.
"""
from __future__ import annotations

import logging
import threading
import time
from pathlib import Path

from .backend import Servable, ServingError, load_version_dir, pick_devices
from .config import ServerConfig

log = logging.getLogger("kdl.serving")

START, LOADING, AVAILABLE, UNLOADING, END = 10, 20, 30, 40, 50
STATE_NAMES = {0: "UNKNOWN", START: "START", LOADING: "LOADING", AVAILABLE: "AVAILABLE",
               UNLOADING: "UNLOADING", END: "END"}


def list_versions(base: Path) -> list[int]:
    if not base.is_dir():
        return []
    return sorted(int(p.name) for p in base.iterdir() if p.is_dir() and p.name.isdigit())


def latest_version_source(cfg: ServerConfig):
    """The ModelSource of the version the manager's initial load would serve (the rccl group's
    rank 0 hands it to the followers before serving: serving/dp.py)."""
    base = Path(cfg.model_base_path)
    versions = list_versions(base) or ([1] if cfg.synthetic else [])
    if not versions:
        raise FileNotFoundError(f"no versions under {base} (use --synthetic_model for random weights)")
    return load_version_dir(base / str(versions[-1]), synthetic=cfg.synthetic)


class ModelManager:
    def __init__(self, cfg: ServerConfig):
        self.cfg = cfg
        self.name = cfg.model_name
        self.base = Path(cfg.model_base_path)
        self.devices = pick_devices(cfg)
        self._lock = threading.RLock()
        self.servables: dict[int, Servable] = {}
        self.states: dict[int, tuple[int, str]] = {}   # version -> (state, error message)
        self._stop = threading.Event()
        self._poller: threading.Thread | None = None
        # called (no arguments) whenever the set of live versions changes: the native gRPC
        # front-end drops its cached routes (serving/native_front.py)
        self.listeners: list = []

    # ------------------------------------------------------------ loading
    def load_initial(self) -> None:
        versions = list_versions(self.base)
        if not versions:
            if not self.cfg.synthetic:
                raise FileNotFoundError(f"no versions under {self.base} (use --synthetic_model for random weights)")
            versions = [1]
        self._load(versions[-1])

    def _load(self, v: int) -> None:
        with self._lock:
            # a version already live or being loaded by another thread (the version poller can
            # fire while the initial load of the same version is still building its engines)
            if v in self.servables or self.states.get(v, (None, ""))[0] == LOADING:
                return
            self.states[v] = (LOADING, "")
        t0 = time.perf_counter()
        try:
            src = load_version_dir(self.base / str(v), synthetic=self.cfg.synthetic)
            s = Servable(self.name, v, src, self.cfg, self.devices)
        except Exception as e:  # noqa: BLE001
            log.exception("loading %s version %d failed", self.name, v)
            with self._lock:
                self.states[v] = (END, f"{type(e).__name__}: {e}")
            raise
        with self._lock:
            self.servables[v] = s
            self.states[v] = (AVAILABLE, "")
            old = [k for k in self.servables if k != v]
        self._changed()
        log.info("loaded %s version %d (%s) on %s in %.1fs", self.name, v, src.origin,
                 f"gpus {self.devices}" if self.devices else "cpu", time.perf_counter() - t0)
        for k in old:  # latest policy: retire older versions once the new one is live
            self._unload(k)

    def _unload(self, v: int) -> None:
        with self._lock:
            s = self.servables.pop(v, None)
            self.states[v] = (UNLOADING, "")
        self._changed()
        if s is not None:
            s.close()
        with self._lock:
            self.states[v] = (END, "")

    def _changed(self) -> None:
        for fn in list(self.listeners):
            try:
                fn()
            except Exception:  # noqa: BLE001 - a listener must not break loading
                log.exception("model-change listener failed")

    def reload(self) -> None:
        versions = list_versions(self.base)
        if versions and versions[-1] not in self.servables:
            self._load(versions[-1])

    def start_polling(self) -> None:
        if self.cfg.file_system_poll_wait_seconds <= 0:
            return

        def loop():
            while not self._stop.wait(self.cfg.file_system_poll_wait_seconds):
                try:
                    self.reload()
                except Exception:  # noqa: BLE001 - keep serving the current version
                    pass
        self._poller = threading.Thread(target=loop, name="model-poller", daemon=True)
        self._poller.start()

    def close(self) -> None:
        self._stop.set()
        for v in list(self.servables):
            self._unload(v)

    # ------------------------------------------------------------ lookup
    def get(self, name: str, version: int | None = None, label: str | None = None) -> Servable:
        if name != self.name:
            raise ServingError("NOT_FOUND", f"Servable not found for request: Latest({name})")
        with self._lock:
            if not self.servables:
                raise ServingError("UNAVAILABLE", f"no version of {name} is available yet")
            if label:
                if label not in ("stable", "latest"):
                    raise ServingError("NOT_FOUND", f"unknown version label {label}")
                return self.servables[max(self.servables)]
            if version is not None and version >= 0:
                s = self.servables.get(version)
                if s is None:
                    raise ServingError("NOT_FOUND", f"Servable not found for request: Specific({name}, {version})")
                return s
            return self.servables[max(self.servables)]

    def ready(self) -> bool:
        """A version is loaded (graphs captured) and it still has a healthy device."""
        with self._lock:
            servables = list(self.servables.values())
        return bool(servables) and all(s.healthy() for s in servables)

    def device_alive(self) -> bool:
        """A version is loaded and its device still works (Servable.device_alive): one signature
        losing its executors (e.g. a shape-specific kernel fault) while another keeps serving does
        not make the process useless; every used signature failing does (server._watch_devices)."""
        with self._lock:
            servables = list(self.servables.values())
        return bool(servables) and all(s.device_alive() for s in servables)

    def status(self, version: int | None = None) -> list[tuple[int, int, str]]:
        with self._lock:
            items = sorted(self.states.items())
        if version is not None and version >= 0:
            items = [kv for kv in items if kv[0] == version]
            if not items:
                raise ServingError("NOT_FOUND", f"Could not find version {version} of model {self.name}")
        return [(v, st, msg) for v, (st, msg) in items]
