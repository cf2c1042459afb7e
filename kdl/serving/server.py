"""``tensorflow_model_server`` replacement entry point (``python -m kdl.serving``).

Same flags/env as the reference's TF-Serving container (`tf-serving.dockerfile:2-5`):
gRPC on --port (8500), REST on --rest_api_port (8501), model from
--model_base_path / $MODEL_BASE_PATH/$MODEL_NAME.
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import sys
import threading
import time

from .config import ServerConfig, config_from_args
from .grpc_server import Servicer, build_grpc_server
from .logs import StatsLogger, setup_logging
from .model_repo import ModelManager
from .rest import start_rest_server

log = logging.getLogger("kdl.serving")


class ModelServer:
    def __init__(self, cfg: ServerConfig):
        self.cfg = cfg
        self.manager = ModelManager(cfg)
        self.grpc = None
        self.native = None                   # native gRPC front-end (serving/native_front.py)
        self.rest = None
        self.grpc_port = None
        self.rest_port = None

    def start(self, block_until_loaded: bool = True) -> "ModelServer":
        cfg = self.cfg
        # serve health/status immediately; Predict returns UNAVAILABLE until loaded
        reuse = cfg.gpu_index >= 0           # a child of the --procs launcher: ports are shared
        if cfg.grpc_frontend == "native":
            from . import native_front
            ok, why = native_front.available()
            if ok:
                self.native = native_front.NativeFront(self.manager, Servicer(self.manager, cfg.f32_exact_u8),
                                                       cfg.host, cfg.port, io_threads=cfg.grpc_io_threads,
                                                       slow_threads=cfg.grpc_max_threads,
                                                       f32_exact_u8=cfg.f32_exact_u8,
                                                       max_request_bytes=cfg.grpc_max_request_bytes,
                                                       reuse_port=reuse)
                self.grpc_port = self.native.port
            else:
                log.warning("native gRPC front-end unavailable (%s): serving gRPC with grpcio", why)
        if self.native is None:
            self.grpc, self.grpc_port, _ = build_grpc_server(self.manager, cfg.host, cfg.port, cfg.grpc_max_threads,
                                                             reuse_port=reuse, f32_exact_u8=cfg.f32_exact_u8,
                                                             max_request_bytes=cfg.grpc_max_request_bytes)
            self.grpc.start()
        if cfg.rest_api_port:
            self.rest = start_rest_server(self.manager, cfg.host, cfg.rest_api_port, reuse_port=reuse,
                                          f32_exact_u8=cfg.f32_exact_u8)
            self.rest_port = self.rest.server_address[1]
        def load():
            try:
                self.manager.load_initial()
            finally:
                self.manager.start_polling()     # after the initial load: never a second loader
        loader = threading.Thread(target=load, name="model-loader", daemon=True)
        loader.start()
        if block_until_loaded:
            loader.join()
            if not self.manager.ready():
                raise RuntimeError("model failed to load; see log")
        log.info("kdl model server: gRPC :%s  REST :%s  model %s from %s", self.grpc_port, self.rest_port,
                 cfg.model_name, cfg.model_base_path)
        return self

    def stop(self, grace: float = 2.0) -> None:
        if self.native:
            self.native.stop()
        if self.grpc:
            self.grpc.stop(grace)
        if self.rest:
            self.rest.shutdown()
        self.manager.close()


def _supervise(kids: list, stop_first: list | None = None) -> int:
    """Forward SIGTERM / SIGINT (to ``stop_first`` only, when given: the rccl group's rank 0,
    whose stop broadcast ends the followers), stop the rest when one child dies, and exit with
    the first failing child's status."""
    stopping = threading.Event()
    targets = stop_first if stop_first is not None else kids

    def forward(signum, _frame):
        stopping.set()
        for k in targets:
            if k.poll() is None:
                k.send_signal(signum)
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, forward)
    rc = 0
    while True:
        dead = [k for k in kids if k.poll() is not None]
        if dead or stopping.is_set():
            rc = next((k.returncode for k in dead if k.returncode), 0)
            break
        time.sleep(0.2)
    if stop_first is not None:
        for k in stop_first:
            if k.poll() is None:
                k.terminate()
        deadline = time.time() + 30
        while time.time() < deadline and any(k.poll() is None for k in kids):
            time.sleep(0.2)
    for k in kids:
        if k.poll() is None:
            k.terminate() if stop_first is None else k.kill()
    for k in kids:
        try:
            k.wait(timeout=30)
        except subprocess.TimeoutExpired:
            k.kill()
    return rc or next((k.returncode for k in kids if k.returncode and k.returncode > 0), 0)


def strip_flags(argv: list[str], names: tuple[str, ...]) -> list[str]:
    """``argv`` without the value-taking flags ``names``, in either form: ``--procs=8`` and
    ``--procs 8`` (the child re-parses strictly, so a stray value token would kill it)."""
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        flag = a.split("=", 1)[0]
        if flag in names:
            skip = "=" not in a
            continue
        out.append(a)
    return out


def launch_dp(argv: list[str], cfg: ServerConfig) -> int:
    """``--scatter rccl``: rank 0 (this node's one front-end) + a follower per further GPU in
    one torch.distributed group on 127.0.0.1 (serving/dp.py)."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    base = strip_flags(argv, ("--dp_rank", "--dp_world", "--procs", "--gpu_index"))
    kids = []
    for r in range(cfg.dp_world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(cfg.dp_world), LOCAL_RANK=str(r))
        kids.append(subprocess.Popen([sys.executable, "-m", "kdl.serving", *base, f"--dp_world={cfg.dp_world}",
                                      f"--dp_rank={r}"], env=env))
    log.info("kdl model server: rccl data-parallel group of %d (pids %s), front-end = rank 0", cfg.dp_world,
             [k.pid for k in kids])
    return _supervise(kids, stop_first=kids[:1])


class ProcsSupervisor:
    """``--procs N`` launcher state: one child per GPU slot, each replaced by a FRESH process
    (never a re-exec: the launcher itself never touches a GPU) when it dies, while the other
    slots keep serving on the shared ports. This is per-GPU fault isolation for the topology
    that ships (deploy/k8s: --procs=8); the reference's only resilience is the Deployment
    controller restarting the whole pod (/root/reference/tf-serving-clothing-model-deployment.yaml:1-8).

    A slot that keeps dying (more than ``max_restarts`` within ``window_s``) is a crash loop:
    the launcher then stops everything and exits with that child's status, so k8s restarts the
    pod. Restarts back off exponentially (``backoff_s`` doubling, capped at 30 s)."""

    def __init__(self, cmd_for, n: int, max_restarts: int = 5, window_s: float = 300.0, backoff_s: float = 1.0):
        self.cmd_for, self.n = cmd_for, n
        self.max_restarts, self.window_s, self.backoff_s = max_restarts, window_s, backoff_s
        self.kids: list = [None] * n
        self.restarts: list[list[float]] = [[] for _ in range(n)]     # restart times per slot
        self.due: list[float | None] = [None] * n                        # pending restart time
        self.stopping = threading.Event()

    def spawn(self, i: int) -> None:
        cmd, env = self.cmd_for(i, len(self.restarts[i]))
        self.kids[i] = subprocess.Popen(cmd, env=env)

    def step(self, now: float) -> int | None:
        """One supervision tick: replace dead children; returns an exit status to give up with."""
        for i, k in enumerate(self.kids):
            if self.due[i] is not None:
                if now >= self.due[i]:
                    self.due[i] = None
                    self.restarts[i].append(now)
                    self.spawn(i)
                    log.warning("kdl launcher: GPU slot %d restarted as pid %d (restart %d)", i, self.kids[i].pid,
                                len(self.restarts[i]))
                continue
            if k is None or k.poll() is None:
                continue
            recent = [t for t in self.restarts[i] if now - t < self.window_s]
            if len(recent) >= self.max_restarts:
                log.error("kdl launcher: GPU slot %d crash loop (%d restarts in %.0f s, last status %s): giving up",
                          i, len(recent), self.window_s, k.returncode)
                return k.returncode or 1
            delay = min(30.0, self.backoff_s * (2 ** len(recent)))
            log.warning("kdl launcher: GPU slot %d (pid %d) exited with status %s; the other %d slot(s) keep "
                        "serving, replacing it in %.1f s", i, k.pid, k.returncode, self.n - 1, delay)
            self.due[i] = now + delay
        return None

    def run(self) -> int:
        def forward(signum, _frame):
            self.stopping.set()
            for k in self.kids:
                if k is not None and k.poll() is None:
                    k.send_signal(signum)
        for sig in (signal.SIGINT, signal.SIGTERM):
            signal.signal(sig, forward)
        for i in range(self.n):
            self.spawn(i)
        rc = 0
        while not self.stopping.is_set():
            r = self.step(time.monotonic())
            if r is not None:
                rc = r
                break
            time.sleep(0.2)
        for k in self.kids:
            if k is not None and k.poll() is None:
                k.terminate()
        for k in self.kids:
            if k is None:
                continue
            try:
                k.wait(timeout=30)
            except subprocess.TimeoutExpired:
                k.kill()
        return rc


def launch_procs(argv: list[str], cfg: ServerConfig) -> int:
    """``--procs N``: one server process per GPU on this node, all on the same gRPC / REST ports
    (SO_REUSEPORT: the kernel spreads client connections over them). The launcher never touches
    a GPU; it forwards SIGTERM / SIGINT and replaces a child that dies (ProcsSupervisor). A child
    whose devices all went unhealthy exits by itself (EXIT_NO_DEVICE) so it is replaced too."""
    if cfg.port == 0 or cfg.rest_api_port < 0:
        raise SystemExit("--procs needs fixed ports (every process binds the same one)")
    base = strip_flags(argv, ("--procs", "--gpu_index"))

    def cmd_for(i: int, restarts: int):
        env = dict(os.environ, KDL_CHILD_RESTARTS=str(restarts))
        return [sys.executable, "-m", "kdl.serving", *base, "--procs=1", f"--gpu_index={i}"], env
    sup = ProcsSupervisor(cmd_for, cfg.procs, max_restarts=int(os.environ.get("KDL_MAX_RESTARTS", "5")),
                          backoff_s=float(os.environ.get("KDL_RESTART_BACKOFF_S", "1")))
    log.info("kdl model server: %d processes sharing gRPC :%d / REST :%d", cfg.procs, cfg.port, cfg.rest_api_port)
    return sup.run()


EXIT_NO_DEVICE = 4       # a --procs child with no healthy executor left: replace me


def _watch_devices(srv: "ModelServer", done: threading.Event, rc: list, grace_s: float = 1.0) -> None:
    """--procs child: once the model has served, a child whose executors all went unhealthy
    (no signature of any loaded version has a healthy executor left) stops accepting (closes
    its listening sockets) and exits EXIT_NO_DEVICE, so the launcher replaces it with a fresh
    process instead of leaving it to fail its share of connections. One failing signature
    alone does not recycle the child: its other signatures keep serving."""
    served, bad_since = False, None
    while not done.wait(0.2):
        ok = srv.manager.device_alive()
        served = served or ok
        if not served or ok:
            bad_since = None
            continue
        bad_since = bad_since or time.monotonic()
        if time.monotonic() - bad_since >= grace_s:
            log.error("kdl model server (GPU slot %d): no healthy device left; closing listeners and exiting %d",
                      srv.cfg.gpu_index, EXIT_NO_DEVICE)
            rc[0] = EXIT_NO_DEVICE
            done.set()


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    cfg = config_from_args(argv)
    setup_logging(cfg.log_format)
    if cfg.scatter == "rccl":
        import torch
        if cfg.dp_world <= 0:
            cfg.dp_world = max(1, torch.cuda.device_count()) if cfg.device != "cpu" else 1
        if cfg.dp_rank < 0:
            return launch_dp(argv, cfg)
        from . import dp
        if cfg.dp_rank > 0:
            return dp.follow(cfg, cfg.dp_rank, cfg.dp_world)
        # rank 0: the front-end. Load the model once, hand it to the group (C1), then serve
        # with the dp signature's batcher feeding collective steps. Hot reload: native path
        # only (the new version's DP executor re-runs C1 with the followers, serving/dp.py)
        dev = dp.init_group(cfg, 0, cfg.dp_world)
        cfg.gpu_index = dev.index if dev.type == "cuda" else -1
        if not dp.native_ok(cfg, dev):
            cfg.file_system_poll_wait_seconds = 0
        if cfg.dp_signature not in cfg.warm_signatures:
            cfg.warm_signatures.append(cfg.dp_signature)
        from .model_repo import latest_version_source
        dp.share_source(latest_version_source(cfg), dev)
        log.info("kdl model server: signature %s is served data parallel over %d GPUs (RCCL); every other "
                 "signature runs on rank 0's GPU alone (f32 requests of exact 8-bit pixels are routed to "
                 "the uint8 signatures by gRPC and REST alike)", cfg.dp_signature, cfg.dp_world)
    elif cfg.procs > 1:
        return launch_procs(argv, cfg)
    srv = ModelServer(cfg).start(block_until_loaded=False)
    if cfg.stats_log_interval_s > 0:
        StatsLogger(cfg.stats_log_interval_s).start()
    done = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: done.set())
    rc = [0]
    if cfg.gpu_index >= 0 and cfg.scatter != "rccl":
        threading.Thread(target=_watch_devices, args=(srv, done, rc), name="device-watch", daemon=True).start()
    done.wait()
    srv.stop(grace=0.5 if rc[0] else 2.0)
    return rc[0]
