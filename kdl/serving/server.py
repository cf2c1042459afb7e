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
from .grpc_server import build_grpc_server
from .logs import StatsLogger, setup_logging
from .model_repo import ModelManager
from .rest import start_rest_server

log = logging.getLogger("kdl.serving")


class ModelServer:
    def __init__(self, cfg: ServerConfig):
        self.cfg = cfg
        self.manager = ModelManager(cfg)
        self.grpc = None
        self.rest = None
        self.grpc_port = None
        self.rest_port = None

    def start(self, block_until_loaded: bool = True) -> "ModelServer":
        cfg = self.cfg
        # serve health/status immediately; Predict returns UNAVAILABLE until loaded
        reuse = cfg.gpu_index >= 0           # a child of the --procs launcher: ports are shared
        self.grpc, self.grpc_port, _ = build_grpc_server(self.manager, cfg.host, cfg.port, cfg.grpc_max_threads,
                                                         reuse_port=reuse, f32_exact_u8=cfg.f32_exact_u8)
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


def launch_procs(argv: list[str], cfg: ServerConfig) -> int:
    """``--procs N``: one server process per GPU on this node, all on the same gRPC / REST ports
    (SO_REUSEPORT: the kernel spreads client connections over them). The launcher itself never
    touches a GPU; it forwards SIGTERM / SIGINT, and when one child dies it stops the others and
    exits with that child's status, so the pod restarts as a whole (k8s restartPolicy)."""
    if cfg.port == 0 or cfg.rest_api_port < 0:
        raise SystemExit("--procs needs fixed ports (every process binds the same one)")
    base = strip_flags(argv, ("--procs", "--gpu_index"))
    kids = [subprocess.Popen([sys.executable, "-m", "kdl.serving", *base, "--procs=1", f"--gpu_index={i}"])
            for i in range(cfg.procs)]
    log.info("kdl model server: %d processes (pids %s) sharing gRPC :%d / REST :%d", cfg.procs,
             [k.pid for k in kids], cfg.port, cfg.rest_api_port)
    return _supervise(kids)


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
    elif cfg.procs > 1:
        return launch_procs(argv, cfg)
    srv = ModelServer(cfg).start(block_until_loaded=False)
    if cfg.stats_log_interval_s > 0:
        StatsLogger(cfg.stats_log_interval_s).start()
    done = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: done.set())
    done.wait()
    srv.stop()
    return 0
