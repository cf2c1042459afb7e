"""``tensorflow_model_server`` replacement entry point (``python -m kdl.serving``).

Same flags/env as the reference's TF-Serving container (`tf-serving.dockerfile:2-5`):
gRPC on --port (8500), REST on --rest_api_port (8501), model from
--model_base_path / $MODEL_BASE_PATH/$MODEL_NAME.
"""
from __future__ import annotations

import logging
import signal
import sys
import threading

from .config import ServerConfig, config_from_args
from .grpc_server import build_grpc_server
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
        self.grpc, self.grpc_port, _ = build_grpc_server(self.manager, cfg.host, cfg.port, cfg.grpc_max_threads)
        self.grpc.start()
        if cfg.rest_api_port:
            self.rest = start_rest_server(self.manager, cfg.host, cfg.rest_api_port)
            self.rest_port = self.rest.server_address[1]
        loader = threading.Thread(target=self.manager.load_initial, name="model-loader", daemon=True)
        loader.start()
        if block_until_loaded:
            loader.join()
            if not self.manager.ready():
                raise RuntimeError("model failed to load; see log")
        self.manager.start_polling()
        log.info("kdl model server: gRPC :%s  REST :%s  model %s from %s", self.grpc_port, self.rest_port,
                 cfg.model_name, cfg.model_base_path)
        return self

    def stop(self, grace: float = 2.0) -> None:
        if self.grpc:
            self.grpc.stop(grace)
        if self.rest:
            self.rest.shutdown()
        self.manager.close()


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s",
                        stream=sys.stdout)
    cfg = config_from_args(argv)
    srv = ModelServer(cfg).start(block_until_loaded=False)
    done = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: done.set())
    done.wait()
    srv.stop()
    return 0
