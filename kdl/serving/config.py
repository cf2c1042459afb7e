"""Model-server configuration: TF-Serving-compatible flags and env.

The reference runs ``tensorflow/serving:2.3.0`` whose entrypoint is
``tensorflow_model_server --port=8500 --rest_api_port=8501
--model_name=$MODEL_NAME --model_base_path=$MODEL_BASE_PATH/$MODEL_NAME``
(`tf-serving.dockerfile:2-5`). The same flags and env vars are
honoured here, plus MI355X-native knobs (devices, batching buckets, executors).
"""
from __future__ import annotations

import argparse
import os
import re
from dataclasses import dataclass, field


@dataclass
class BatchingParams:
    """TF-Serving BatchingParameters (text proto) subset."""
    max_batch_size: int = 32
    batch_timeout_micros: int = 2000
    max_enqueued_batches: int = 1000
    # TF-Serving: threads that process batches concurrently. kdl: concurrent batch executors,
    # spread over the GPUs (ServerConfig.executors_for); --executors_per_gpu overrides it
    num_batch_threads: int = 1
    allowed_batch_sizes: list[int] = field(default_factory=lambda: [1, 2, 4, 8, 16, 32])
    # kdl extension (not a TF-Serving knob): an executor whose device is idle takes whatever is
    # queued at once instead of waiting out batch_timeout_micros (work-conserving dispatch)
    eager_when_idle: bool = True

    @classmethod
    def parse(cls, text: str) -> "BatchingParams":
        """Parse the text-proto file format, e.g. ``max_batch_size { value: 32 }``."""
        p = cls()
        for key in ("max_batch_size", "batch_timeout_micros", "max_enqueued_batches", "num_batch_threads"):
            m = re.search(rf"{key}\s*\{{\s*value\s*:\s*(\d+)\s*\}}", text)
            if m:
                setattr(p, key, int(m.group(1)))
        sizes = [int(v) for v in re.findall(r"allowed_batch_sizes\s*:\s*(\d+)", text)]
        if sizes:
            p.allowed_batch_sizes = sizes
        else:
            p.allowed_batch_sizes = [b for b in p.allowed_batch_sizes if b <= p.max_batch_size]
        if p.allowed_batch_sizes and p.allowed_batch_sizes[-1] != p.max_batch_size:
            p.allowed_batch_sizes.append(p.max_batch_size)
        return p


@dataclass
class ServerConfig:
    port: int = 8500
    rest_api_port: int = 8501
    model_name: str = "clothing-model"
    model_base_path: str = "/models/clothing-model"
    enable_batching: bool = True
    batching: BatchingParams = field(default_factory=BatchingParams)
    file_system_poll_wait_seconds: int = 1
    grpc_max_threads: int = 64
    # native: the C++ gRPC front-end (runtime/grpc_front.h; Predict fast path without Python);
    # python: the grpcio server. Falls back to python when libnghttp2 is missing
    grpc_frontend: str = "native"
    grpc_io_threads: int = 4      # native front-end epoll workers (one SO_REUSEPORT listener each)
    # largest request message either front-end accepts (RESOURCE_EXHAUSTED beyond it): one f32
    # batch-32 299x299 request is 34.3 MB
    grpc_max_request_bytes: int = 64 << 20
    rest_api_num_threads: int = 16
    device: str = "auto"          # auto | cpu | gpu | null (front-end ceiling: zero-latency fake device)
    gpus: int = 0                 # 0 = all visible
    executors_per_gpu: int = 0    # 0 = derive from batching.num_batch_threads (executors_for)
    synthetic: bool = False       # random-init weights when the repo has no artifact
    labels: list[str] = field(default_factory=list)
    host: str = "0.0.0.0"
    # MI355X-native engine knobs (SURVEY.md §5 "Config / flag system")
    dtype: str = "auto"           # auto | bf16 | fp16 | fp8: picks the family's engine variant
    graph: bool = True            # hipGraph replay per (bucket, slot); off = eager kernel launches
    stages: str = ""              # stage-pipeline cut ("" = the family's default, "none" = off)
    lanes: int = 1                # split-batch hipGraph lanes for the top bucket
    exec_depth: int = 2           # batches in flight per GPU executor
    # one-process-per-GPU serving (--procs N): N server processes share the gRPC / REST ports
    # through SO_REUSEPORT; process i serves GPU i % visible GPUs (gpu_index), -1 = all GPUs
    procs: int = 1
    gpu_index: int = -1
    warm_signatures: list[str] = field(default_factory=list)   # built at load, besides serving_default
    f32_exact_u8: bool = True    # f32 requests that are exactly x/127.5-1 of 8-bit pixels ride the uint8 path
    # --scatter rccl: ONE front-end (rank 0) + one process per GPU, batches scattered / logits
    # gathered over RCCL (serving/dp.py); host = every process ingests its own requests
    scatter: str = "host"
    dp_world: int = 0             # processes (GPUs) of the rccl group; 0 = every visible GPU
    dp_rank: int = -1             # set by the launcher
    dp_signature: str = "serving_uint8"
    log_format: str = "text"      # text | json (one JSON object per line, for log shippers)
    stats_log_interval_s: float = 0.0   # > 0: a "stats" log record (metrics snapshot) this often

    def executors_for(self, n_devices: int) -> int:
        """Executors per device: --executors_per_gpu when given, else TF-Serving's
        num_batch_threads (batches processed concurrently) spread over the devices."""
        if self.executors_per_gpu > 0:
            return self.executors_per_gpu
        # derived counts stop at 2 per GPU: each executor keeps a compute and a copy stream
        # busy, and a process gets GPU_MAX_HW_QUEUES = 4 hardware queues per device
        return min(2, max(1, -(-self.batching.num_batch_threads // max(1, n_devices))))

    def rank_buckets(self) -> list[int]:
        """Per-GPU graph buckets (the allowed batch sizes); the data-parallel signature's
        batcher forms batches of world x these (--scatter rccl)."""
        bp = self.batching
        return sorted(set(bp.allowed_batch_sizes)) if self.enable_batching else [bp.max_batch_size]

    def engine_kwargs(self) -> dict:
        return {"graph": self.graph, "stages": self.stages, "lanes": self.lanes, "depth": self.exec_depth}


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="kdl-model-server",
                                 description="MI355X-native TF-Serving-compatible model server")
    ap.add_argument("--port", type=int, default=8500)
    ap.add_argument("--rest_api_port", type=int, default=8501)
    ap.add_argument("--model_name", default=None)
    ap.add_argument("--model_base_path", default=None)
    ap.add_argument("--enable_batching", default="true")
    ap.add_argument("--batching_parameters_file", default=None)
    ap.add_argument("--file_system_poll_wait_seconds", type=int, default=1)
    ap.add_argument("--grpc_max_threads", type=int, default=64)
    ap.add_argument("--rest_api_num_threads", type=int, default=16)
    ap.add_argument("--grpc_frontend", choices=["native", "python"], default=None,
                    help="native: C++ HTTP/2 front-end whose Predict fast path parses, batches and answers "
                         "without Python; python: the grpcio server (env KDL_GRPC_FRONTEND, default native)")
    ap.add_argument("--grpc_max_request_bytes", type=int, default=None,
                    help="largest gRPC request message accepted, both front-ends (env KDL_GRPC_MAX_REQUEST_BYTES, "
                         "default 64 MiB; an f32 batch-32 Xception request is 34.3 MB)")
    ap.add_argument("--grpc_io_threads", type=int, default=None,
                    help="native front-end I/O threads (env KDL_GRPC_IO_THREADS, default 4)")
    ap.add_argument("--device", choices=["auto", "cpu", "gpu", "null"], default="auto",
                    help="null: the native executor over a zero-latency fake device (logits = first "
                         "input byte + class index) -- measures the serving front-end's own ceiling")
    ap.add_argument("--gpus", type=int, default=0)
    ap.add_argument("--executors_per_gpu", type=int, default=0,
                    help="batch executors per GPU (default: num_batch_threads of the batching "
                         "parameters file spread over the GPUs, at least 1)")
    ap.add_argument("--max_batch_size", type=int, default=None)
    ap.add_argument("--batch_timeout_micros", type=int, default=None)
    ap.add_argument("--eager_dispatch", default="true",
                    help="an idle executor takes whatever is queued at once instead of waiting out "
                         "batch_timeout_micros (kdl extension; 'false' = TF-Serving behaviour)")
    ap.add_argument("--allowed_batch_sizes", default=None, help="comma separated, e.g. 1,4,8,16,32")
    ap.add_argument("--synthetic_model", action="store_true")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--dtype", choices=["auto", "bf16", "fp16", "fp8"], default="auto",
                    help="compute dtype: selects the family's engine variant (resnet50: fp16 | bf16; "
                         "vit_b16: bf16 | fp8 e4m3 linears; xception / efficientnet_b7: bf16)")
    ap.add_argument("--graph", choices=["on", "off"], default="on",
                    help="replay one captured hipGraph per (batch bucket, slot); off = eager launches")
    ap.add_argument("--stages", default=None,
                    help="stage-pipeline cut step (default: the family's; 'none' disables)")
    ap.add_argument("--lanes", type=int, default=None, help="split-batch hipGraph lanes (top bucket)")
    ap.add_argument("--exec_depth", type=int, default=None, help="batches in flight per GPU executor")
    ap.add_argument("--procs", type=int, default=1,
                    help="server processes on this node (one per GPU): each binds the same ports with "
                         "SO_REUSEPORT, so the kernel spreads client connections over them; process i "
                         "serves GPU i (mod the visible GPUs)")
    ap.add_argument("--gpu_index", type=int, default=-1, help=argparse.SUPPRESS)   # set by the --procs launcher
    ap.add_argument("--f32_exact_u8", default=None, choices=["true", "false"],
                    help="serve an f32 request on the uint8 path when its values are exactly x/127.5-1 of "
                         "8-bit pixels (the reference gateway's request); env KDL_F32_EXACT_U8 (default true)")
    ap.add_argument("--warm_signatures", default="",
                    help="comma list of signatures whose engines / graphs are built at model load (like "
                         "TF-Serving warmup requests); serving_default always is")
    ap.add_argument("--scatter", choices=["host", "rccl"], default="host",
                    help="rccl: one front-end process scatters each batch over the node's GPUs and gathers "
                         "the logits on RCCL (one process per GPU, --dp_world of them); host: every server "
                         "process feeds its own GPU (see --procs)")
    ap.add_argument("--dp_world", type=int, default=0, help="GPUs of the --scatter rccl group (0 = all visible)")
    ap.add_argument("--dp_rank", type=int, default=-1, help=argparse.SUPPRESS)   # set by the rccl launcher
    ap.add_argument("--dp_signature", default="serving_uint8",
                    help="the signature served data parallel under --scatter rccl (others run on rank 0's GPU)")
    ap.add_argument("--log_format", choices=["text", "json"], default=None,
                    help="json: one JSON object per log line (env KDL_LOG_FORMAT)")
    ap.add_argument("--stats_log_interval_s", type=float, default=None,
                    help="log a metrics snapshot (requests, latency quantiles, batch sizes, queue depth, "
                         "per-GPU busy ratio) every N seconds; 0 = off (env KDL_STATS_LOG_INTERVAL_S)")
    return ap


def _truthy(v) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def config_from_args(argv=None, env=None) -> ServerConfig:
    env = os.environ if env is None else env
    a = build_parser().parse_args(argv)
    name = a.model_name or env.get("MODEL_NAME", "clothing-model")
    base = a.model_base_path or os.path.join(env.get("MODEL_BASE_PATH", "/models"), name)
    bp = BatchingParams()
    if a.batching_parameters_file:
        with open(a.batching_parameters_file) as f:
            bp = BatchingParams.parse(f.read())
    if a.max_batch_size:
        bp.max_batch_size = a.max_batch_size
        bp.allowed_batch_sizes = [b for b in bp.allowed_batch_sizes if b < a.max_batch_size] + [a.max_batch_size]
    if a.batch_timeout_micros is not None:
        bp.batch_timeout_micros = a.batch_timeout_micros
    bp.eager_when_idle = _truthy(a.eager_dispatch)
    if a.allowed_batch_sizes:
        bp.allowed_batch_sizes = sorted(int(x) for x in a.allowed_batch_sizes.split(","))
        bp.max_batch_size = bp.allowed_batch_sizes[-1]
    labels = [s for s in env.get("LABELS", "").split(",") if s]
    return ServerConfig(port=a.port, rest_api_port=a.rest_api_port, model_name=name, model_base_path=base,
                        enable_batching=_truthy(a.enable_batching), batching=bp,
                        file_system_poll_wait_seconds=a.file_system_poll_wait_seconds,
                        grpc_max_threads=a.grpc_max_threads, rest_api_num_threads=a.rest_api_num_threads,
                        grpc_frontend=a.grpc_frontend or env.get("KDL_GRPC_FRONTEND", "native"),
                        grpc_io_threads=(a.grpc_io_threads if a.grpc_io_threads is not None
                                         else int(env.get("KDL_GRPC_IO_THREADS", "4"))),
                        grpc_max_request_bytes=(a.grpc_max_request_bytes if a.grpc_max_request_bytes is not None
                                                else int(env.get("KDL_GRPC_MAX_REQUEST_BYTES", str(64 << 20)))),
                        device=a.device, gpus=a.gpus, executors_per_gpu=a.executors_per_gpu,
                        synthetic=a.synthetic_model or _truthy(env.get("KDL_SYNTHETIC_MODEL", "0")),
                        labels=labels, host=a.host, dtype=a.dtype, graph=a.graph == "on",
                        stages=a.stages if a.stages is not None else env.get("KDL_STAGES", ""),
                        lanes=a.lanes if a.lanes is not None else int(env.get("KDL_LANES", "1")),
                        exec_depth=a.exec_depth if a.exec_depth is not None else int(env.get("KDL_EXEC_DEPTH", "2")),
                        procs=max(1, a.procs), gpu_index=a.gpu_index,
                        warm_signatures=[s for s in a.warm_signatures.split(",") if s],
                        f32_exact_u8=(a.f32_exact_u8 or env.get("KDL_F32_EXACT_U8", "true")).lower() != "false",
                        scatter=a.scatter, dp_world=a.dp_world, dp_rank=a.dp_rank, dp_signature=a.dp_signature,
                        log_format=a.log_format or env.get("KDL_LOG_FORMAT", "text"),
                        stats_log_interval_s=(a.stats_log_interval_s if a.stats_log_interval_s is not None
                                              else float(env.get("KDL_STATS_LOG_INTERVAL_S", "0"))))
