"""Model-server flag parsing (SURVEY.md §5 "Config / flag system"): TF-Serving flags and
env (tf-serving.dockerfile:2-5 entrypoint), the batching-parameters text proto, and the
MI355X-native engine knobs (--dtype variant selection, --graph, --stages, --lanes,
--exec_depth)."""
import pytest

from kdl.engine import registry
from kdl.serving.config import BatchingParams, config_from_args


def test_tf_serving_flags_and_env():
    c = config_from_args(["--port", "9000", "--rest_api_port", "9001"],
                         env={"MODEL_NAME": "clothing-model", "MODEL_BASE_PATH": "/m"})
    assert (c.port, c.rest_api_port, c.model_name, c.model_base_path) == (9000, 9001, "clothing-model",
                                                                          "/m/clothing-model")
    assert c.enable_batching and c.graph and c.dtype == "auto"


def test_batching_parameters_text_proto(tmp_path):
    p = tmp_path / "batching.txt"
    p.write_text("max_batch_size { value: 16 }\nbatch_timeout_micros { value: 500 }\n"
                 "allowed_batch_sizes: 4\nallowed_batch_sizes: 16\n")
    c = config_from_args(["--batching_parameters_file", str(p)], env={})
    assert c.batching.max_batch_size == 16 and c.batching.batch_timeout_micros == 500
    assert c.batching.allowed_batch_sizes == [4, 16]
    assert BatchingParams.parse("max_batch_size { value: 8 }").allowed_batch_sizes == [1, 2, 4, 8]


def test_native_engine_flags():
    c = config_from_args(["--dtype", "fp8", "--graph", "off", "--stages", "none", "--lanes", "2",
                          "--exec_depth", "3"], env={})
    assert c.dtype == "fp8" and not c.graph
    assert c.engine_kwargs() == {"graph": False, "stages": "none", "lanes": 2, "depth": 3}
    # env fallbacks of the same knobs
    c = config_from_args([], env={"KDL_STAGES": "block7_sepconv1", "KDL_LANES": "2", "KDL_EXEC_DEPTH": "4"})
    assert c.engine_kwargs() == {"graph": True, "stages": "block7_sepconv1", "lanes": 2, "depth": 4}


def test_dtype_selects_engine_variant():
    assert registry.variant("resnet50", "auto") == "resnet50"
    assert registry.variant("resnet50", "fp16") == "resnet50"
    assert registry.variant("resnet50", "bf16") == "resnet50_bf16"
    assert registry.variant("vit_b16", "fp8") == "vit_b16_fp8"
    assert registry.variant("vit_b16_fp8", "bf16") == "vit_b16"
    assert registry.variant("xception", "bf16") == "xception"
    for fam in registry.models():
        assert registry.variant(fam, "auto") == fam
    with pytest.raises(ValueError):
        registry.variant("xception", "fp8")
    with pytest.raises(SystemExit):
        config_from_args(["--dtype", "int4"], env={})


def test_num_batch_threads_sets_concurrent_executors(tmp_path):
    """TF-Serving's num_batch_threads (batches processed concurrently) is honoured: it sets the
    executor count, spread over the GPUs, unless --executors_per_gpu is given."""
    from kdl.serving.config import config_from_args
    f = tmp_path / "batching.txt"
    f.write_text("max_batch_size { value: 32 }\nnum_batch_threads { value: 8 }\n")
    cfg = config_from_args([f"--batching_parameters_file={f}"], env={})
    assert cfg.batching.num_batch_threads == 8
    assert cfg.executors_for(8) == 1 and cfg.executors_for(4) == 2 and cfg.executors_for(1) == 2
    cfg = config_from_args([f"--batching_parameters_file={f}", "--executors_per_gpu=3"], env={})
    assert cfg.executors_for(8) == 3
    assert config_from_args([], env={}).executors_for(8) == 1


def test_json_logs_and_stats_snapshot():
    import io
    import json
    import logging

    from kdl.serving.config import config_from_args
    from kdl.serving.logs import StatsLogger, setup_logging
    from kdl.serving.metrics import Metrics

    cfg = config_from_args(["--log_format=json", "--stats_log_interval_s=0.05"], env={})
    assert cfg.log_format == "json" and cfg.stats_log_interval_s == 0.05
    assert config_from_args([], env={"KDL_LOG_FORMAT": "json"}).log_format == "json"
    assert config_from_args([], env={}).log_format == "text"
    buf = io.StringIO()
    old = logging.getLogger().handlers[:]
    try:
        setup_logging("json", buf)
        logging.getLogger("kdl.serving").info("loaded %s", "m", extra={"version": 3})
        rec = json.loads(buf.getvalue().splitlines()[-1])
        assert rec["msg"] == "loaded m" and rec["version"] == 3 and rec["level"] == "INFO" and rec["pid"] > 0
        m = Metrics()
        m.inc("kdl_requests_total", code="OK")
        for v in (1.0, 2.0, 3.0):
            m.observe("kdl_request_latency_ms", v)
        m.gauge("kdl_gpu_busy_ratio", lambda: 0.5, executor="gpu0")
        snap = m.snapshot()
        assert snap["counters"]["kdl_requests_total{code=OK}"] == 1
        h = snap["histograms"]["kdl_request_latency_ms"]
        assert h["count"] == 3 and h["p50"] == 2.0 and h["mean"] == 2.0
        assert snap["gauges"]["kdl_gpu_busy_ratio{executor=gpu0}"] == 0.5
        sl = StatsLogger(0.02)
        sl.start()
        import time
        time.sleep(0.15)
        sl.stop.set()
        sl.join(2)
        stats = [json.loads(l) for l in buf.getvalue().splitlines() if '"event": "stats"' in l]
        assert stats and "counters" in stats[0] and "gauges" in stats[0]
    finally:
        logging.getLogger().handlers[:] = old


def test_launcher_strips_both_flag_forms():
    """--procs / --dp_world children re-parse strictly: the launcher must drop a flag's value
    token in the space form too (kdl/serving/server.py strip_flags)."""
    from kdl.serving.config import config_from_args
    from kdl.serving.server import strip_flags
    argv = ["--procs", "8", "--port=8500", "--dp_world=4", "--gpu_index", "3", "--scatter", "rccl",
            "--dp_rank", "1", "--model_name", "m"]
    names = ("--dp_rank", "--dp_world", "--procs", "--gpu_index")
    out = strip_flags(argv, names)
    assert out == ["--port=8500", "--scatter", "rccl", "--model_name", "m"]
    cfg = config_from_args(out + ["--procs=1", "--gpu_index=0"])      # what a child parses
    assert cfg.procs == 1 and cfg.gpu_index == 0 and cfg.port == 8500
