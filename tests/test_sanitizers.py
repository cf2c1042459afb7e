"""Race detection / memory safety of the native runtime on CPU builds
(SURVEY.md §5): the DynamicBatcher stress test under ThreadSanitizer and under
AddressSanitizer + UndefinedBehaviorSanitizer, and the proto codec / SSTable /
snappy parsers fed malformed bytes under ASan+UBSan."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "kdl" / "csrc"
RT = [CSRC / "runtime" / n for n in ("batcher.cpp", "executor.cpp", "tfproto.cpp", "sstable.cpp", "dp_loop.cpp",
                                     "h2.cpp", "grpc_front.cpp", "grpc_load.cpp")]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
# TSAN: LLVM's runtime. GCC 11's libtsan does not intercept pthread_cond_clockwait (what
# libstdc++'s condition_variable::wait_for calls), so every timed wait is reported as a
# "double lock of a mutex" false positive.
CLANG = next((c for c in ("/opt/rocm/lib/llvm/bin/clang++", shutil.which("clang++")) if c and Path(c).exists()),
             None)


def _build(tmp_path, name, main, flags, cxx="g++"):
    exe = tmp_path / name
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, str(main),
           *[str(s) for s in RT], "-I", str(CSRC), "-o", str(exe), "-lpthread", "-ldl"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def _run(exe, *args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, timeout=300, env=e)


@pytest.mark.skipif(CLANG is None, reason="needs clang++ (LLVM TSAN runtime)")
def test_batcher_under_tsan(tmp_path):
    exe = _build(tmp_path, "stress_tsan", CSRC / "tests" / "batcher_stress.cpp", ["-fsanitize=thread"], cxx=CLANG)
    r = _run(exe, 8, 200, env={"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr
    # 256 KiB items: full batches take the persistent copy pool, from 3 consumers at once
    r = _run(exe, 6, 60, 262144, env={"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr


def test_batcher_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "stress_asan", CSRC / "tests" / "batcher_stress.cpp",
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    r = _run(exe, 8, 200, env={"ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    r = _run(exe, 6, 60, 262144, env={"ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(CLANG is None, reason="needs clang++ (LLVM TSAN runtime)")
def test_native_executor_under_tsan(tmp_path):
    exe = _build(tmp_path, "exec_tsan", CSRC / "tests" / "exec_stress.cpp", ["-fsanitize=thread"], cxx=CLANG)
    r = _run(exe, 8, 120, env={"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr


def test_native_executor_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "exec_asan", CSRC / "tests" / "exec_stress.cpp",
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    r = _run(exe, 8, 150, env={"ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(CLANG is None, reason="needs clang++ (LLVM TSAN runtime)")
@pytest.mark.parametrize("world", [2, 4])
def test_dp_loopback_under_tsan(tmp_path, world):
    """The data-parallel leader/follower state machine (dp_core.h) on the loopback platform:
    batcher + executor + leader heartbeat + follower threads + reload + a dead follower."""
    exe = _build(tmp_path, "dp_tsan", CSRC / "tests" / "dp_loop_stress.cpp", ["-fsanitize=thread"], cxx=CLANG)
    r = _run(exe, world, 3, 25, env={"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr


def test_dp_loopback_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "dp_asan", CSRC / "tests" / "dp_loop_stress.cpp",
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    r = _run(exe, 4, 3, 25, env={"ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(CLANG is None, reason="needs clang++ (LLVM TSAN runtime)")
def test_native_grpc_front_under_tsan(tmp_path):
    """The native gRPC front-end (grpc_front.h): epoll workers + slow pool + eventfd mailbox +
    batcher callbacks under fast- and slow-path load, routes flipping, stop with calls in flight."""
    exe = _build(tmp_path, "front_tsan", CSRC / "tests" / "front_stress.cpp", ["-fsanitize=thread"], cxx=CLANG)
    r = _run(exe, 4, 4, 2, env={"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr


def test_native_grpc_front_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "front_asan", CSRC / "tests" / "front_stress.cpp",
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    r = _run(exe, 4, 4, 2, env={"ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, r.stdout + r.stderr


def test_parsers_fuzz_under_asan(tmp_path):
    exe = _build(tmp_path, "fuzz_asan", CSRC / "tests" / "parser_fuzz.cpp",
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    r = _run(exe, 3000)
    assert r.returncode == 0, r.stdout + r.stderr
