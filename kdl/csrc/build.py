"""In-tree build of the native extensions (no JIT cache, no hipify).

* ``kdl/_C``  : HIP kernels (gfx950) + native executor + pybind11 bindings,
                compiled with ``hipcc --offload-arch=gfx950``.
* ``kdl/_rt`` : CPU-only C++ runtime (dynamic batcher, TensorProto/PredictRequest
                codec, TensorBundle SSTable reader) compiled with ``g++``; it has no
                HIP dependency so the serving stack and its tests run on CPU boxes.

Usage: ``python -m kdl.csrc.build [--force] [--jobs N]``. Objects go to
``build/obj`` (git-ignored); the ``.so`` files land next to the package and
travel to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
ROOT = PKG.parent
OBJ = ROOT / "build" / "obj"
ARCH = os.environ.get("KDL_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_includes() -> list[str]:
    import pybind11
    return ["-I" + sysconfig.get_paths()["include"], "-I" + pybind11.get_include()]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build kdl._C)")


GPU_SOURCES = sorted((HERE / "kernels").glob("*.hip")) + [HERE / "runtime" / "engine.cpp",
                                                         HERE / "runtime" / "hip_backend.cpp",
                                                         HERE / "runtime" / "comm.cpp",
                                                         # the HIP loopback DP platform (dp_hiploop.h) reuses
                                                         # the loopback rendezvous of dp_loop.cpp
                                                         HERE / "runtime" / "dp_loop.cpp",
                                                         HERE / "runtime" / "dp_hiploop.cpp",
                                                         HERE / "bindings_gpu.cpp"]
RT_SOURCES = [HERE / "runtime" / n for n in ("batcher.cpp", "executor.cpp", "tfproto.cpp", "sstable.cpp", "dp_loop.cpp",
                                                "h2.cpp", "grpc_front.cpp", "grpc_load.cpp")] + [
    HERE / "bindings_rt.cpp"]
HEADERS = sorted(HERE.rglob("*.h"))


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in HEADERS)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _compile_all(jobs: list[tuple[list[str], Path]], njobs: int) -> list[Path]:
    with cf.ThreadPoolExecutor(max_workers=njobs) as ex:
        futs = [ex.submit(_run, cmd) for cmd, _ in jobs]
        for f in futs:
            f.result()
    return [o for _, o in jobs]


def build_gpu(force: bool = False, njobs: int = 8, verbose: bool = True) -> Path:
    hipcc = _hipcc()
    OBJ.mkdir(parents=True, exist_ok=True)
    out = PKG / f"_C{EXT}"
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", str(HERE),
              "-Wno-unused-result", "-Wno-unused-command-line-argument"] + _pybind_includes()
    jobs, objs = [], []
    for src in GPU_SOURCES:
        obj = OBJ / (src.stem + ("_hip" if src.suffix == ".hip" else "_cpp") + ".o")
        objs.append(obj)
        if force or _stale(obj, src):
            lang = ["-x", "hip"] if src.suffix == ".hip" else []
            jobs.append(([hipcc, *common, *lang, "-c", str(src), "-o", str(obj)], obj))
    if jobs and verbose:
        print(f"[kdl.build] compiling {len(jobs)} GPU source(s) for {ARCH}", flush=True)
    _compile_all(jobs, njobs)
    if force or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        # RCCL (runtime/comm.cpp): SONAME librccl.so.1, the same as the copy torch loads first
        # (import torch precedes kdl._C), so one instance is shared. No vendor BLAS: every GEMM
        # of the product is a hand-written MFMA kernel (hipBLASLt lives in tools/probes/blaslt)
        # link to a temporary name, then rename: a reader (an import, a tree snapshot) sees the old
        # or the new library, never a half-written one
        tmp = out.with_name(out.name + ".tmp")
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-L/opt/rocm/lib",
              "-lrccl", "-o", str(tmp)])
        os.replace(tmp, out)
        if verbose:
            print(f"[kdl.build] linked {out.relative_to(ROOT)}", flush=True)
    return out


def build_rt(force: bool = False, njobs: int = 8, verbose: bool = True) -> Path:
    cxx = os.environ.get("CXX", "g++")
    OBJ.mkdir(parents=True, exist_ok=True)
    out = PKG / f"_rt{EXT}"
    common = ["-O3", "-fPIC", "-std=c++17", "-pthread", "-I", str(HERE)] + _pybind_includes()
    jobs, objs = [], []
    for src in RT_SOURCES:
        obj = OBJ / (src.stem + "_rt.o")
        objs.append(obj)
        if force or _stale(obj, src):
            jobs.append(([cxx, *common, "-c", str(src), "-o", str(obj)], obj))
    if jobs and verbose:
        print(f"[kdl.build] compiling {len(jobs)} runtime source(s)", flush=True)
    _compile_all(jobs, njobs)
    if force or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        tmp = out.with_name(out.name + ".tmp")
        # libnghttp2 (the native gRPC front-end's HTTP/2) is dlopen'ed at first use (runtime/h2.cpp)
        _run([cxx, "-shared", "-fPIC", "-pthread", *map(str, objs), "-ldl", "-o", str(tmp)])
        os.replace(tmp, out)
        if verbose:
            print(f"[kdl.build] linked {out.relative_to(ROOT)}", flush=True)
    return out


def build_all(force: bool = False, njobs: int | None = None) -> None:
    njobs = njobs or min(8, os.cpu_count() or 4)
    build_rt(force, njobs)
    build_gpu(force, njobs)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--only", choices=["gpu", "rt"], default=None)
    a = ap.parse_args(argv)
    njobs = a.jobs or min(8, os.cpu_count() or 4)
    if a.only != "gpu":
        build_rt(a.force, njobs)
    if a.only != "rt":
        build_gpu(a.force, njobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
