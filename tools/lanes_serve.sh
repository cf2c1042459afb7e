#!/bin/bash
# Serving path with lanes: GPU serving tests, then closed-loop gRPC A/B (KDL_LANES=1 vs default 2).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_serving_gpu.py tests/test_engine_gpu.py -p no:cacheprovider > gpurun_out/ls_tests.log 2>&1 || exit $?
tail -1 gpurun_out/ls_tests.log
for L in 2 1; do
  KDL_LANES=$L timeout -k 10 200 python tools/serve_bench.py --clients 64 --images 1 --seconds 15 --device gpu > gpurun_out/ls_c64_l$L.log 2>&1 || exit $?
  echo "c64 lanes=$L: $(tail -1 gpurun_out/ls_c64_l$L.log)"
  KDL_LANES=$L timeout -k 10 200 python tools/serve_bench.py --clients 16 --images 8 --seconds 15 --device gpu > gpurun_out/ls_c16x8_l$L.log 2>&1 || exit $?
  echo "c16x8 lanes=$L: $(tail -1 gpurun_out/ls_c16x8_l$L.log)"
done
