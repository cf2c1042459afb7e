#!/bin/bash
# serving executor pipelining A/B (KDL_EXEC_DEPTH = batches in flight per GPU)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_serve 400 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  s16x8_d2 200 env KDL_EXEC_DEPTH=2 python tools/serve_bench.py --clients 16 --images 8 --seconds 15 --device gpu -- \
  s16x8_d1 200 env KDL_EXEC_DEPTH=1 python tools/serve_bench.py --clients 16 --images 8 --seconds 15 --device gpu -- \
  s64x1_d2 200 env KDL_EXEC_DEPTH=2 python tools/serve_bench.py --clients 64 --images 1 --seconds 15 --device gpu -- \
  s64x1_d1 200 env KDL_EXEC_DEPTH=1 python tools/serve_bench.py --clients 64 --images 1 --seconds 15 --device gpu -- \
  s32x8_d2 200 env KDL_EXEC_DEPTH=2 python tools/serve_bench.py --clients 32 --images 8 --seconds 15 --device gpu
