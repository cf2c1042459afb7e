#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_k 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_efficientnet_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  bx 300 python -u bench.py --steps 100 --warmup 20 --profile-layers -- \
  be 300 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5
