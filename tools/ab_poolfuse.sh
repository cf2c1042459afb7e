#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_k 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  bf 300 python -u bench.py --steps 100 --warmup 20 -- \
  bo 300 env KDL_POOLFUSE=0 python -u bench.py --steps 100 --warmup 20 -- \
  bf2 300 python -u bench.py --steps 100 --warmup 20 --profile-layers
