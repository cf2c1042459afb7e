#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_e 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  b1 300 python -u bench.py --steps 100 --warmup 20 -- \
  b2 300 python -u bench.py --steps 100 --warmup 20
