#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_eng 300 python -u -m pytest tests/test_engine_gpu.py tests/test_serving_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  br1 200 python bench.py --steps 100 --warmup 20 -- \
  br0 200 env KDL_BRANCHES=0 python bench.py --steps 100 --warmup 20 -- \
  br1b 200 python bench.py --steps 100 --warmup 20 -- \
  br0b 200 env KDL_BRANCHES=0 python bench.py --steps 100 --warmup 20
