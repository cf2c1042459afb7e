#!/bin/bash
# row-streaming max-pool + residual add (numerics, sweep, headline A/B); uniform middle-flow
# tile assignments (fewer, larger workgroups leave CUs to the other pipeline stage); later cuts
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py"
tools/gpu_session.sh \
  t_pool 120 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "pool" --timeout 100 --timeout-method thread -- \
  poolb 200 python tools/poolbench.py -- \
  p1 200 env KDL_POOL_ALGO=1 $B -- \
  p2 200 env KDL_POOL_ALGO=2 $B -- \
  m135 200 $B --tuning tools/exp_tuning/m135.json -- \
  m136 200 $B --tuning tools/exp_tuning/m136.json -- \
  m137 200 $B --tuning tools/exp_tuning/m137.json -- \
  s25 200 $B --tuning tools/exp_tuning/s25.json -- \
  s38 200 $B --tuning tools/exp_tuning/s38.json -- \
  s24 200 $B --tuning tools/exp_tuning/s24.json -- \
  base 200 $B -- \
  c73 200 $B --stages block7_sepconv3 -- \
  c81 200 $B --stages block8_sepconv1 -- \
  c83 200 $B --stages block8_sepconv3 -- \
  c63 200 $B --stages block6_sepconv3 -- \
  p1b 200 env KDL_POOL_ALGO=1 $B -- \
  p2b 200 env KDL_POOL_ALGO=2 $B
