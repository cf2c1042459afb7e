#!/bin/bash
# ws: the two N tiles of an M tile start half a K loop apart (KDL_WS_NROT=1) vs together, interleaved
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_ws 200 env KDL_WS_NROT=1 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "separable or race" --timeout 150 --timeout-method thread -- \
  n0 200 python bench.py -- n1 200 env KDL_WS_NROT=1 python bench.py -- n0b 200 python bench.py -- n1b 200 env KDL_WS_NROT=1 python bench.py -- \
  n0c 200 python bench.py -- n1c 200 env KDL_WS_NROT=1 python bench.py
