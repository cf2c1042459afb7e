#!/bin/bash
# stage pipelining (kdl/engine/stages.py) vs 2 half-batch lanes, Xception b32, one MI355X
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_stage 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  lanes2a 200 python bench.py --steps 100 --warmup 20 -- \
  st_b4 200 python bench.py --steps 100 --warmup 20 --stages block4_pool -- \
  st_b5 200 python bench.py --steps 100 --warmup 20 --stages block5_sepconv3 -- \
  st_b3 200 python bench.py --steps 100 --warmup 20 --stages block3_pool -- \
  st_b6 200 python bench.py --steps 100 --warmup 20 --stages block6_sepconv3 -- \
  lanes2b 200 python bench.py --steps 100 --warmup 20 -- \
  st_b4b 200 python bench.py --steps 100 --warmup 20 --stages block4_pool
