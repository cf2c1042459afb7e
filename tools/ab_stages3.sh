#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_stage 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  st_b6 200 python bench.py --steps 100 --warmup 20 --stages block6_sepconv3 -- \
  st_b7m 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv1 -- \
  st_b7m2 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv2 -- \
  st_b6m 200 python bench.py --steps 100 --warmup 20 --stages block6_sepconv2 -- \
  st_b6b 200 python bench.py --steps 100 --warmup 20 --stages block6_sepconv3 -- \
  st_b7mb 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv1
