#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_stage 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  s2 200 python bench.py --steps 100 --warmup 20 -- \
  s3a 200 python bench.py --steps 100 --warmup 20 --stages block3_pool,block9_sepconv3 -- \
  s3b 200 python bench.py --steps 100 --warmup 20 --stages block4_pool,block10_sepconv3 -- \
  s3c 200 python bench.py --steps 100 --warmup 20 --stages block2_pool,block8_sepconv3 -- \
  s3d 200 python bench.py --steps 100 --warmup 20 --stages block3_pool,block8_sepconv2 -- \
  s3e 200 python bench.py --steps 100 --warmup 20 --stages block4_sepconv1,block10_sepconv1 -- \
  s2b 200 python bench.py --steps 100 --warmup 20
