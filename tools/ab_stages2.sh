#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  st_b6 200 python bench.py --steps 100 --warmup 20 --stages block6_sepconv3 -- \
  st_b7 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv3 -- \
  st_b8 200 python bench.py --steps 100 --warmup 20 --stages block8_sepconv3 -- \
  st_b9 200 python bench.py --steps 100 --warmup 20 --stages block9_sepconv3 -- \
  st_b6m 200 python bench.py --steps 100 --warmup 20 --stages block6_sepconv2 -- \
  st_b7m 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv1 -- \
  st_b6b 200 python bench.py --steps 100 --warmup 20 --stages block6_sepconv3 -- \
  st_b7b 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv3
