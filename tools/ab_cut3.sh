#!/bin/bash
# 3-stage cut pairs vs the 2-stage default
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in block7_sepconv1 block3_pool,block9_sepconv1 block4_pool,block9_sepconv3 block2_pool,block8_sepconv1 block5_sepconv2,block10_sepconv2; do
  n=$(echo $c | tr ',' '_')
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 --stages $c > gpurun_out/cut3_$n.log 2>&1 || exit $?
  echo "$c $(grep -o '"value": [0-9.]*' gpurun_out/cut3_$n.log)"
done
