#!/bin/bash
# same-box A/B: block1_conv2 on the implicit-GEMM cfg 1 vs the 2-D tiled DMA-wave conv (cfg 215)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 --tuning tools/ab/x_c1.json > gpurun_out/ab_c1_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 > gpurun_out/ab_c215_$r.log 2>&1 || exit $?
  echo "run $r: cfg1 $(grep -o '"value": [0-9.]*' gpurun_out/ab_c1_$r.log)  cfg215 $(grep -o '"value": [0-9.]*' gpurun_out/ab_c215_$r.log)"
done
