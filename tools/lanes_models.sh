#!/bin/bash
# lanes 1 vs 2 for the other model families (bench defaults otherwise).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for M in resnet50 vit_b16 vit_b16_fp8 efficientnet_b7; do
  for L in 1 2; do
    timeout -k 10 240 python bench.py --model $M --steps 50 --warmup 5 --lanes $L > gpurun_out/lm_${M}_$L.log 2>&1 || exit $?
    echo "$M lanes=$L $(grep -o '"value": [0-9.]*' gpurun_out/lm_${M}_$L.log)"
  done
done
