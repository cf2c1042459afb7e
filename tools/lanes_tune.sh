#!/bin/bash
# Concurrent-lanes autotune (2 lanes), then A/B: lanes-tuned table vs single-lane b32 table.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
M=${1:-xception}
timeout -k 10 600 python bench.py --model $M --steps 100 --warmup 10 --retune --save-tuning gpurun_out/${M}_b32_l2.json > gpurun_out/lt_${M}_tune.log 2>&1 || exit $?
echo "tune run: $(grep -o '"value": [0-9.]*' gpurun_out/lt_${M}_tune.log)"
for r in 1 2; do
  timeout -k 10 200 python bench.py --model $M --steps 200 --warmup 10 --tuning gpurun_out/${M}_b32_l2.json > gpurun_out/lt_${M}_l2tab.log 2>&1 || exit $?
  echo "l2 table: $(grep -o '"value": [0-9.]*' gpurun_out/lt_${M}_l2tab.log)"
  timeout -k 10 200 python bench.py --model $M --steps 200 --warmup 10 > gpurun_out/lt_${M}_b32tab.log 2>&1 || exit $?
  echo "b32 table: $(grep -o '"value": [0-9.]*' gpurun_out/lt_${M}_b32tab.log)"
done
