#!/bin/bash
# stage-cut sweep for the 2-stage Xception pipeline (bench.py --stages)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in block5_sepconv3 block6_sepconv2 block7_sepconv1 block7_sepconv3 block8_sepconv2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 --stages $c > gpurun_out/cut_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"value": [0-9.]*' gpurun_out/cut_$c.log)"
done
for c in block5_sepconv3 block6_sepconv2 block7_sepconv1 block7_sepconv3 block8_sepconv2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 --stages $c > gpurun_out/cut2_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"value": [0-9.]*' gpurun_out/cut2_$c.log)"
done
