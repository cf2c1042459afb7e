#!/bin/bash
# Lanes A/B: lane-group test, then bench at 1 / 2 / 4 lanes (same box, back to back).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k lane -p no:cacheprovider > gpurun_out/lanes_test.log 2>&1 || exit $?
for L in 1 2 4 1 2 4; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --lanes $L > gpurun_out/lanes_b$L.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*' gpurun_out/lanes_b$L.log | sed "s/^/lanes=$L /"
done
