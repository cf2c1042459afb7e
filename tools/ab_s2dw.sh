#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_sep 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "separable or race" --timeout 200 --timeout-method thread || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 > gpurun_out/ab_s187_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 --tuning tools/ab/x_s204.json > gpurun_out/ab_s204_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 --tuning tools/ab/x_s201.json > gpurun_out/ab_s201_$r.log 2>&1 || exit $?
  echo "run $r: 187 $(grep -o '"value": [0-9.]*' gpurun_out/ab_s187_$r.log)  204 $(grep -o '"value": [0-9.]*' gpurun_out/ab_s204_$r.log)  201 $(grep -o '"value": [0-9.]*' gpurun_out/ab_s201_$r.log)"
done
