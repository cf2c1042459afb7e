#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_eff 400 python -u -m pytest tests/test_efficientnet_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 > gpurun_out/sf_on_$r.log 2>&1 || exit $?
  KDL_SEFOLD=0 timeout -k 10 300 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 > gpurun_out/sf_off_$r.log 2>&1 || exit $?
  echo "run $r: fold $(grep -o '"value": [0-9.]*' gpurun_out/sf_on_$r.log)  chscale $(grep -o '"value": [0-9.]*' gpurun_out/sf_off_$r.log)"
done
