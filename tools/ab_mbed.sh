#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_efficientnet_gpu.py -x -v --timeout 200 --timeout-method thread -k mbconv > gpurun_out/t_mbed.log 2>&1 || { tail -30 gpurun_out/t_mbed.log; exit 1; }
tail -3 gpurun_out/t_mbed.log
timeout -k 10 400 python -u -m pytest tests/test_efficientnet_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_eff.log 2>&1 || { tail -30 gpurun_out/t_eff.log; exit 1; }
tail -2 gpurun_out/t_eff.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 > gpurun_out/mb_on_$r.log 2>&1 || exit $?
  KDL_MBED=0 timeout -k 10 300 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 > gpurun_out/mb_off_$r.log 2>&1 || exit $?
  echo "run $r: fused $(grep -o '"value": [0-9.]*' gpurun_out/mb_on_$r.log)  unfused $(grep -o '"value": [0-9.]*' gpurun_out/mb_off_$r.log)"
done
