#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_efficientnet_gpu.py -x -v --timeout 200 --timeout-method thread -k mbconv > gpurun_out/t_mbed.log 2>&1 || { tail -30 gpurun_out/t_mbed.log; exit 1; }
tail -2 gpurun_out/t_mbed.log
timeout -k 10 300 python -u tools/mbed_probe.py > gpurun_out/mbed_probe.log 2>&1 || exit $?
cat gpurun_out/mbed_probe.log | grep -v amdgpu
