#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_st 300 python -u -m pytest tests/test_resnet_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  r_l2 200 python bench.py --model resnet50 --steps 100 --warmup 20 -- \
  r_s22 200 python bench.py --model resnet50 --steps 100 --warmup 20 --stages layer2.3.conv3 -- \
  r_s31 200 python bench.py --model resnet50 --steps 100 --warmup 20 --stages layer3.1.conv3 -- \
  r_s32 200 python bench.py --model resnet50 --steps 100 --warmup 20 --stages layer3.2.conv3 -- \
  r_s33 200 python bench.py --model resnet50 --steps 100 --warmup 20 --stages layer3.3.conv3 -- \
  r_s35 200 python bench.py --model resnet50 --steps 100 --warmup 20 --stages layer3.5.conv3 -- \
  x_def 200 python bench.py --steps 100 --warmup 20
