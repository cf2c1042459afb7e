#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_st 400 python -u -m pytest tests/test_efficientnet_gpu.py tests/test_resnet_gpu.py -x -q --timeout 300 --timeout-method thread -- \
  e_l2 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 -- \
  e_s2 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 --stages features.2.6.block.3 -- \
  e_s3 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 --stages features.3.6.block.3 -- \
  e_s4 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 --stages features.4.9.block.3 -- \
  r_s31 200 python bench.py --model resnet50 --steps 100 --warmup 20 -- \
  r_s30 200 python bench.py --model resnet50 --steps 100 --warmup 20 --stages layer3.0.conv3 -- \
  r_3st 200 python bench.py --model resnet50 --steps 100 --warmup 20 --stages layer2.1.conv3,layer3.3.conv3
