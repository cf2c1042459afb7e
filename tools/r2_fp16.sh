#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_resnet 400 python -u -m pytest tests/test_resnet_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  b_r50_fp16 200 python bench.py --model resnet50 --steps 100 --warmup 20 -- \
  b_r50_bf16 200 python bench.py --model resnet50_bf16 --steps 100 --warmup 20 -- \
  b_r50_fp16b 200 python bench.py --model resnet50 --steps 100 --warmup 20 -- \
  b_r50_bf16b 200 python bench.py --model resnet50_bf16 --steps 100 --warmup 20
