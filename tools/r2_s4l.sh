#!/bin/bash
# K-rotated LDS-DMA GEMM (gemm_pipe, KDL_PIPE_KROT=1) per family, interleaved A/B; GEMM numerics first
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_k 200 env KDL_PIPE_KROT=1 python -u -m pytest tests/test_kernels_gpu.py tests/test_vit_gpu.py tests/test_resnet_gpu.py -x -q --timeout 150 --timeout-method thread -- \
  x0 200 python bench.py -- \
  x1 200 env KDL_PIPE_KROT=1 python bench.py -- \
  r0 200 python bench.py --model resnet50 -- \
  r1 200 env KDL_PIPE_KROT=1 python bench.py --model resnet50 -- \
  v0 200 python bench.py --model vit_b16 -- \
  v1 200 env KDL_PIPE_KROT=1 python bench.py --model vit_b16 -- \
  e0 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 -- \
  e1 300 env KDL_PIPE_KROT=1 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 -- \
  x0b 200 python bench.py -- \
  x1b 200 env KDL_PIPE_KROT=1 python bench.py -- \
  r0b 200 python bench.py --model resnet50 -- \
  r1b 200 env KDL_PIPE_KROT=1 python bench.py --model resnet50 -- \
  v0b 200 python bench.py --model vit_b16 -- \
  v1b 200 env KDL_PIPE_KROT=1 python bench.py --model vit_b16 -- \
  f0 200 python bench.py --model vit_b16_fp8 -- \
  f1 200 env KDL_PIPE_KROT=1 python bench.py --model vit_b16_fp8
