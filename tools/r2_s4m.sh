#!/bin/bash
# K-rotated fp8 GEMM (KDL_F8_KROT) on ViT-B/16 fp8, interleaved A/B; fp8 numerics first
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --model vit_b16_fp8"
tools/gpu_session.sh \
  t_f8 200 env KDL_F8_KROT=1 python -u -m pytest tests/test_fp8_gpu.py tests/test_vit_gpu.py -x -q --timeout 150 --timeout-method thread -- \
  f0 200 $B -- \
  f1 200 env KDL_F8_KROT=1 $B -- \
  f2 200 env KDL_F8_KROT=1 KDL_PIPE_KROT=1 $B -- \
  f0b 200 $B -- \
  f1b 200 env KDL_F8_KROT=1 $B -- \
  f2b 200 env KDL_F8_KROT=1 KDL_PIPE_KROT=1 $B -- \
  v0 200 python bench.py --model vit_b16 -- \
  v1 200 env KDL_PIPE_KROT=1 python bench.py --model vit_b16
