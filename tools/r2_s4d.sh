#!/bin/bash
# HIP stream priorities per pipeline stage (KDL_STAGE_PRIO), interleaved A/B on the headline bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py"
timeout -k 10 120 python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" > gpurun_out/prange.log 2>&1 && cat gpurun_out/prange.log &&
tools/gpu_session.sh \
  pr_base 200 $B -- \
  pr_01 200 env KDL_STAGE_PRIO=0,-1 $B -- \
  pr_10 200 env KDL_STAGE_PRIO=-1,0 $B -- \
  pr_base2 200 $B -- \
  pr_01b 200 env KDL_STAGE_PRIO=0,-1 $B -- \
  pr_10b 200 env KDL_STAGE_PRIO=-1,0 $B -- \
  pr_r50 200 $B --model resnet50 -- \
  pr_r50_01 200 env KDL_STAGE_PRIO=0,-1 $B --model resnet50 -- \
  pr_vit 200 $B --model vit_b16_fp8 -- \
  pr_vit_01 200 env KDL_STAGE_PRIO=0,-1 $B --model vit_b16_fp8
