#!/bin/bash
# round-2 snapshot: families bench lines + Xception kernel stats under the default (stage-pipelined) bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/snap
tools/gpu_session.sh \
  f_xc 200 python bench.py --steps 100 --warmup 20 -- \
  f_r50 200 python bench.py --model resnet50 --steps 100 --warmup 20 -- \
  f_r50bf 200 python bench.py --model resnet50_bf16 --steps 100 --warmup 20 -- \
  f_vit 200 python bench.py --model vit_b16 --steps 100 --warmup 20 -- \
  f_vit8 200 python bench.py --model vit_b16_fp8 --steps 100 --warmup 20 -- \
  f_eff 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/snap/xc -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/snap/xc.log 2>&1
echo "prof rc=$?"
