#!/bin/bash
# session 5 (fresh container, rebuilt .so): every family's bench at HEAD, kernel stats of
# the headline step, closed-loop serving, 2-rank rehearsal. Each GPU step has its own limit.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
tools/gpu_session.sh \
  v_xc 200 python bench.py --steps 200 --warmup 20 -- \
  v_xc_drv 200 python bench.py --gpus 1 --steps 20 --warmup 5 -- \
  v_r50 200 python bench.py --model resnet50 --steps 100 --warmup 20 -- \
  v_vit 200 python bench.py --model vit_b16 --steps 100 --warmup 20 -- \
  v_eff 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 -- \
  s_xc 200 python tools/serve_bench.py --clients 16 --images 8 --seconds 12 --device gpu --client-procs 4 --max-batch 32 || exit $?
mkdir -p gpurun_out/prof_s5
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s5 -o run -- python bench.py --steps 50 --warmup 10 > gpurun_out/prof_s5.log 2>&1 || exit $?
echo "prof rc=0"
tools/dist_rehearsal.sh && echo "rehearsal ok" && tail -2 gpurun_out/d_local.log gpurun_out/d_scatter.log
