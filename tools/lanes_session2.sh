#!/bin/bash
# Default bench (lanes=2) + 2-rank gloo pipeline rehearsal on one GPU (both ranks on cuda:0).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > gpurun_out/l2_default.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/l2_default.log
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --lanes 1 > gpurun_out/l2_lanes1.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/l2_lanes1.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend gloo > gpurun_out/l2_gloo2.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/l2_gloo2.log
