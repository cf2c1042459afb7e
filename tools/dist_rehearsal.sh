#!/bin/bash
# Two ranks sharing the box's one GPU over gloo: exercises bench.py's multi-rank pipeline
# (ingress local / scatter, logits gather, MAX-over-ranks timing) without RCCL, which
# refuses two ranks on one device. Never run N=8 here (the driver's job).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 $R --master-port 29555 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo > gpurun_out/d_local.log 2>&1 &&
timeout -k 10 300 $R --master-port 29556 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --ingress scatter > gpurun_out/d_scatter.log 2>&1
