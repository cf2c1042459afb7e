#!/bin/bash
# EfficientNet-B7: per-layer serial times + kernel stats at HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 300 python bench.py --model efficientnet_b7 --steps 10 --warmup 3 --profile-layers > gpurun_out/b7_layers.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/b7 -o b7 -- python bench.py --model efficientnet_b7 --steps 10 --warmup 3 > gpurun_out/prof_b7.log 2>&1
