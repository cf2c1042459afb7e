#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  gtune 900 python -u -m kdl.engine.graph_tune --model xception --batch 32 --lanes 2 --out gpurun_out/xception_b32_l2.json -- \
  bench_old 200 python bench.py --steps 100 --warmup 20 --tuning kdl/tuning/xception_b32.json -- \
  bench_new 200 python bench.py --steps 100 --warmup 20 --tuning gpurun_out/xception_b32_l2.json -- \
  bench_old2 200 python bench.py --steps 100 --warmup 20 --tuning kdl/tuning/xception_b32.json -- \
  bench_new2 200 python bench.py --steps 100 --warmup 20 --tuning gpurun_out/xception_b32_l2.json
