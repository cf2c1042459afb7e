#!/bin/bash
# stage-pipelined whole-graph retune starting from the K-rotated table, then interleaved bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  gt 900 python -u -m kdl.engine.graph_tune --model xception --batch 32 --stages block7_sepconv1 --out gpurun_out/xception_b32_st2.json -- \
  w0 200 python bench.py -- w1 200 python bench.py --tuning gpurun_out/xception_b32_st2.json -- \
  w0b 200 python bench.py -- w1b 200 python bench.py --tuning gpurun_out/xception_b32_st2.json -- \
  w0c 200 python bench.py -- w1c 200 python bench.py --tuning gpurun_out/xception_b32_st2.json
