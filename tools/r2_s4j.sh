#!/bin/bash
# B7 with the 5x5 stride-1 table rows on the direct kernel: GPU tests + bench A/B against HEAD~ numbers
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --model efficientnet_b7 --steps 20 --warmup 5"
tools/gpu_session.sh \
  t_b7 300 python -u -m pytest tests/test_efficientnet_gpu.py -x -q --timeout 250 --timeout-method thread -- \
  b7_a 300 $B -- \
  b7_b 300 $B
