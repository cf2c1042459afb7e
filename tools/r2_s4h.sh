#!/bin/bash
# B7 direct depthwise with wide non-power-of-two chunk blocks (KDL_DWV_WIDE): numerics (B7 GPU
# tests + dwkbench numerics on the affected shapes), standalone A/B, and the B7 bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --model efficientnet_b7 --steps 20 --warmup 5"
tools/gpu_session.sh \
  t_b7 300 python -u -m pytest tests/test_efficientnet_gpu.py -x -q --timeout 250 --timeout-method thread -- \
  dk_wide 200 python tools/dwkbench.py --shapes s2,s2a,s4,s4a,s7 -- \
  dk_pow2 200 env KDL_DWV_WIDE=0 python tools/dwkbench.py --shapes s2,s2a,s4,s4a,s7 -- \
  b7_pow2 300 env KDL_DWV_WIDE=0 $B -- \
  b7_wide 300 $B -- \
  b7_pow2b 300 env KDL_DWV_WIDE=0 $B -- \
  b7_wideb 300 $B
