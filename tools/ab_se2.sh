#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_eff 300 python -u -m pytest tests/test_efficientnet_gpu.py -x -q --timeout 200 --timeout-method thread -- \
  e1 300 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 -- \
  e2 300 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 --profile-layers
