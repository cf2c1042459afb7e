#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_c3 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv3x3" --timeout 200 --timeout-method thread -- \
  kb_c3 300 python -u tools/kbench.py --shapes stem2 --batch 32 --rounds 5 --cfgs 1,208,209,212,213,214,215
