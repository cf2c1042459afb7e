#!/bin/bash
# sepconv_ws with per-M-tile rotated K order (cfgs 143-146) vs the plain order (120/122/123/125)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_sep 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k separable --timeout 200 --timeout-method thread -- \
  kb32 300 python -u tools/kbench.py --shapes mid_sep --batch 32 --rounds 5 --cfgs 120,143,122,144,123,145,125,146 -- \
  kb16 300 python -u tools/kbench.py --shapes mid_sep --batch 16 --rounds 5 --cfgs 120,143,122,144,123,145,125,146
