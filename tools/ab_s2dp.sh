#!/bin/bash
# persistent 2-D sepconv: ring depth (cfgs 190-192 = deeper rings) on the 147x147 early-flow layers
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_sep 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "separable or race" --timeout 200 --timeout-method thread -- \
  kb_s2 300 python -u tools/kbench.py --shapes b2_sep2,b2_sep1 --batch 32 --rounds 5 --cfgs 184,185,186,187,188,189,190,191,192
