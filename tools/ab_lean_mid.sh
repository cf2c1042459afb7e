#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_sep 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "separable or race" --timeout 200 --timeout-method thread -- \
  kb32 200 python tools/kbench.py --batch 32 --shapes mid_sep --cfgs 120,122,140,141,142 --rounds 3 -- \
  base 200 python bench.py --steps 100 --warmup 20 -- \
  m140 200 python bench.py --steps 100 --warmup 20 --tuning gpurun_out/xc_mid140.json -- \
  m142 200 python bench.py --steps 100 --warmup 20 --tuning gpurun_out/xc_mid142.json -- \
  m140s2 200 python bench.py --steps 100 --warmup 20 --tuning gpurun_out/xc_mid140_s2.json -- \
  base2 200 python bench.py --steps 100 --warmup 20
