#!/bin/bash
# GEMM core-efficiency probe: our pipe GEMM vs hipBLASLt on Xception + square shapes, PMC of mid_pw.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_session.sh \
  blas 300 python tools/blas_probe.py -- \
  kb_mid 300 python tools/kbench.py --shapes mid_pw,b14_sep2 --top 6 -- \
  kb_sq 300 python tools/kbench.py --shapes sq2k,sq4k --batch 4 --top 6 --iters 5 || exit $?
tools/pmc_gemm.sh mid_pw25 --shape mid_pw --cfg 25 --iters 20
