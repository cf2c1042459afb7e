#!/bin/bash
# headline bench, two runs (box-to-box spread is ~2 %)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  b1 300 python -u bench.py --steps 100 --warmup 20 -- \
  b2 300 python -u bench.py --steps 100 --warmup 20
