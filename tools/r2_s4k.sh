#!/bin/bash
# K-rotated ws variants (each M tile starts its K loop at its own chunk: no L2 hot-spot on the
# same weight fragments at launch) for every ws layer / middle flow only, interleaved A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py"
tools/gpu_session.sh \
  k_base 200 $B -- \
  k_all 200 $B --tuning tools/exp_tuning/krot.json -- \
  k_mid 200 $B --tuning tools/exp_tuning/krot_mid.json -- \
  k_base2 200 $B -- \
  k_all2 200 $B --tuning tools/exp_tuning/krot.json -- \
  k_mid2 200 $B --tuning tools/exp_tuning/krot_mid.json
