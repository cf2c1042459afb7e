#!/bin/bash
# K-rotation multiplier of the rotated ws ids (KDL_WS_KMUL; default 7), interleaved
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
args=()
for m in 7 1 3 5 11 7 1 3 5 11; do args+=(m$m\_$RANDOM 200 env KDL_WS_KMUL=$m python bench.py --); done
tools/gpu_session.sh "${args[@]}"
