#!/bin/bash
# B7 5x5 depthwise: tiled (algo 1, table) vs the direct kernel with wide chunk blocks (algo 2), sweep
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  dk5 400 python tools/dwkbench.py --shapes s3,s5,s6,s5a,s6a,s3a --direct
