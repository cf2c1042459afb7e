#!/bin/bash
# stage cut re-check with the K-rotated table (stage 2 got faster), interleaved
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py"
tools/gpu_session.sh \
  cb 200 $B -- c62 200 $B --stages block6_sepconv2 -- c63 200 $B --stages block6_sepconv3 -- c72 200 $B --stages block7_sepconv2 -- c73 200 $B --stages block7_sepconv3 -- \
  cb2 200 $B -- c62b 200 $B --stages block6_sepconv2 -- c63b 200 $B --stages block6_sepconv3 -- c72b 200 $B --stages block7_sepconv2 -- c73b 200 $B --stages block7_sepconv3
