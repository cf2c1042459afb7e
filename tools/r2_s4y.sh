#!/bin/bash
# ResNet-50 / ViT: engine-enabled K rotation (default) vs forced off (KDL_PIPE_KROT=0), interleaved
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python bench.py --model resnet50"
V="python bench.py --model vit_b16"
tools/gpu_session.sh \
  ra 200 $R -- rz 200 env KDL_PIPE_KROT=0 $R -- ra2 200 $R -- rz2 200 env KDL_PIPE_KROT=0 $R -- ra3 200 $R -- \
  va 200 $V -- vz 200 env KDL_PIPE_KROT=0 $V -- va2 200 $V -- vz2 200 env KDL_PIPE_KROT=0 $V
