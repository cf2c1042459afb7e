#!/bin/bash
# whole-graph tile tuning (kdl/engine/graph_tune.py) of the other families' 2-lane b32 tables + A/B bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in resnet50 vit_b16 vit_b16_fp8 efficientnet_b7; do
  tools/gpu_session.sh \
    gt_$m 600 python -u -m kdl.engine.graph_tune --model $m --batch 32 --lanes 2 --out gpurun_out/${m}_b32_l2.json -- \
    bo_$m 200 python bench.py --model $m --steps 50 --warmup 10 --tuning kdl/tuning/${m}_b32.json -- \
    bn_$m 200 python bench.py --model $m --steps 50 --warmup 10 --tuning gpurun_out/${m}_b32_l2.json || exit $?
done
