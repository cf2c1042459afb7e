#!/bin/bash
# session 4: verify HEAD on one box (GPU tests, smoke, headline bench), then the direct
# depthwise sweep on the Xception shapes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_all 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -- \
  smoke 200 python -c "import __graft_entry__ as g; g.smoke()" -- \
  v_xc 200 python bench.py -- \
  dwd 300 python tools/dwbench.py --direct -- \
  v_r50 200 python bench.py --model resnet50 --steps 100 --warmup 20 -- \
  v_vit8 200 python bench.py --model vit_b16_fp8 --steps 100 --warmup 20 -- \
  v_eff 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5
