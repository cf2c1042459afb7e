#!/bin/bash
# final verify of HEAD: full GPU suite, smoke, headline bench (default and driver-style), families, 2-rank rehearsal
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_all 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -- \
  smoke 200 python -c "import __graft_entry__ as g; g.smoke()" -- \
  z_xc 200 python bench.py -- \
  z_xc_d 200 python bench.py --gpus 1 --steps 20 --warmup 5 -- \
  z_r50 200 python bench.py --model resnet50 --steps 100 --warmup 20 -- \
  z_vit 200 python bench.py --model vit_b16 --steps 100 --warmup 20 -- \
  z_vit8 200 python bench.py --model vit_b16_fp8 --steps 100 --warmup 20 -- \
  z_eff 300 python bench.py --model efficientnet_b7 --steps 20 --warmup 5 -- \
  z_dist 700 bash tools/dist_rehearsal.sh
