#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  cm_none 200 python bench.py --steps 100 --warmup 20 -- \
  cm_55 200 python bench.py --steps 100 --warmup 20 --cu-share 0.5,0.5 -- \
  cm_64 200 python bench.py --steps 100 --warmup 20 --cu-share 0.6,0.4 -- \
  cm_73 200 python bench.py --steps 100 --warmup 20 --cu-share 0.7,0.3 -- \
  cm_r64 200 python bench.py --model resnet50 --steps 100 --warmup 20 --cu-share 0.6,0.4 -- \
  cm_rnone 200 python bench.py --model resnet50 --steps 100 --warmup 20
