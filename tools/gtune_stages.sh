#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  gt_st 900 python -u -m kdl.engine.graph_tune --model xception --batch 32 --stages block7_sepconv1 --out gpurun_out/xception_b32_st.json -- \
  st_old 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv1 --tuning kdl/tuning/xception_b32.json -- \
  st_new 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv1 --tuning gpurun_out/xception_b32_st.json -- \
  st_old2 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv1 --tuning kdl/tuning/xception_b32.json -- \
  st_new2 200 python bench.py --steps 100 --warmup 20 --stages block7_sepconv1 --tuning gpurun_out/xception_b32_st.json
