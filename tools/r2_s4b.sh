#!/bin/bash
# direct depthwise: numerics, A/B against the tiled kernel in the headline bench, then a
# stage-pipelined whole-graph retune (split vs fused per layer can change) and its A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_dw 120 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "dw3x3 or separable" --timeout 100 --timeout-method thread -- \
  ab_tiled 200 env KDL_DW_ALGO=1 python bench.py -- \
  ab_direct 200 python bench.py -- \
  ab_tiled2 200 env KDL_DW_ALGO=1 python bench.py -- \
  ab_direct2 200 python bench.py -- \
  gt_st 900 python -u -m kdl.engine.graph_tune --model xception --batch 32 --stages block7_sepconv1 --out gpurun_out/xception_b32_st.json -- \
  st_old 200 python bench.py --tuning kdl/tuning/xception_b32.json -- \
  st_new 200 python bench.py --tuning gpurun_out/xception_b32_st.json -- \
  st_old2 200 python bench.py --tuning kdl/tuning/xception_b32.json -- \
  st_new2 200 python bench.py --tuning gpurun_out/xception_b32_st.json
