#!/bin/bash
# uniform K-rotated ws band sizes for the middle flow (143: XB 9, 144: XB 11, 145: XB 16) vs the
# table; then the closed-loop gRPC serving bench at HEAD
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py"
tools/gpu_session.sh \
  rb 200 $B -- r143 200 $B --tuning tools/exp_tuning/r143.json -- r144 200 $B --tuning tools/exp_tuning/r144.json -- r145 200 $B --tuning tools/exp_tuning/r145.json -- \
  rb2 200 $B -- r143b 200 $B --tuning tools/exp_tuning/r143.json -- r144b 200 $B --tuning tools/exp_tuning/r144.json -- r145b 200 $B --tuning tools/exp_tuning/r145.json -- \
  serve 300 python tools/serve_bench.py --clients 16 --images 8 --seconds 12 --device gpu --client-procs 4 --max-batch 32
