#!/bin/bash
# closed-loop gRPC: batch timeout / concurrency probes (mean batch 30.1 at 1 ms, 16 x 8)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S="python tools/serve_bench.py --images 8 --seconds 12 --device gpu --client-procs 4 --max-batch 32"
tools/gpu_session.sh \
  s_t1 300 $S --clients 16 --timeout-us 1000 -- \
  s_t3 300 $S --clients 16 --timeout-us 3000 -- \
  s_c24 300 $S --clients 24 --timeout-us 1000 -- \
  s_c24t3 300 $S --clients 24 --timeout-us 3000
