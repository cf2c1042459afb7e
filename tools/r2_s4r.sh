#!/bin/bash
# closed-loop gRPC: batch timeout sweep (16 clients x 8 images), interleaved
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S="python tools/serve_bench.py --images 8 --seconds 12 --device gpu --client-procs 4 --max-batch 32 --clients 16"
tools/gpu_session.sh \
  s1 300 $S --timeout-us 1000 -- s2 300 $S --timeout-us 2000 -- s3 300 $S --timeout-us 3000 -- s5 300 $S --timeout-us 5000 -- \
  s1b 300 $S --timeout-us 1000 -- s2b 300 $S --timeout-us 2000 -- s3b 300 $S --timeout-us 3000 -- s5b 300 $S --timeout-us 5000 -- \
  l2 300 python tools/serve_bench.py --images 1 --seconds 10 --device gpu --client-procs 1 --max-batch 32 --clients 1 --timeout-us 2000 -- \
  l3 300 python tools/serve_bench.py --images 1 --seconds 10 --device gpu --client-procs 1 --max-batch 32 --clients 1 --timeout-us 3000
