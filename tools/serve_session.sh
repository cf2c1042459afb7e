#!/bin/bash
# closed-loop gRPC serving on one MI355X with clients in separate processes (server GIL alone)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  sp16x8 200 python tools/serve_bench.py --clients 16 --images 8 --seconds 15 --device gpu --client-procs 4 -- \
  sp32x8 200 python tools/serve_bench.py --clients 32 --images 8 --seconds 15 --device gpu --client-procs 8 -- \
  sp64x1 200 python tools/serve_bench.py --clients 64 --images 1 --seconds 15 --device gpu --client-procs 8 -- \
  sp16x32 200 python tools/serve_bench.py --clients 16 --images 32 --seconds 15 --device gpu --client-procs 8
