#!/bin/bash
# eager (work-conserving) dispatch vs TF-Serving-style timeout wait: closed loop 16 x 8 and 1 x 1
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S="python tools/serve_bench.py --images 8 --seconds 12 --device gpu --client-procs 4 --max-batch 32 --clients 16 --timeout-us 2000"
L="python tools/serve_bench.py --images 1 --seconds 10 --device gpu --client-procs 1 --max-batch 32 --clients 1 --timeout-us 2000"
tools/gpu_session.sh \
  t_srv 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 250 --timeout-method thread -- \
  e1 300 $S -- n1 300 $S --no-eager -- e2 300 $S -- n2 300 $S --no-eager -- \
  le 300 $L -- ln 300 $L --no-eager -- \
  m4e 300 python tools/serve_bench.py --images 8 --seconds 10 --device gpu --client-procs 2 --max-batch 32 --clients 4 --timeout-us 2000 -- \
  m4n 300 python tools/serve_bench.py --images 8 --seconds 10 --device gpu --client-procs 2 --max-batch 32 --clients 4 --timeout-us 2000 --no-eager
