#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -- \
  smoke 200 python -c "import __graft_entry__ as g; g.smoke()" -- \
  bdef 200 python bench.py -- \
  bdef2 200 python bench.py --steps 100 --warmup 20 -- \
  blanes 200 python bench.py --steps 100 --warmup 20 --stages none -- \
  sp16x8 200 python tools/serve_bench.py --clients 16 --images 8 --seconds 15 --device gpu --client-procs 4 -- \
  sp32x16 200 python tools/serve_bench.py --clients 32 --images 16 --seconds 15 --device gpu --client-procs 8
