#!/bin/bash
# post-retune check: engine + serving + stage GPU tests, smoke, headline bench (driver-style and default)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  t_eng 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -- \
  smoke 200 python -c "import __graft_entry__ as g; g.smoke()" -- \
  u_d 200 python bench.py --gpus 1 --steps 20 --warmup 5 -- \
  u_x 200 python bench.py
