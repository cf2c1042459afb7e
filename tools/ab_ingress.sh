#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  d3a 200 python bench.py --steps 100 --warmup 20 -- \
  d2a 200 python bench.py --steps 100 --warmup 20 --depth 2 -- \
  none1 200 python bench.py --steps 100 --warmup 20 --ingress none -- \
  d3b 200 python bench.py --steps 100 --warmup 20 -- \
  d2b 200 python bench.py --steps 100 --warmup 20 --depth 2 -- \
  free 200 python bench.py --steps 100 --warmup 20 --lanes-free -- \
  short 200 python bench.py
