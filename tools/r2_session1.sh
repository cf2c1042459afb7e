#!/bin/bash
# Round-2 first GPU session: gpu tests, smoke, bench (layer profile), kernel-trace stats.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r2
tools/gpu_session.sh \
  pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -- \
  smoke 300 python -c "import __graft_entry__ as g; g.smoke()" -- \
  bench 300 python bench.py --steps 50 --warmup 10 --profile-layers || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2 -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_r2.log 2>&1
echo "prof rc=$?"
