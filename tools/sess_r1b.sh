#!/bin/bash
# GPU session: gpu tests, smoke, fused-sepconv kernel sweep, bench (stored + fresh tuning), rocprof stats.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
tools/gpu_session.sh \
  pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -- \
  smoke 300 python -c "import __graft_entry__ as g; g.smoke()" -- \
  kbench 400 python tools/kbench.py --shapes mid_sep,b4_sep2,b2_sep2,b14_sep2 --top 8 -- \
  bench 600 python bench.py --steps 50 --warmup 10 --profile-layers -- \
  bench_retune 600 python bench.py --steps 50 --warmup 10 --retune --save-tuning gpurun_out/xception_b32.json --profile-layers || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/bench -o bench -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?"
