#!/bin/bash
# One GPU-box session: tests, smoke, bench (+tuning), serve bench, kernel-trace profile.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
tools/gpu_session.sh \
  pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider -- \
  smoke 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" -- \
  bench 600 python bench.py --steps 50 --warmup 10 --save-tuning gpurun_out/xception_b32.json --profile-layers -- \
  serve_c64 300 python tools/serve_bench.py --clients 64 --images 1 --seconds 20 --device gpu -- \
  serve_c16x8 300 python tools/serve_bench.py --clients 16 --images 8 --seconds 20 --device gpu || exit $?
cp gpurun_out/xception_b32.json kdl/tuning/xception_b32.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/bench -o bench -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?"
