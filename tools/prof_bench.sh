set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench -o bench -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_bench.log 2>&1
echo "rc=$?"
