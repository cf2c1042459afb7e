cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --profile-layers > gpurun_out/bench_now.log 2>&1 && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1
echo "rc=$?"
