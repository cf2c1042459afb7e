#!/bin/bash
# kernel stats of the headline bench at HEAD (rocprofv3 kernel trace) + 2-rank gloo rehearsal
# of bench.py's multi-rank path on the one GPU (tools/dist_rehearsal.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench -o bench -- python bench.py --steps 50 --warmup 10 > gpurun_out/prof_bench.log 2>&1 &&
echo "prof ok" && bash tools/dist_rehearsal.sh && echo "rehearsal ok" && grep -h '"value"' gpurun_out/d_local.log gpurun_out/d_scatter.log
