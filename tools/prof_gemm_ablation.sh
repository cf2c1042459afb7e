#!/bin/bash
# exact GPU kernel durations (rocprofv3 kernel trace) of the gemm_pipe ablations
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/p5
cd /tmp
for b in 32 64; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/p5/b$b -o k -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --shapes mid_pw --batch $b --cfgs 25,43,44,45,46,47,50,57,58,52,53,55 --rounds 2 --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/p5/b$b.log 2>&1 || exit $?
done
echo done
