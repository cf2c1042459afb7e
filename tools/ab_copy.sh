#!/bin/bash
# closed-loop gRPC serving: batcher payload copy on 1 vs 4 threads
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
  KDL_COPY_THREADS=4 timeout -k 10 200 python -u tools/serve_bench.py --clients 16 --images 8 --seconds 12 --device gpu --client-procs 4 > gpurun_out/cp4_$r.log 2>&1 || exit $?
  KDL_COPY_THREADS=1 timeout -k 10 200 python -u tools/serve_bench.py --clients 16 --images 8 --seconds 12 --device gpu --client-procs 4 > gpurun_out/cp1_$r.log 2>&1 || exit $?
  echo "run $r: 4 threads $(grep -o '"images_per_s": [0-9.]*' gpurun_out/cp4_$r.log)  1 thread $(grep -o '"images_per_s": [0-9.]*' gpurun_out/cp1_$r.log)"
done
KDL_COPY_THREADS=4 timeout -k 10 200 python -u tools/serve_bench.py --clients 32 --images 16 --seconds 12 --device gpu --client-procs 8 > gpurun_out/cp4_big.log 2>&1 || exit $?
echo "32x16, 4 threads: $(grep -o '"images_per_s": [0-9.]*\|"p50_ms": [0-9.]*' gpurun_out/cp4_big.log | tr '\n' ' ')"
