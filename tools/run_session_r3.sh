set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 300 --warmup 30"
tools/gpu_session.sh \
  chain 240 python -u -m pytest tests/test_kernels_gpu.py -v -x --timeout 110 --timeout-method thread -k "chained" -- \
  base1 100 $B -- \
  ch2 100 env KDL_CHAIN=143 $B -- \
  ch8 100 env KDL_CHAIN=143 KDL_CHAIN_MIN=8 $B -- \
  base2 100 $B -- \
  sp207 100 env KDL_SEP_POOL=1 KDL_SEP_POOL_CFG=207 $B -- \
  nost 100 env KDL_STAGES=none $B -- \
  nostch 100 env KDL_STAGES=none KDL_CHAIN=143 $B -- \
  base3 100 $B -- \
  gemm 200 python tools/gemm_vs_vendor.py -- \
  null1 100 python tools/serve_bench.py --device null --procs 1 --clients 32 --images 8 --seconds 12 --client-procs 8 -- \
  null2 100 python tools/serve_bench.py --device null --procs 2 --clients 32 --images 8 --seconds 12 --client-procs 8 -- \
  g1 250 python tools/serve_bench.py --procs 1 --clients 32 --images 8 --seconds 15 --client-procs 8 -- \
  g2 250 python tools/serve_bench.py --procs 2 --clients 32 --images 8 --seconds 15 --client-procs 8
rc=$?
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trace0
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace0 -o run -- python bench.py --steps 100 --warmup 20 > gpurun_out/trace0.log 2>&1
echo "trace rc=$?"
