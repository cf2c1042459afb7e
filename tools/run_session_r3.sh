set -o pipefail
cd $GRAFT_REPO_ROOT
tools/gpu_session.sh \
  chain 240 python -u -m pytest tests/test_kernels_gpu.py -v -x --timeout 110 --timeout-method thread -k "chained" -- \
  resize 200 python -u -m pytest tests/test_resize.py tests/test_serving_gpu.py -v --timeout 110 --timeout-method thread -k "resize" -- \
  ktests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_serving_gpu.py -v --timeout 200 --timeout-method thread -k "sepconv_pool or seppool or native or separable" -- \
  gate 200 python -u -m pytest tests/test_bench_configs_gpu.py -v -rP --timeout 150 --timeout-method thread -k xception -- \
  b_on1 100 python bench.py --steps 200 --warmup 20 -- \
  b_ch1 100 env KDL_CHAIN=143 python bench.py --steps 200 --warmup 20 -- \
  b_off1 100 env KDL_SEP_POOL=0 python bench.py --steps 200 --warmup 20 -- \
  b_ch2 100 env KDL_CHAIN=143 python bench.py --steps 200 --warmup 20 -- \
  b_on2 100 python bench.py --steps 200 --warmup 20 -- \
  layers 100 env KDL_CHAIN=143 python bench.py --steps 20 --warmup 5 --profile-layers
rc=$?
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trace gpurun_out/trace0
KDL_CHAIN=143 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python bench.py --steps 100 --warmup 20 > gpurun_out/trace.log 2>&1
echo "trace rc=$?"
