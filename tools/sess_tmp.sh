cd $GRAFT_REPO_ROOT
tools/gpu_session.sh \
  pytest_k 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -p no:cacheprovider -- \
  bench 600 python bench.py --steps 50 --warmup 10 --save-tuning gpurun_out/xception_b32.json --profile-layers || exit $?
grep -v amdgpu gpurun_out/bench.log | head -3
