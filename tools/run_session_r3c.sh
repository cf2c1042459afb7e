set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 300 --warmup 30"
tools/gpu_session.sh \
  chain 240 python -u -m pytest tests/test_kernels_gpu.py -v -x --timeout 110 --timeout-method thread -k "chained" -- \
  diag 150 python -u tools/chain_diag.py --batch 2 -- \
  base1 100 $B -- \
  ch2 100 env KDL_CHAIN=143 $B -- \
  ch8 100 env KDL_CHAIN=143 KDL_CHAIN_MIN=8 $B -- \
  base2 100 $B -- \
  ch2b 100 env KDL_CHAIN=143 $B
rc=$?
[ $rc -ne 0 ] && exit $rc
grep -q "FAILED\|Error" gpurun_out/chain.log && { echo "chain tests failed: stopping"; exit 3; }
bash tools/run_session_r3b.sh
