# round 3: ViT tiles that fill the chip in whole waves (graph-tuned against the committed
# tables), f32 compat serving, fp8 ViT kernel statistics
set -o pipefail
cd $GRAFT_REPO_ROOT
VC=encoder.layers.encoder_layer_5.mlp.3
tools/gpu_session.sh \
  vt 300 python -m kdl.engine.graph_tune --model vit_b16 --stages $VC --cfgs 61,62,63 --reps 20 --out gpurun_out/vit_b16_b32.json -- \
  v_old 100 python bench.py --model vit_b16 --steps 200 --warmup 20 -- \
  v_new 100 python bench.py --model vit_b16 --steps 200 --warmup 20 --tuning gpurun_out/vit_b16_b32.json -- \
  v8t 300 python -m kdl.engine.graph_tune --model vit_b16_fp8 --stages $VC --cfgs 8,9,10 --reps 20 --out gpurun_out/vit_b16_fp8_b32.json -- \
  v8_old 100 python bench.py --model vit_b16_fp8 --steps 200 --warmup 20 -- \
  v8_new 100 python bench.py --model vit_b16_fp8 --steps 200 --warmup 20 --tuning gpurun_out/vit_b16_fp8_b32.json -- \
  svf 250 python tools/serve_bench.py --procs 1 --clients 32 --images 8 --seconds 15 --client-procs 8 --signature serving_default
rc=$?
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_v8
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v8 -o run -- python bench.py --model vit_b16_fp8 --steps 50 --warmup 10 --tuning gpurun_out/vit_b16_fp8_b32.json > gpurun_out/prof_v8.log 2>&1
echo "prof rc=$?"
