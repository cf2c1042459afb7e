# ViT: graph-tune with the 12 encoder layers tied (all candidate tiles), then A/B against the committed tables
set -o pipefail
cd $GRAFT_REPO_ROOT
VC=encoder.layers.encoder_layer_5.mlp.3
T='encoder_layer_\d+'
tools/gpu_session.sh \
  vt 300 python -m kdl.engine.graph_tune --model vit_b16 --stages $VC --tie "$T" --passes 2 --reps 20 --out gpurun_out/vit_b16_b32.json -- \
  v8t 300 python -m kdl.engine.graph_tune --model vit_b16_fp8 --stages $VC --tie "$T" --passes 2 --reps 20 --out gpurun_out/vit_b16_fp8_b32.json -- \
  v_old 100 python bench.py --model vit_b16 --steps 300 --warmup 30 -- \
  v_new 100 python bench.py --model vit_b16 --steps 300 --warmup 30 --tuning gpurun_out/vit_b16_b32.json -- \
  v8_old 100 python bench.py --model vit_b16_fp8 --steps 300 --warmup 30 -- \
  v8_new 100 python bench.py --model vit_b16_fp8 --steps 300 --warmup 30 --tuning gpurun_out/vit_b16_fp8_b32.json -- \
  v_old2 100 python bench.py --model vit_b16 --steps 300 --warmup 30 -- \
  v_new2 100 python bench.py --model vit_b16 --steps 300 --warmup 30 --tuning gpurun_out/vit_b16_b32.json -- \
  v8_old2 100 python bench.py --model vit_b16_fp8 --steps 300 --warmup 30 -- \
  v8_new2 100 python bench.py --model vit_b16_fp8 --steps 300 --warmup 30 --tuning gpurun_out/vit_b16_fp8_b32.json
