#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=encoder.layers.encoder_layer_
tools/gpu_session.sh \
  t_st 500 python -u -m pytest tests/test_vit_gpu.py tests/test_engine_gpu.py tests/test_resnet_gpu.py tests/test_efficientnet_gpu.py -x -q --timeout 300 --timeout-method thread -- \
  v_l2 200 python bench.py --model vit_b16 --steps 100 --warmup 20 -- \
  v_s4 200 python bench.py --model vit_b16 --steps 100 --warmup 20 --stages ${L}4.mlp.3 -- \
  v_s5 200 python bench.py --model vit_b16 --steps 100 --warmup 20 --stages ${L}5.mlp.3 -- \
  v_s6 200 python bench.py --model vit_b16 --steps 100 --warmup 20 --stages ${L}6.mlp.3 -- \
  v8_l2 200 python bench.py --model vit_b16_fp8 --steps 100 --warmup 20 -- \
  v8_s5 200 python bench.py --model vit_b16_fp8 --steps 100 --warmup 20 --stages ${L}5.mlp.3 -- \
  v8_s6 200 python bench.py --model vit_b16_fp8 --steps 100 --warmup 20 --stages ${L}6.mlp.3
