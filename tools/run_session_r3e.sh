# tied graph tuning of the repeated blocks (Xception middle flow, ResNet-50 stages), A/B vs committed tables
set -o pipefail
cd $GRAFT_REPO_ROOT
tools/gpu_session.sh \
  xt 420 python -m kdl.engine.graph_tune --model xception --stages block7_sepconv1 --tie 'block([5-9]|1[0-2])_' --passes 2 --reps 20 --out gpurun_out/xception_b32.json -- \
  x_old 100 python bench.py --steps 300 --warmup 30 -- \
  x_new 100 python bench.py --steps 300 --warmup 30 --tuning gpurun_out/xception_b32.json -- \
  rt 300 python -m kdl.engine.graph_tune --model resnet50 --stages layer3.1.conv3 --tie '(?<=layer\d\.)[1-9]' --passes 2 --reps 20 --out gpurun_out/resnet50_b32.json -- \
  r_old 100 python bench.py --model resnet50 --steps 300 --warmup 30 -- \
  r_new 100 python bench.py --model resnet50 --steps 300 --warmup 30 --tuning gpurun_out/resnet50_b32.json -- \
  x_old2 100 python bench.py --steps 300 --warmup 30 -- \
  x_new2 100 python bench.py --steps 300 --warmup 30 --tuning gpurun_out/xception_b32.json -- \
  r_old2 100 python bench.py --model resnet50 --steps 300 --warmup 30 -- \
  r_new2 100 python bench.py --model resnet50 --steps 300 --warmup 30 --tuning gpurun_out/resnet50_b32.json
