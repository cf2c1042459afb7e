set -o pipefail
cd $GRAFT_REPO_ROOT
tools/gpu_session.sh \
  et 800 python -m kdl.engine.graph_tune --model efficientnet_b7 --stages features.4.9.block.3 --tie '(?<=features\.\d\.)[1-9]\d*' --passes 1 --reps 8 --out gpurun_out/efficientnet_b7_b32.json -- \
  e_old 100 python bench.py --model efficientnet_b7 --steps 100 --warmup 10 -- \
  e_new 100 python bench.py --model efficientnet_b7 --steps 100 --warmup 10 --tuning gpurun_out/efficientnet_b7_b32.json -- \
  e_old2 100 python bench.py --model efficientnet_b7 --steps 100 --warmup 10 -- \
  e_new2 100 python bench.py --model efficientnet_b7 --steps 100 --warmup 10 --tuning gpurun_out/efficientnet_b7_b32.json
