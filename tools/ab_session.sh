set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --model resnet50 --steps 400 --warmup 30"
tools/gpu_session.sh \
  r2 100 $B -- \
  r3 100 $B --stages layer2.1.conv3,layer3.3.conv3 -- \
  r3a 100 $B --stages layer2.0.conv3,layer3.2.conv3 -- \
  r3b 100 $B --stages layer2.2.conv3,layer3.4.conv3 -- \
  r3c 100 $B --stages layer1.2.conv3,layer3.1.conv3 -- \
  r2b 100 $B -- \
  r3x 100 $B --stages layer2.1.conv3,layer3.3.conv3
