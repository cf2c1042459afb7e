#!/bin/bash
# uniform middle-flow assignments of smaller-footprint fused kernels (sepconv_pipe 98/101/103/104,
# register-B fused conv_gemm 66/69/71, ws 124/125/140/141): can stage-2 workgroups that do not need
# an empty CU beat the 512-thread ws tiles under the stage pipeline?
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py"
args=()
for c in base 98 101 103 104 66 69 71 124 125 140 141 base; do
  if [ $c == base ]; then args+=(x_$c 200 $B --); else args+=(x_$c 200 $B --tuning tools/exp_tuning/m$c.json --); fi
done
tools/gpu_session.sh "${args[@]}"
