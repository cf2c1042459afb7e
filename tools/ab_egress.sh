#!/bin/bash
# A/B on one GPU: plain single-rank bench vs the multi-rank code path at world 1 (process
# group up, RCCL gather of logits each step) vs multi-rank with local egress.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
for k in 1 2; do
  tools/gpu_session.sh \
    a$k 200 python bench.py -- \
    g$k 200 $R --master-port 2955$k bench.py --force-dist -- \
    l$k 200 $R --master-port 2956$k bench.py --force-dist --egress local || exit $?
done
grep -h '"value"' gpurun_out/{a,g,l}[12].log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['value'], d['config'].get('egress'), d['p50_latency_ms'])"
