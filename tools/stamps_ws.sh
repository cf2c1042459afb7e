#!/bin/bash
# sepconv_ws phase stamps at b32 / b16: plain (127), no loop DMA (131), no B reloads (147), producers idle (133)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_session.sh \
  st32 300 bash -c 'for c in 127 131 147 133; do python -u tools/stamps.py --shape mid_sep --cfg $c --batch 32 --no-relu || exit $?; done' -- \
  st16 300 bash -c 'for c in 127 131 147 133; do python -u tools/stamps.py --shape mid_sep --cfg $c --batch 16 --no-relu || exit $?; done'
