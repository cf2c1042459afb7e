#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/pmc_cmd.sh c3_209 tools/kbench.py --shapes stem2 --batch 32 --rounds 1 --iters 3 --cfgs 209 &&
tools/pmc_cmd.sh c3_208 tools/kbench.py --shapes stem2 --batch 32 --rounds 1 --iters 3 --cfgs 208 &&
python tools/pmc_summary.py c3_209 c3_208 > gpurun_out/pmc_c3.txt
