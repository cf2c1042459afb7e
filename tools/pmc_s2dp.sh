#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/pmc_cmd.sh s2dp185 tools/kbench.py --shapes b2_sep1 --batch 32 --rounds 1 --iters 3 --cfgs 185 &&
tools/pmc_cmd.sh s2dp187 tools/kbench.py --shapes b2_sep2 --batch 32 --rounds 1 --iters 3 --cfgs 187 &&
python tools/pmc_summary.py s2dp185 s2dp187 > gpurun_out/pmc_s2dp.txt
