#!/bin/bash
# rocprofv3 kernel-trace + stats of one command (no PMC, no other tracing domains):
#   tools/prof_stats.sh <outdir> <cmd...>      e.g. tools/prof_stats.sh gpurun_out/prof python3 bench.py --steps 50
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
exec rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- "$@"
