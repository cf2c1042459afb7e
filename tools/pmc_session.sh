#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass; --pmc never mixed with tracing domains).
#   tools/pmc_session.sh <case-name> <kprof args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
name=$1; shift
mkdir -p gpurun_out/pmc
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
  "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr"
  "FETCH_SIZE"
)
i=0
for p in "${passes[@]}"; do
  out="gpurun_out/pmc/${name}_p$i"
  timeout -k 10 120 rocprofv3 --pmc $p -f csv -d "$out" -o run -- python tools/kprof.py "$@" > "$out.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 "$out.log"; [ $rc -gt 2 ] && exit $rc; fi
  i=$((i+1))
done
exit 0
