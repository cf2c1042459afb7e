#!/bin/bash
# PMC passes over the headline bench (one rocprofv3 --pmc run per pass, no tracing domains, each
# under its own kill timer), for tools/pmc_table.py:
#   bash tools/pmc_head.sh <case> [bench args...]      -> gpurun_out/pmc/<case>_p<i>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
case=$1; shift
mkdir -p gpurun_out/pmc
passes=(
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_WAVES"
  "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
)
i=0
for p in "${passes[@]}"; do
  out="gpurun_out/pmc/${case}_p$i"
  timeout -s KILL 120 rocprofv3 --pmc $p -f csv -d "$out" -o run -- python bench.py --steps 10 --warmup 3 "$@" > "$out.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out.log"; exit $rc; fi
  i=$((i+1))
done
