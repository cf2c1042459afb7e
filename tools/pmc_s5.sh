#!/bin/bash
# PMC passes over the headline bench step at HEAD (counters only, no tracing domains)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_s5
passes=(
  "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
)
i=0
for p in "${passes[@]}"; do
  out="gpurun_out/pmc_s5/p$i"
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $p -f csv -d "$out" -o run -- python bench.py --steps 5 --warmup 2 --settle 0 > "$out.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"; tail -3 "$out.log"
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
