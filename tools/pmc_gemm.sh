#!/bin/bash
# Detailed PMC passes for one GEMM case (kprof.py args after the case name).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
name=$1; shift
mkdir -p gpurun_out/pmc
passes=(
  "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_VMEM_RD"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_MFMA SQ_INSTS_VALU"
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
