#!/bin/bash
# PMC passes (never mixed with tracing domains) + one kernel-trace pass for an
# arbitrary python tool command:  tools/pmc_cmd.sh <case> <python args...>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
name=$1; shift
mkdir -p gpurun_out/pmc
passes=(
  "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVES"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
)
i=0
for p in "${passes[@]}"; do
  out="gpurun_out/pmc/${name}_p$i"
  timeout -k 10 180 rocprofv3 --pmc $p -f csv -d "$out" -o run -- python "$@" > "$out.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 "$out.log"; [ $rc -gt 2 ] && exit $rc; fi
  i=$((i+1))
done
timeout -k 10 180 rocprofv3 --kernel-trace -f csv -d "gpurun_out/pmc/${name}_kt" -o run -- python "$@" > "gpurun_out/pmc/${name}_kt.log" 2>&1
exit 0
