#!/bin/bash
# Diagnostic PMC passes (load path, L1, LDS, stall levels) of the gather of each config in CFGS.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
passes=(
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum"
  "TD_TD_BUSY_sum TD_TC_STALL_sum SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
)
for c in ${CFGS:-E Eneo}; do
  i=0; mkdir -p gpurun_out/diag_$c
  for p in "${passes[@]}"; do
    timeout -s KILL 300 rocprofv3 --kernel-include-regex 'k_gather' --pmc $p -d gpurun_out/diag_$c/pass$i -o run --output-format csv -- \
      python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-probe --no-eneo > gpurun_out/diag_$c/pass$i.log 2>&1 || { echo "$c pass $i failed"; tail -3 gpurun_out/diag_$c/pass$i.log; exit 1; }
    i=$((i+1))
  done
  python tools/pmc_summary.py gpurun_out/diag_$c > gpurun_out/diag_$c.txt || exit 1
  find gpurun_out/diag_$c -name "*kernel_trace.csv" -delete
  cat gpurun_out/diag_$c.txt
done
