#!/bin/bash
# TD / TA / LDS counters of the config-E gather for ablation builds (LIBS="label:path ...")
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $LIBS; do
  lab=${v%%:*}; lib=${v#*:}
  mkdir -p gpurun_out/dabl_$lab
  FEMASM_LIB=$PWD/$lib timeout -s KILL 300 rocprofv3 --kernel-include-regex 'k_gather' --pmc TD_TD_BUSY_sum TD_TC_STALL_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE -d gpurun_out/dabl_$lab -o run --output-format csv -- \
    python bench.py --config E --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dabl_$lab.log 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/dabl_$lab.log; exit 1; }
  echo "== $lab"; python tools/pmc_summary.py gpurun_out/dabl_$lab
  find gpurun_out/dabl_$lab -name "*kernel_trace.csv" -delete
done
