#!/bin/bash
# LDS / VALU / TD counter passes of the gather kernels of config $CFG (default E) for the current
# build, FEMASM_CONTRIB as set by the caller.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
c=${CFG:-E}; tag=${TAG:-own}
passes=(
  "SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
  "TD_TD_BUSY_sum TD_TC_STALL_sum SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_FLOPS_FP64 GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0; d=gpurun_out/diag_${tag}_$c; mkdir -p $d
for p in "${passes[@]}"; do
  timeout -s KILL 300 rocprofv3 --kernel-include-regex 'k_gather' --pmc $p -d $d/pass$i -o run --output-format csv -- \
    python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $d/pass$i.log 2>&1 || { echo "$c pass $i failed"; tail -3 $d/pass$i.log; exit 1; }
  i=$((i+1))
done
python tools/pmc_summary.py $d > $d.txt || exit 1
find $d -name "*kernel_trace.csv" -delete
cat $d.txt
