#!/bin/bash
# PMC passes (tools/prof_passes.sh) of the gather launch of one bench config; summary to gpurun_out/pmc_<cfg>.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
c=${CFG:-Eneo}
bash tools/prof_passes.sh gpurun_out/pmc_$c 'k_gather|k_cell_records' -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline || exit $?
python tools/pmc_summary.py gpurun_out/pmc_$c > gpurun_out/pmc_$c.txt || exit $?
find gpurun_out/pmc_$c -name "*kernel_trace.csv" -delete
cat gpurun_out/pmc_$c.txt
