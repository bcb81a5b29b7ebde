#!/bin/bash
# One PMC pass (LDS / VALU busy) on the assembly kernels of a config: tools/pmc_lin.sh CFG
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
c=${1:-E}
timeout -s KILL 300 rocprofv3 --kernel-include-regex 'k_gather' --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmcl_$c -o run --output-format csv -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/pmcl_$c.log 2>&1 || { tail -5 gpurun_out/pmcl_$c.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmcl_$c
