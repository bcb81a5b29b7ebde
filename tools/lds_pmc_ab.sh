#!/bin/bash
# One LDS PMC pass of k_gather on config ${CFG:-E}, with the current defaults and with AB_ENV
# (e.g. FEMASM_SLOT_ORDER=0): bank-conflict cycles vs LDS-active cycles per dispatch.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for leg in cur alt; do
  E=""; [ $leg = alt ] && E="$AB_ENV"
  rm -rf gpurun_out/lds_$leg
  env $E timeout -s KILL 240 rocprofv3 --kernel-include-regex k_gather --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
    -d gpurun_out/lds_$leg/pass0 -o run --output-format csv -- python bench.py --config ${CFG:-E} --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/lds_$leg.log 2>&1 || { tail -5 gpurun_out/lds_$leg.log; exit 1; }
  echo "== $leg $E"
  python tools/pmc_summary.py gpurun_out/lds_$leg || exit 1
  find gpurun_out/lds_$leg -name "*.csv" -size +5M -delete
done
