#!/bin/bash
# PMC traffic (and executed FP64 flop) records for bench.py: for each config in CFGS, the
# tools/prof_passes.sh passes over the assembly kernels, a summary under gpurun_out/pmc_<cfg>.txt and
# the record "<cfg>:<side>" in gpurun_out/traffic.json, keyed on the femasm.hip hash.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -f profiles/traffic.json ] && cp profiles/traffic.json gpurun_out/traffic.json
for cs in ${CFGS:-E:203}; do
  c=${cs%%:*}; n=${cs#*:}
  pm=0; [ "$c" = Dmfma ] && pm=1
  PASS_MFMA=$pm bash tools/prof_passes.sh gpurun_out/pmc_$c 'k_gather|k_cell_records|k_rec_bcbits|k_neo_records|k_hex_mfma|k_bc_diag' -- python bench.py --config $c --side $n --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-probe --no-eneo || exit $?
  python tools/pmc_summary.py gpurun_out/pmc_$c > gpurun_out/pmc_$c.txt || exit $?
  python tools/pmc_summary.py gpurun_out/pmc_$c $c:$n gpurun_out/traffic.json || exit $?
  find gpurun_out/pmc_$c -name "*kernel_trace.csv" -delete
done
cat gpurun_out/traffic.json
