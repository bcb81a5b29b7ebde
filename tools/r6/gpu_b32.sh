#!/bin/bash
# round 6 batch 32: per-kernel stats of config E, previous library vs product (k_rec_bcbits / k_bc_diag changes)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in prev product; do
    if [ $lib = product ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    CFGS="E" STEPS=10 bash tools/prof_all.sh > gpurun_out/b32_prof.txt 2>&1 || { tail -5 gpurun_out/b32_prof.txt; exit 1; }
    echo "== $lib"
    python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_E/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('k_gather', 'k_cell', 'k_bc', 'k_rec')):
        print(r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
  done
done
