#!/bin/bash
# round 6 batch 36: config E's set_diagonal pass with a 1024 / 512-entry queue (variants) -- kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in product bcq1024 bcq512; do
  if [ $lib = product ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
  CFGS="E" STEPS=10 bash tools/prof_all.sh > gpurun_out/b36_prof.txt 2>&1 || { tail -5 gpurun_out/b36_prof.txt; exit 1; }
  echo "== $lib"
  python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_E/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('k_bc', 'k_gather_lin')):
        print(r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
done
