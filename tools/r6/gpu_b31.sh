#!/bin/bash
# round 6 batch 30: k_rec_bcbits, a wave per 64 nodes and a lane per adjacency entry -- GPU suite (with the component-bc parity tests), then E A/B against
# the library before the node-side bits (abl/libfemasm_prev.so) and kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b31_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/b31_pytest.log; [ $rc -eq 0 ] || { grep -h "Error\|FAILED" gpurun_out/b31_pytest.log | head -20; exit $rc; }
: > gpurun_out/b31_ab.txt
for rep in 1 2; do
  for lib in prev product; do
    if [ $lib = product ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    timeout -k 10 300 python tools/r6/order_variants.py 203 row,row E > gpurun_out/b31_tmp.txt 2> gpurun_out/b31_$lib.err || { tail -5 gpurun_out/b31_$lib.err; exit 1; }
    sed "s/^{/{\"lib\": \"$lib\", \"cfg\": \"E\", /" gpurun_out/b31_tmp.txt | tee -a gpurun_out/b31_ab.txt
  done
done
unset FEMASM_LIB
CFGS="E" STEPS=5 bash tools/prof_all.sh > gpurun_out/b31_prof.txt 2>&1 || { tail -5 gpurun_out/b31_prof.txt; exit 1; }
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_E/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('k_gather', 'k_cell', 'k_bc', 'k_rec')):
        print(r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
