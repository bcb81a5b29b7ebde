#!/bin/bash
# round 6 batch 35: diagonal offsets kept with the plan (fa_plan_diag_offsets) -- GPU suite, then per-kernel stats
# of config E and the E / C A/B against the previous library (abl/libfemasm_prev.so: searched diagonals)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b35_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/b35_pytest.log; [ $rc -eq 0 ] || { grep -h "Error\|FAILED" gpurun_out/b35_pytest.log | head -20; exit $rc; }
for rep in 1 2; do
  for lib in prev product; do
    if [ $lib = product ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    for c in E C; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-hbm-probe --no-eneo > gpurun_out/b35_$c.json 2> gpurun_out/b35_$c.err || { tail -5 gpurun_out/b35_$c.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b35_$c.json'));print('$lib $c', d['ms_per_step'], d['roofline']['launch_ms'])"
    done
  done
done
unset FEMASM_LIB
CFGS="E" STEPS=10 bash tools/prof_all.sh > gpurun_out/b35_prof.txt 2>&1 || { tail -5 gpurun_out/b35_prof.txt; exit 1; }
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_E/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('k_gather', 'k_cell', 'k_bc', 'k_rec', 'diag_off')):
        print(r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
