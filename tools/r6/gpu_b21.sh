#!/bin/bash
# round 6 batch 21: affine quadrilaterals through k_gather_lin -- GPU suite, then config B A/B (base library = the
# previous build, abl/libfemasm_base.so)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b21_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/b21_pytest.log; [ $rc -eq 0 ] || { grep -h "Error\|FAILED" gpurun_out/b21_pytest.log | head -20; exit $rc; }
for rep in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export FEMASM_LIB=$PWD/abl/libfemasm_base.so; else unset FEMASM_LIB; fi
    timeout -k 10 300 python bench.py --config B --steps 20 --warmup 3 --no-cpu-baseline --no-hbm-probe > gpurun_out/b21_B_$lib.json 2> gpurun_out/b21_B_$lib.err || { tail -5 gpurun_out/b21_B_$lib.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b21_B_$lib.json'));print('B $lib', d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
  done
done
unset FEMASM_LIB
CFGS="B" STEPS=10 bash tools/prof_all.sh > gpurun_out/b21_prof.txt 2>&1 || { tail -5 gpurun_out/b21_prof.txt; exit 1; }
grep -E "^B |k_gather" gpurun_out/b21_prof.txt
