#!/bin/bash
# round 6 batch 33: chunk arrays cached in the plan (fa_plan_chunk_desc) -- GPU suite, then E / B / C A/B against
# the previous library (abl/libfemasm_prev.so, which ignores the new plan field: arrays rebuilt per launch)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b33_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/b33_pytest.log; [ $rc -eq 0 ] || { grep -h "Error\|FAILED" gpurun_out/b33_pytest.log | head -20; exit $rc; }
: > gpurun_out/b33_ab.txt
for rep in 1 2; do
  for lib in prev product; do
    if [ $lib = product ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    for c in E B C; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-hbm-probe --no-eneo > gpurun_out/b33_$c.json 2> gpurun_out/b33_$c.err || { tail -5 gpurun_out/b33_$c.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b33_$c.json'));print('$lib $c', d['ms_per_step'], d['roofline']['launch_ms'])" | tee -a gpurun_out/b33_ab.txt
    done
  done
done
