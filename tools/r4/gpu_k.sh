#!/bin/bash
# plan passes (plan_stats) and E launch / plan time per build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for name in ${VARS:-rel base}; do
  L=""; [ $name != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$name.so"
  env $L timeout -k 10 300 python tools/r4/plan_stats.py 16 2>&1 | grep "passes" | sed "s/^/$name /"
done
for name in ${VARS:-rel base}; do
  L=""; [ $name != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$name.so"
  env $L timeout -k 10 300 python bench.py --config E --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$name failed"; tail -5 gpurun_out/v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('E $name', d['roofline']['launch_ms'], 'plan_s', d['setup']['plan_s'])"
done
