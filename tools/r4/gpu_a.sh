#!/bin/bash
# Round-4 first GPU call: LDS op probe + config E with compile-time variants (abl/), alternating with the default build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probe/lds_op_probe 4000 > gpurun_out/lds_op_probe.txt 2>&1 || { cat gpurun_out/lds_op_probe.txt; exit 1; }
cat gpurun_out/lds_op_probe.txt
for name in base ${VARS:-nt192 u64 nozero} base; do
  L=""; [ $name != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$name.so"
  env $L timeout -k 10 300 python bench.py --config ${CFG:-E} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/v_$name.json 2> gpurun_out/v_$name.err || { echo "$name failed"; tail -5 gpurun_out/v_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v_$name.json'));print('$name', d['value'], d['roofline']['launch_ms'])"
done
