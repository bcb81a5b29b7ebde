#!/bin/bash
# A/B benches (no tests) and phase clocks
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-E}; do
for dm in ${DETS:-def}; do
d=""; [ "$dm" = det ] && d="--deterministic"
for name in ${VARS:-base}; do
  L=""; [ $name != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$name.so"
  env $L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe $d > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$name failed"; tail -5 gpurun_out/v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('$c $name $d', d['value'], d['roofline']['launch_ms'])"
done; done; done
[ -n "$TIMING" ] && CFGS=E ./tools/r4/gpu_e.sh
exit 0
