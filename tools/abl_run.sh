#!/bin/bash
# Bench config E with the in-tree library and each prebuilt ablation variant in abl/ (timing only).
set -o pipefail
export TMPDIR=/tmp FEMASM_ORDER_KICKS=${FEMASM_ORDER_KICKS:-0}
mkdir -p gpurun_out
for k in 0 ${ABL:-3 4 6 7 8 10}; do
  L=""; [ $k != 0 ] && L="FEMASM_LIB=$PWD/abl/libfemasm_abl$k.so"
  env $L timeout -k 10 300 python bench.py --config ${CFG:-E} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abl$k.json 2> gpurun_out/abl$k.err || { echo "abl $k failed"; tail -3 gpurun_out/abl$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abl$k.json'));print('abl$k', d['value'], d['roofline']['launch_ms'])"
done
