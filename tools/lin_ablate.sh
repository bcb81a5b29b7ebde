#!/bin/bash
# Timing-only ablations of k_gather_lin (FA_LIN_ABL, prebuilt into abl/): bench config E with each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 0 ${ABL:-1 2 3 4 5}; do
  L=""; [ $k != 0 ] && L="FEMASM_LIB=$PWD/abl/libfemasm_lin$k.so"
  env $L timeout -k 10 300 python bench.py --config ${CFG:-E} --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/labl$k.json 2> gpurun_out/labl$k.err || { echo "abl $k failed"; tail -3 gpurun_out/labl$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/labl$k.json'));print('lin_abl$k', d['value'], d['roofline']['launch_ms'])"
done
