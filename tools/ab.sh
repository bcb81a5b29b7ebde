#!/bin/bash
# A/B on one box: bench config(s) with the in-tree library and with prev/libfemasm_prev.so
# (the previous commit's build), alternating, so box-to-box variance cancels.
# AB_ENV="VAR=value ...": the second leg is the in-tree library under that environment instead.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in cur prev; do
    for c in ${CFGS:-E}; do
      L=""; [ $lib = prev ] && L="${AB_ENV:-FEMASM_LIB=$PWD/prev/libfemasm_prev.so}"
      env $L timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$lib $c', d['value'], d['roofline']['launch_ms'])"
    done
  done
done
