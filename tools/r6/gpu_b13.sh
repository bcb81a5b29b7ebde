#!/bin/bash
# round 6 batch 13: E-neo with the dealt chunk order, drain store policy nt (default) / plain / sc0 sc1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in default xnts0 xnts3 default; do
  if [ $lib = default ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
  timeout -k 10 400 python bench.py --config Eneo --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/b13_$lib.json 2> gpurun_out/b13_$lib.err || { tail -5 gpurun_out/b13_$lib.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b13_$lib.json'));print('$lib', d['ms_per_step'], d['roofline']['launch_ms'])"
done
unset FEMASM_LIB
