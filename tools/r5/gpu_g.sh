#!/bin/bash
# Round 5: k_gather_neo record-load / store ablations (timing only) on config E-neo
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in new neo_norec neo_halfrec neo_nostore2 new; do
  if [ $v = new ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$v.so; fi
  timeout -k 10 240 python bench.py --config Eneo --steps 8 --warmup 2 --no-cpu-baseline --no-hbm-probe \
    > gpurun_out/g_$v.json 2> gpurun_out/g_$v.err || { tail -5 gpurun_out/g_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/g_$v.json'));print('$v', d['ms_per_step'], d['roofline']['launch_ms'])"
done
