#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for e in "X=1" "FEMASM_SLOT_ORDER=0" "FEMASM_SLOT_ORDER=1" "FEMASM_SLOTS=0"; do
    env $e FEMASM_LIB=$PWD/abl/libfemasm_fz0.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$e', d['value'], d['roofline']['launch_ms'], d['setup_s'])"
  done
done
