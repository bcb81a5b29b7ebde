#!/bin/bash
# E-neo grid multiple A/B, alternating (env only)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name config env...
  n=$1; c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/y_$n.json 2> gpurun_out/y_$n.err || { echo "$n failed"; tail -3 gpurun_out/y_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/y_$n.json'));print('$n', d['value'], d['roofline']['launch_ms'])"
}
for p in a b c; do run Eneo_m1_$p Eneo FEMASM_GATHER_GRID_MULT=1 && run Eneo_m64_$p Eneo FEMASM_GATHER_GRID_MULT=64 || exit 1; done
