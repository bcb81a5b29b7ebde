#!/bin/bash
# k_gather_lin grid size sweep, large multiples (FEMASM_GATHER_GRID_MULT)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name config env...
  n=$1; c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 8 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/w_$n.json 2> gpurun_out/w_$n.err || { echo "$n failed"; tail -3 gpurun_out/w_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/w_$n.json'));print('$n', d['value'], d['roofline']['launch_ms'])"
}
for m in 32 64 128 256 512 1024; do run E_$m E FEMASM_GATHER_GRID_MULT=$m || exit 1; done
for m in 32 128; do run C_$m C FEMASM_GATHER_GRID_MULT=$m || exit 1; done
for m in 0.5 1; do run Eneo_$m Eneo FEMASM_GATHER_GRID_MULT=$m || exit 1; done
