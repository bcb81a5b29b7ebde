#!/bin/bash
# grid multiples of the generic gather (dynamic chunk counters) on D, Dq2, B, Dmfma
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name config env...
  n=$1; c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 8 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/x_$n.json 2> gpurun_out/x_$n.err || { echo "$n failed"; tail -3 gpurun_out/x_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/x_$n.json'));print('$n', d['value'], d['roofline']['launch_ms'])"
}
for c in D Dq2 B; do for m in 1 2 4 8; do run ${c}_$m $c FEMASM_GATHER_GRID_MULT=$m || exit 1; done; done
for m in 1 4; do run Dmfma_$m Dmfma FEMASM_GATHER_GRID_MULT=$m || exit 1; done
