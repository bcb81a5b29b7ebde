#!/bin/bash
# environment-only variants of the final build: chunk order for E-neo, grid size for E / E-neo
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name config env...
  n=$1; c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/v_$n.json 2> gpurun_out/v_$n.err || { echo "$n failed"; tail -3 gpurun_out/v_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/v_$n.json'));print('$n', d['value'], d['roofline']['launch_ms'])"
}
run Eneo Eneo X=1 && run Eneo_roworder Eneo FEMASM_CHUNK_ORDER=0 && run Eneo_grid2 Eneo FEMASM_GATHER_GRID_MULT=2 && \
run E E X=1 && run E_grid2 E FEMASM_GATHER_GRID_MULT=2 && run E_grid05 E FEMASM_GATHER_GRID_MULT=0.5
