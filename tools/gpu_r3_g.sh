#!/bin/bash
# quick benches of every config after a kernel change (launch ms); E also with the generic gather
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name config [env]
  env ${3:-X=1} timeout -k 10 300 python bench.py --config $2 --steps 4 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/g_$1.json 2> gpurun_out/g_$1.err || { echo "$1 failed"; tail -3 gpurun_out/g_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/g_$1.json'));print('$1', d['value'], d['roofline']['launch_ms'])"
}
for c in ${CFGS:-E Eneo C D Dmfma B Dq2 A}; do run $c $c || exit 1; done
run Egeneric E FEMASM_LIN_GATHER=0 && run Cgeneric C FEMASM_LIN_GATHER=0
