#!/bin/bash
# neo-Hookean gather ablations (timing only) + plain-store lin variant
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name lib config
  env ${2:+FEMASM_LIB=$PWD/abl/$2} timeout -k 10 300 python bench.py --config $3 --steps 4 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/e_$1.json 2> gpurun_out/e_$1.err || { echo "$1 failed"; tail -3 gpurun_out/e_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e_$1.json'));print('$1', d['value'], d['roofline']['launch_ms'])"
}
run eneo "" Eneo && run neo1 libfemasm_neo1.so Eneo && run neo2 libfemasm_neo2.so Eneo && run neo8 libfemasm_neo8.so Eneo && run E "" E && run Eplain libfemasm_linplain.so E && run E2 "" E
