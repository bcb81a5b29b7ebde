#!/bin/bash
# block-store gather entry unroll (Dmfma) and table-free P1 blocks (C): GPU suite, benches, kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/o_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/o_pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name config lib
  env ${3:+FEMASM_LIB=$PWD/abl/$3} timeout -k 10 300 python bench.py --config $2 --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/o_$1.json 2> gpurun_out/o_$1.err || { echo "$1 failed"; tail -3 gpurun_out/o_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/o_$1.json'));print('$1', d['value'], d['roofline']['launch_ms'])"
}
run Dmfma Dmfma && run Dmfma_u1 Dmfma libfemasm_u1.so && run Dmfma_u3 Dmfma libfemasm_u3.so && run C C && run C_p1g0 C libfemasm_p1g0.so || exit 1
CFGS="Dmfma C" STEPS=4 bash tools/prof_all.sh || exit 1
