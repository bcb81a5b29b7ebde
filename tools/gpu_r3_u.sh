#!/bin/bash
# fused records for P2 simplices (FA_LIN_FUSE2, late coordinate loads, B table): GPU suite, E benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/u_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/u_pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name config lib
  env ${3:+FEMASM_LIB=$PWD/abl/$3} timeout -k 10 300 python bench.py --config $2 --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/u_$1.json 2> gpurun_out/u_$1.err || { echo "$1 failed"; tail -3 gpurun_out/u_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/u_$1.json'));print('$1', d['value'], d['roofline']['launch_ms'])"
}
run E E && run E_off E libfemasm_fuse2off.so && run E2 E && run E_off2 E libfemasm_fuse2off.so || exit 1
CFGS="E" STEPS=6 bash tools/prof_all.sh || exit 1
