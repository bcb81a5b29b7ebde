#!/bin/bash
# half-size reference table for k_gather_lin (FA_LIN_HALFTAB) with 32 / 36 KB accumulators: parity with
# the 36 KB build, E benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
FEMASM_LIB=$PWD/abl/libfemasm_ht36.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py tests/test_gpu_plan_guards.py tests/test_gpu_split.py tests/test_gpu_linu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/s_pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name config lib
  env ${3:+FEMASM_LIB=$PWD/abl/$3} timeout -k 10 300 python bench.py --config $2 --steps 6 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/s_$1.json 2> gpurun_out/s_$1.err || { echo "$1 failed"; tail -3 gpurun_out/s_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/s_$1.json'));print('$1', d['value'], d['roofline']['launch_ms'])"
}
run E E && run E_ht36 E libfemasm_ht36.so && run E_ht32 E libfemasm_ht32.so && run E2 E && run E_ht36b E libfemasm_ht36.so
