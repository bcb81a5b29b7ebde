#!/bin/bash
# barrier-free chunk drain: parity (linear + neo, small and full size), then E / E-neo benches of
# the default build and variants (abl/)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_neohookean.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_plan_guards.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/k_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/k_pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name config lib
  env ${3:+FEMASM_LIB=$PWD/abl/$3} timeout -k 10 300 python bench.py --config $2 --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/k_$1.json 2> gpurun_out/k_$1.err || { echo "$1 failed"; tail -3 gpurun_out/k_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/k_$1.json'));print('$1', d['value'], d['roofline']['launch_ms'])"
}
run Eneo Eneo && run Eneo_drain0 Eneo libfemasm_drain0.so && run Eneo_w3u1 Eneo libfemasm_w3u1.so && run E E && run E_lds32 E libfemasm_lds32.so && run E_drainlin E libfemasm_drainlin.so
