#!/bin/bash
# q-split neo gather: neo tests, E-neo bench (q-split vs one lane per item), kernel stats, PMC
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_neohookean.py tests/test_gpu_configs.py tests/test_gpu_parallel.py -k "neo or Neo or neohookean" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/m_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/m_pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name config lib
  env ${3:+FEMASM_LIB=$PWD/abl/$3} timeout -k 10 300 python bench.py --config $2 --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/m_$1.json 2> gpurun_out/m_$1.err || { echo "$1 failed"; tail -3 gpurun_out/m_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/m_$1.json'));print('$1', d['value'], d['roofline']['launch_ms'])"
}
run Eneo Eneo && run Eneo_qs1 Eneo libfemasm_qs1.so || exit 1
CFGS="Eneo" STEPS=4 bash tools/prof_all.sh || exit 1
bash tools/pmc_lin.sh Eneo
