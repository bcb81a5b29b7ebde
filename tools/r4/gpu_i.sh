#!/bin/bash
# targeted parity (P2 table path), then A/B benches and phase clocks
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_deterministic.py tests/test_gpu_linu.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_split.py -x -q --timeout 600 --timeout-method thread > gpurun_out/i_pytest.log 2>&1 || { tail -30 gpurun_out/i_pytest.log; exit 1; }
tail -2 gpurun_out/i_pytest.log
for c in ${CFGS:-E}; do
for d in "" "--deterministic"; do
for name in ${VARS:-xchg base xchg base}; do
  L=""; [ $name != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$name.so"
  env $L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe $d > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$name failed"; tail -5 gpurun_out/v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('$c $name $d', d['value'], d['roofline']['launch_ms'])"
done; done; done
CFGS=E ./tools/r4/gpu_e.sh
