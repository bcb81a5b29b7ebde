#!/bin/bash
# A/B of the k_gather_lin drain / loop changes: targeted parity tests, then config E (and C) with the
# committed build (abl/libfemasm_head.so) alternating with the working tree build, default and deterministic
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_deterministic.py tests/test_gpu_linu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/d_pytest.log 2>&1 || { tail -40 gpurun_out/d_pytest.log; exit 1; }
tail -2 gpurun_out/d_pytest.log
for c in ${CFGS:-E}; do
for d in "" "--deterministic"; do
for name in ${VARS:-head base head base}; do
  L=""; [ $name != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$name.so"
  env $L timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-hbm-probe $d > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$name failed"; tail -5 gpurun_out/v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('$c $name $d', d['value'], d['roofline']['launch_ms'])"
done; done; done
