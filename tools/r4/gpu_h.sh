#!/bin/bash
# full GPU suite, then A/B benches of the drains and the phase clocks
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_pytest.log 2>&1 || { tail -30 gpurun_out/gpu_pytest.log; exit 1; }
tail -2 gpurun_out/gpu_pytest.log
for c in E C; do
for d in "" "--deterministic"; do
for name in ${VARS:-dyn base lin_drain2 lin_drain0 dyn base lin_drain2 lin_drain0}; do
  L=""; [ $name != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$name.so"
  env $L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe $d > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$name failed"; tail -5 gpurun_out/v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('$c $name $d', d['value'], d['roofline']['launch_ms'])"
done; done; done
./tools/r4/gpu_e.sh
