#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
FEMASM_SLOT_ORDER=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_linu.py tests/test_gpu_split.py tests/test_gpu_fullsize.py -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_bary.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_bary.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for e in "X=1" "FEMASM_SLOT_ORDER=0"; do
    for c in E C; do
    env $e timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$e $c', d['value'], d['roofline']['launch_ms'], d['setup_s'])"
    done
  done
done
