#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plan_guards.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/d_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/d_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-E C}; do
  timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/d_$c.json 2> gpurun_out/d_$c.err || { tail -5 gpurun_out/d_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/d_$c.json'));print('$c', d['value'], d['roofline']['launch_ms'])"
done
