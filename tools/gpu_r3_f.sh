#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_neohookean.py tests/test_gpu_parallel.py tests/test_gpu_configs.py -k "neo or Neo or slab or neohookean" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/f_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in Eneo; do
  timeout -k 10 300 python bench.py --config $c --steps 4 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/f_$c.json 2> gpurun_out/f_$c.err || { tail -5 gpurun_out/f_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/f_$c.json'));print('$c', d['value'], d['roofline']['launch_ms'])"
done
