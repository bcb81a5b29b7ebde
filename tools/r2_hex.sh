#!/bin/bash
# affine tensor gather: parity (small meshes, full-size B / D / D'), then benches of B, D, D', E
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_hex.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_hex.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-B D Dq2 E}; do
  timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -5 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', d['value'], d['roofline']['launch_ms'], d['setup_s'], d['roofline']['frac'])"
done
