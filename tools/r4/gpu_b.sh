#!/bin/bash
# deterministic-mode tests + full GPU suite + E / C benches (default vs deterministic)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_deterministic.py -x -v --timeout 600 --timeout-method thread > gpurun_out/det_pytest.log 2>&1 || { tail -40 gpurun_out/det_pytest.log; exit 1; }
tail -3 gpurun_out/det_pytest.log
for c in E C; do
  for d in "" "--deterministic"; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe $d > gpurun_out/b_${c}${d}.json 2> gpurun_out/b_${c}${d}.err || { echo "bench $c $d failed"; tail -5 gpurun_out/b_${c}${d}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b_${c}${d}.json'));print('$c $d', d['value'], d['roofline']['launch_ms'])"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_pytest.log 2>&1 || { tail -40 gpurun_out/gpu_pytest.log; exit 1; }
tail -3 gpurun_out/gpu_pytest.log
