#!/bin/bash
# Round-2 GPU session: full GPU suite (incl. full-size configs), then the headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_configs.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -v --durations=0 --timeout 400 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_configs.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_configs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_E.json 2> gpurun_out/bench_E.err || exit $?
cat gpurun_out/bench_E.json; tail -2 gpurun_out/bench_E.err
