#!/bin/bash
# Round-2 first GPU session: GPU test suite, headline bench, LDS accumulate-op probe.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_E.json 2> gpurun_out/bench_E.err || exit $?
cat gpurun_out/bench_E.json
timeout -k 10 60 ./tools/probe/lds_atomic_probe 2000 > gpurun_out/lds_atomic_probe.txt 2>&1 || exit $?
cat gpurun_out/lds_atomic_probe.txt
