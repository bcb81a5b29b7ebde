#!/bin/bash
# round 6 batch 7: staged neo records -- neo tests, E-neo A/B, kernel stats of both
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_neohookean.py tests/test_gpu_configs.py -k "neo or Eneo" -x -q --timeout 300 --timeout-method thread > gpurun_out/b7_neo.log 2>&1
rc=$?; tail -3 gpurun_out/b7_neo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/r6/neo_ab.py 203 > gpurun_out/b7_ab.txt 2> gpurun_out/b7_ab.err || { tail -5 gpurun_out/b7_ab.err; exit 1; }
cat gpurun_out/b7_ab.txt
