#!/bin/bash
# round 6 batch 9: hash-set sparsity -- pattern tests, the whole suite, setup phases
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pattern_check.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/b9_pat.log 2>&1
rc=$?; tail -3 gpurun_out/b9_pat.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6/gpu_suite.sh || exit 1
timeout -k 10 300 python tools/r6/setup_profile.py > gpurun_out/b9_setup.json 2> gpurun_out/b9_setup.err || { tail -5 gpurun_out/b9_setup.err; exit 1; }
cat gpurun_out/b9_setup.json
