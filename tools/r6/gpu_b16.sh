#!/bin/bash
# round 6 batch 16: the 3-rank slab test with the base library and with the stealing product library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="tests/test_gpu_parallel.py::test_slab_problem_gpu_gloo"
FEMASM_LIB=$PWD/abl/libfemasm_base.so timeout -k 10 200 python -u -m pytest "$T" -q --timeout 120 --timeout-method thread > gpurun_out/b16_base.log 2>&1; echo "base rc=$?"; tail -2 gpurun_out/b16_base.log
timeout -k 10 200 python -u -m pytest "$T" -q --timeout 120 --timeout-method thread > gpurun_out/b16_steal.log 2>&1; echo "steal rc=$?"; tail -2 gpurun_out/b16_steal.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_split.py -q --timeout 120 --timeout-method thread > gpurun_out/b16_steal2.log 2>&1; echo "steal2 rc=$?"; tail -2 gpurun_out/b16_steal2.log
grep -h "AssertionError: rank" gpurun_out/b16_*.log | head
