#!/bin/bash
# round 6 batch 28: affine Q1 hexahedra through k_gather_lin -- GPU suite, then Q1 hex A/B vs the previous
# library (abl/libfemasm_prev.so: tensor-factor gather)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b28_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/b28_pytest.log; [ $rc -eq 0 ] || { grep -h "Error\|FAILED" gpurun_out/b28_pytest.log | head -20; exit $rc; }
for rep in 1 2; do
  FEMASM_LIB=$PWD/abl/libfemasm_prev.so timeout -k 10 300 python tools/r6/hex1_ab.py 160 || exit 1
  timeout -k 10 300 python tools/r6/hex1_ab.py 160 || exit 1
done
