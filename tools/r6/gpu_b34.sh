#!/bin/bash
# round 6 batch 34: the whole GPU suite three times on the final release library (intermittent-failure check)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/b34_pytest_$r.log 2>&1; rc=$?
  echo "run $r rc=$rc"; tail -2 gpurun_out/b34_pytest_$r.log
  [ $rc -eq 0 ] || { grep -h "AssertionError\|FAILED" gpurun_out/b34_pytest_$r.log | head; exit $rc; }
done
