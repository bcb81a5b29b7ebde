#!/bin/bash
# round 6 batch 27: the XDMF input path on the GPU, then the whole GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/b27_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/b27_pytest.log; grep -h "FAILED\|Error" gpurun_out/b27_pytest.log | head; exit $rc
