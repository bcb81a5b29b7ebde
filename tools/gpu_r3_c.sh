#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python tools/probe/hbm_probe.py > gpurun_out/probe3.txt 2>&1 || exit 1
grep -E "oneshot|torch|write plain" gpurun_out/probe3.txt
bash tools/lin_ablate.sh && CFG=C bash tools/lin_ablate.sh
