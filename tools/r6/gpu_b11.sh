#!/bin/bash
# round 6 batch 11: compact slot words + row order for P2 tets -- suite, then the plan A/B on E and C
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r6/gpu_suite.sh || exit 1
timeout -k 10 500 python tools/r6/lin_ab.py 203 E > gpurun_out/b11_ab_E.txt 2> gpurun_out/b11_ab_E.err || { tail -5 gpurun_out/b11_ab_E.err; exit 1; }
cat gpurun_out/b11_ab_E.txt | cut -c1-110
timeout -k 10 300 python tools/r6/lin_ab.py 119 C > gpurun_out/b11_ab_C.txt 2> gpurun_out/b11_ab_C.err || { tail -5 gpurun_out/b11_ab_C.err; exit 1; }
cat gpurun_out/b11_ab_C.txt | cut -c1-110
