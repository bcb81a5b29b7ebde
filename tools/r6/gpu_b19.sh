#!/bin/bash
# round 6 batch 19: repeated row-parts assemblies, base vs stealing library (tools/r6/steal_diag.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
FEMASM_LIB=$PWD/abl/libfemasm_base.so timeout -k 10 200 python tools/r6/steal_diag.py 60 1 > gpurun_out/b19_base_det.txt 2>&1; echo "base det rc=$?"; tail -4 gpurun_out/b19_base_det.txt
timeout -k 10 200 python tools/r6/steal_diag.py 60 1 > gpurun_out/b19_steal_det.txt 2>&1; echo "steal det rc=$?"; tail -6 gpurun_out/b19_steal_det.txt
timeout -k 10 200 python tools/r6/steal_diag.py 60 0 > gpurun_out/b19_steal_fp.txt 2>&1; echo "steal fp rc=$?"; tail -6 gpurun_out/b19_steal_fp.txt
FEMASM_LIB=$PWD/abl/libfemasm_base.so timeout -k 10 200 python tools/r6/steal_diag.py 60 0 > gpurun_out/b19_base_fp.txt 2>&1; echo "base fp rc=$?"; tail -4 gpurun_out/b19_base_fp.txt
