#!/bin/bash
# round 6 batch 25: config C (P1 tets, fused k_gather_lin): 128-item workgroups, 8 / 24 KB accumulators (variants)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VS="p1tet_nt128 p1tet_nt128_lds8k p1tet_lds24k"
for v in $VS; do
  FEMASM_LIB=$PWD/abl/libfemasm_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deterministic.py -x -q -k "4-1" --timeout 120 --timeout-method thread > gpurun_out/b25_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc"; tail -1 gpurun_out/b25_$v.log; [ $rc -eq 0 ] || exit $rc
done
: > gpurun_out/b25_ab.txt
for rep in 1 2; do
  for lib in product $VS; do
    if [ $lib = product ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    timeout -k 10 300 python tools/r6/order_variants.py 119 row,row C > gpurun_out/b25_tmp.txt 2> gpurun_out/b25_$lib.err || { tail -5 gpurun_out/b25_$lib.err; exit 1; }
    sed "s/^{/{\"lib\": \"$lib\", /" gpurun_out/b25_tmp.txt | tee -a gpurun_out/b25_ab.txt
  done
done
