#!/bin/bash
# round 6 batch 24: config E with a larger k_gather_lin accumulator (variants p2tet_b500 / b540 vs the product's
# 455 blocks): P2-tet parity tests on each variant, then E A/B in row order (tools/r6/order_variants.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in p2tet_b500 p2tet_b540; do
  FEMASM_LIB=$PWD/abl/libfemasm_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deterministic.py -x -q -k "4-2" --timeout 120 --timeout-method thread > gpurun_out/b24_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc"; tail -1 gpurun_out/b24_$v.log; [ $rc -eq 0 ] || exit $rc
done
: > gpurun_out/b24_ab.txt
for rep in 1 2; do
  for lib in product p2tet_b500 p2tet_b540; do
    if [ $lib = product ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    timeout -k 10 300 python tools/r6/order_variants.py 203 row,row E > gpurun_out/b24_tmp.txt 2> gpurun_out/b24_$lib.err || { tail -5 gpurun_out/b24_$lib.err; exit 1; }
    sed "s/^{/{\"lib\": \"$lib\", /" gpurun_out/b24_tmp.txt | tee -a gpurun_out/b24_ab.txt
  done
done
