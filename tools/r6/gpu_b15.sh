#!/bin/bash
# round 6 batch 15: k_gather_lin tail work stealing in the product library vs the base (abl/libfemasm_base.so),
# config E and C in their default (row) order, alternating libraries; then the GPU suite on the product library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/b15_ab.txt
for rep in 1 2; do
  for lib in base steal; do
    if [ $lib = base ]; then export FEMASM_LIB=$PWD/abl/libfemasm_base.so; else unset FEMASM_LIB; fi
    for cfg in E:203 C:119; do
      c=${cfg%%:*}; n=${cfg#*:}
      timeout -k 10 300 python tools/r6/order_variants.py $n row,row $c > gpurun_out/b15_tmp.txt 2> gpurun_out/b15_$lib.err || { tail -5 gpurun_out/b15_$lib.err; exit 1; }
      sed "s/^{/{\"lib\": \"$lib\", \"cfg\": \"$c\", /" gpurun_out/b15_tmp.txt >> gpurun_out/b15_ab.txt
    done
  done
done
unset FEMASM_LIB
cat gpurun_out/b15_ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b15_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/b15_pytest.log; exit $rc
