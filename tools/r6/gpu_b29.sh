#!/bin/bash
# round 6 batch 29: the records' bc bits from the constrained nodes (k_rec_bcbits) -- GPU suite, then E / B A/B
# against the previous library (abl/libfemasm_prev.so)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b29_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/b29_pytest.log; [ $rc -eq 0 ] || { grep -h "Error\|FAILED" gpurun_out/b29_pytest.log | head -20; exit $rc; }
: > gpurun_out/b29_ab.txt
for rep in 1 2; do
  for lib in prev product; do
    if [ $lib = product ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    for cfg in E:203 B:1000; do
      c=${cfg%%:*}; n=${cfg#*:}
      timeout -k 10 300 python tools/r6/order_variants.py $n row,row $c > gpurun_out/b29_tmp.txt 2> gpurun_out/b29_$lib.err || { tail -5 gpurun_out/b29_$lib.err; exit 1; }
      sed "s/^{/{\"lib\": \"$lib\", \"cfg\": \"$c\", /" gpurun_out/b29_tmp.txt | tee -a gpurun_out/b29_ab.txt
    done
  done
done
unset FEMASM_LIB
CFGS="E" STEPS=5 bash tools/prof_all.sh > gpurun_out/b29_prof.txt 2>&1 || { tail -5 gpurun_out/b29_prof.txt; exit 1; }
grep -E "k_cell_records|k_rec_bcbits|k_gather_lin" gpurun_out/prof_E/run_kernel_stats.csv | cut -d, -f1-4
