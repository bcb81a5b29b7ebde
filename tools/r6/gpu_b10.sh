#!/bin/bash
# round 6 batch 10: suite (two-per-lane sparsity sort); chunk order x store cache policy on config E
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r6/gpu_suite.sh || exit 1
timeout -k 10 300 python tools/r6/setup_profile.py > gpurun_out/b10_setup.json 2> gpurun_out/b10_setup.err || { tail -5 gpurun_out/b10_setup.err; exit 1; }
cat gpurun_out/b10_setup.json
for lib in default nts0 nts3; do
  if [ $lib = default ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
  timeout -k 10 400 python tools/r6/order_variants.py 203 morton,row,morton,row > gpurun_out/b10_order_$lib.txt 2> gpurun_out/b10_order_$lib.err || { tail -5 gpurun_out/b10_order_$lib.err; exit 1; }
  echo "== $lib"; cat gpurun_out/b10_order_$lib.txt | cut -c1-100
done
unset FEMASM_LIB
