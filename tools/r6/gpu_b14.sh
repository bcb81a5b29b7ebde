#!/bin/bash
# round 6 batch 14: chunk visiting orders with and without tail work stealing (variant "steal"), E-neo and E
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/r6/order_variants.py 203 morton,deal2,row,morton Eneo > gpurun_out/b14_eneo_base.txt 2> gpurun_out/b14_eneo_base.err || { tail -5 gpurun_out/b14_eneo_base.err; exit 1; }
cat gpurun_out/b14_eneo_base.txt
FEMASM_LIB=$PWD/abl/libfemasm_steal.so timeout -k 10 300 python tools/r6/order_variants.py 203 morton,deal2,row,morton Eneo > gpurun_out/b14_eneo_steal.txt 2> gpurun_out/b14_eneo_steal.err || { tail -5 gpurun_out/b14_eneo_steal.err; exit 1; }
cat gpurun_out/b14_eneo_steal.txt
timeout -k 10 300 python tools/r6/order_variants.py 203 row,morton,row E > gpurun_out/b14_e_base.txt 2> gpurun_out/b14_e_base.err || { tail -5 gpurun_out/b14_e_base.err; exit 1; }
cat gpurun_out/b14_e_base.txt
FEMASM_LIB=$PWD/abl/libfemasm_steal.so timeout -k 10 300 python tools/r6/order_variants.py 203 row,morton,row E > gpurun_out/b14_e_steal.txt 2> gpurun_out/b14_e_steal.err || { tail -5 gpurun_out/b14_e_steal.err; exit 1; }
cat gpurun_out/b14_e_steal.txt
