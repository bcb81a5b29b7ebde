#!/bin/bash
# round 6 batch 12: chunk visiting order for config E-neo (Morton vs row order per XCD eighth)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/r6/order_variants.py 203 morton,deal1,deal2,deal4,deal8,deal16,morton,deal4,deal2 Eneo > gpurun_out/b12_order_Eneo.txt 2> gpurun_out/b12_order_Eneo.err || { tail -5 gpurun_out/b12_order_Eneo.err; exit 1; }
cat gpurun_out/b12_order_Eneo.txt | cut -c1-110
