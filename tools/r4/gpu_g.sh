#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for name in ${VARS:-base lin_drain0 dyn}; do
  L=""; [ $name != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$name.so"
  echo "== $name"
  env $L timeout -k 10 300 python tools/r4/diag_default.py 2>&1 | tail -20 || exit 1
done
