#!/bin/bash
# Round 5: rocprofv3 kernel stats of one config for the working-tree library and abl/libfemasm_$B.so
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
c=${CFG:-Eneo}
for lib in new ${B:-}; do
  [ -z "$lib" ] && continue
  if [ $lib = new ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_${c}_$lib -o run --output-format csv -- \
    python bench.py --config $c --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-hbm-probe --no-eneo > gpurun_out/ks_${c}_$lib.json 2> gpurun_out/ks_${c}_$lib.err || { tail -5 gpurun_out/ks_${c}_$lib.err; exit 1; }
  find gpurun_out/ks_${c}_$lib -name "*kernel_trace.csv" -delete
  f=$(find gpurun_out/ks_${c}_$lib -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; head -5 $f | cut -d, -f1-4 | cut -c1-140
done
unset FEMASM_LIB
