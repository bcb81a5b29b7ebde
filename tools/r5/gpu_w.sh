#!/bin/bash
# Round 5: config E launch time and gather HBM bytes (FETCH_SIZE, WRITE_SIZE passes) per library in LIBS
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in ${LIBS:-new}; do
  if [ $lib = new ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
  for rep in 1 2; do
    timeout -k 10 240 python bench.py --config ${CFG:-E} --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe --no-eneo > gpurun_out/w_$lib.json 2> gpurun_out/w_$lib.err || { tail -5 gpurun_out/w_$lib.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/w_$lib.json'));print('$lib', d['ms_per_step'], d['roofline']['launch_ms'])"
  done
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --kernel-include-regex 'k_gather' --pmc $c -d gpurun_out/w_${lib}_$c -o run --output-format csv -- \
      python bench.py --config ${CFG:-E} --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-probe --no-eneo > gpurun_out/w_${lib}_$c.log 2>&1 || { echo "pmc $lib $c failed"; exit 1; }
  done
  python tools/pmc_summary.py gpurun_out/w_${lib}_FETCH_SIZE | grep -E "FETCH|^void" ; python tools/pmc_summary.py gpurun_out/w_${lib}_WRITE_SIZE | grep -E "WRITE"
  find gpurun_out/w_${lib}_* -name "*.csv" -delete 2>/dev/null
done
unset FEMASM_LIB
