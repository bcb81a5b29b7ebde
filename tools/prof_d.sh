#!/bin/bash
# rocprof kernel stats of config D (Q3 hex, MFMA path) and D' (Q2 hex)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-D Dq2}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.err || { tail -5 gpurun_out/prof_$c.err; exit 1; }
  find gpurun_out/prof_$c -name "*kernel_trace.csv" -delete
  cat gpurun_out/prof_$c.json | python -c "import json,sys;d=json.load(sys.stdin);print('$c', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
  f=$(find gpurun_out/prof_$c -name "*kernel_stats.csv" | head -1); head -8 $f | cut -c1-200
done
