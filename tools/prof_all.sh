#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py for each config (no CPU baseline under the profiler)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-E Eneo D Dq2 B C A}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python bench.py --config $c --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-eneo > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.err || { tail -5 gpurun_out/prof_$c.err; exit 1; }
  find gpurun_out/prof_$c -name "*kernel_trace.csv" -delete
  python -c "import json;d=json.load(open('gpurun_out/prof_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
  f=$(find gpurun_out/prof_$c -name "*kernel_stats.csv" | head -1); head -4 $f | cut -d, -f1-4 | cut -c1-150
done
