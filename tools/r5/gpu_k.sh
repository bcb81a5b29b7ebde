#!/bin/bash
# Round 5: E with and without the plan's alternating-path search (FA_PLAN_ORDER_SEARCH), alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in plain search plain search; do
  f=""; [ $v = search ] && f="--plan-search"
  timeout -k 10 240 python bench.py --config E --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe --no-eneo $f \
    > gpurun_out/k_$v.json 2> gpurun_out/k_$v.err || { tail -5 gpurun_out/k_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/k_$v.json'));print('$v', d['ms_per_step'], d['roofline']['launch_ms'], d['setup']['plan_s'])"
done
