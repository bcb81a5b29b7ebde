#!/bin/bash
# Round 5: E with 32 / 36 / 38 KB accumulators (variant libraries), alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in new lin38k lin36k new lin38k lin36k; do
  if [ $v = new ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$v.so; fi
  timeout -k 10 240 python bench.py --config ${CFG:-E} --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe --no-eneo \
    > gpurun_out/m_$v.json 2> gpurun_out/m_$v.err || { tail -5 gpurun_out/m_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/m_$v.json'));print('$v', d['ms_per_step'], d['roofline']['launch_ms'], d['setup']['plan_s'])"
done
