#!/bin/bash
# Round 5: several libraries / bench options alternating on one box, twice.
# usage: RUNS="new:--plan-search kr1:--plan-search new:" CFGS="E" bash tools/r5/gpu_multi.sh
#   (lib "new" = the working tree; others abl/libfemasm_<lib>.so; after ':' extra bench flags)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-E}; do
  for rep in 1 2; do
    for run in $RUNS; do
      lib=${run%%:*}; extra=${run#*:}; extra=${extra//,/ }
      if [ $lib = new ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
      tag=${cfg}_${lib}_$(echo "$extra" | tr -dc 'a-z')_$rep
      timeout -k 10 240 python bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-hbm-probe --no-eneo $extra \
        > gpurun_out/mr_$tag.json 2> gpurun_out/mr_$tag.err || { tail -5 gpurun_out/mr_$tag.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/mr_$tag.json'));print('$cfg $lib [$extra]', d['ms_per_step'], d['roofline']['launch_ms'], d['setup']['plan_s'])"
    done
  done
done
unset FEMASM_LIB
