#!/bin/bash
# Round 5 A/B: the working-tree library against abl/libfemasm_$B.so, alternating on one box.
# usage: B=h1 CFGS="E Eneo C" PYT=1 bash tools/r5/gpu_ab.sh   (PYT=1: the GPU suite first)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PYT:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CFGS:-E Eneo C}; do
  for lib in new $B new $B; do
    if [ $lib = new ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    timeout -k 10 240 python bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-hbm-probe --no-eneo ${EXTRA:-} \
      > gpurun_out/ab_${cfg}_${lib}.json 2> gpurun_out/ab_${cfg}_${lib}.err || { tail -5 gpurun_out/ab_${cfg}_${lib}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${cfg}_${lib}.json'));print('$cfg $lib', d['ms_per_step'], d['roofline']['launch_ms'], d['setup']['plan_s'])"
  done
done
unset FEMASM_LIB
