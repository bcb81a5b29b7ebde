#!/bin/bash
# Round 5, first GPU check: the whole GPU suite on the new build, then an A/B of the new build against
# the round-4 library (abl/libfemasm_r4.so) on configs E, E-neo and C (launch ms, HIP events).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/a_pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in E Eneo C; do
  for lib in new r4 new r4; do
    if [ $lib = r4 ]; then export FEMASM_LIB=$PWD/abl/libfemasm_r4.so; else unset FEMASM_LIB; fi
    timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe \
      > gpurun_out/a_${cfg}_${lib}.json 2> gpurun_out/a_${cfg}_${lib}.err || { tail -5 gpurun_out/a_${cfg}_${lib}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/a_${cfg}_${lib}.json'));print('$cfg $lib', d['ms_per_step'], d['roofline']['launch_ms'], d['setup'])"
  done
done
unset FEMASM_LIB
