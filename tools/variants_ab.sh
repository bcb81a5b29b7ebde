#!/bin/bash
# A/B of library variants on one box: the in-tree build ("cur") and abl/libfemasm_<name>.so, each
# benched on CFGS (default E), alternating over REPS rounds so box drift cancels. Optional quick
# parity first (PARITY=1: the gather parity tests on the in-tree build).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_linu.py tests/test_gpu_split.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq ${REPS:-2}); do
  for v in cur ${VARIANTS}; do
    for c in ${CFGS:-E}; do
      L=""; [ $v != cur ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$v.so"
      env $L ${AB_ENV:-} timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline \
        > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "$v $c failed"; tail -5 gpurun_out/ab_$v.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v $c', d['value'], d['roofline']['launch_ms'], d['setup_s'])"
    done
  done
done
