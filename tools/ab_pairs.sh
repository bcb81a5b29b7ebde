#!/bin/bash
# A/B of (label, env) pairs on one box, alternating REPS rounds; PAIRS="label:ENV=V,ENV2=W label2:..."
# (FEMASM_LIB=<path> in an env selects a prebuilt variant). Optional quick parity first (PARITY=1).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PARITY:-0}" = 1 ]; then
  env ${PARITY_ENV:-X=1} timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_linu.py tests/test_gpu_split.py tests/test_gpu_neohookean.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq ${REPS:-2}); do
  for pair in $PAIRS; do
    lab=${pair%%:*}; envs=${pair#*:}; envs=${envs//,/ }
    for c in ${CFGS:-E}; do
      env $envs timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline \
        > gpurun_out/ab_$lab.json 2> gpurun_out/ab_$lab.err || { echo "$lab $c failed"; tail -5 gpurun_out/ab_$lab.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab_$lab.json'));print('$lab $c', d['value'], d['roofline']['launch_ms'], d['setup_s'])"
    done
  done
done
