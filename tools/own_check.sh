#!/bin/bash
# Block-owner gather check: small-mesh parity suites, then configs C and E with the contribution
# plan (default) and with the LDS-atomic gather (FEMASM_CONTRIB=0). No build here: the .so travels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_linu.py -m gpu -q -x -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/own_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/own_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-C E}; do
  for e in ${ENVS:-FEMASM_CONTRIB=1 FEMASM_CONTRIB=0}; do
    env $e timeout -k 10 400 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline \
      > gpurun_out/own_$c.json 2> gpurun_out/own_$c.err || { tail -5 gpurun_out/own_$c.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/own_$c.json'));print('$c $e', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d.get('setup_s'))"
  done
done
