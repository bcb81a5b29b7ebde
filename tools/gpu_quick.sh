#!/bin/bash
# Quick GPU cycle: GPU tests (optionally a -k filter in $1), then benches of configs E, C, B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
make -C fem-libraries_amd/csrc -j16 > gpurun_out/make.log 2>&1 || exit 1
K=${1:-}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x ${K:+-k "$K"} > gpurun_out/pytest_quick.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-E C B}; do
  timeout -k 10 400 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_q_$c.json 2> gpurun_out/bench_q_$c.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_q_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
done
