#!/bin/bash
# One GPU session: full GPU test suite, then config-E bench with/without the slot map, then the
# other configs. Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
make -C fem-libraries_amd/csrc -j16 > gpurun_out/make.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_all.log; [ $rc -eq 0 ] || exit $rc
for sl in 0 1; do
  FEMASM_SLOTS=$sl timeout -k 10 400 python bench.py --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_E_slots$sl.json 2> gpurun_out/bench_E_slots$sl.err || exit $?
  cat gpurun_out/bench_E_slots$sl.json
done
for c in C B Dq2; do
  for sl in 0 1; do
    FEMASM_SLOTS=$sl timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline \
      > gpurun_out/bench_${c}_slots$sl.json 2> gpurun_out/bench_${c}_slots$sl.err || exit $?
    cat gpurun_out/bench_${c}_slots$sl.json
  done
done
