#!/bin/bash
# round 6 batch 23: affine Q2 quads in k_gather_lin: items per workgroup x accumulator blocks (variant libraries),
# quad parity tests on each, then config B A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VS="q2quad_nt128 q2quad_nt128_b767 q2quad_nt128_b511 q2quad_nt64_b511 q2quad_nt64_b383"
for v in $VS; do
  FEMASM_LIB=$PWD/abl/libfemasm_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deterministic.py -x -q -k "4-2 or 4-1" --timeout 120 --timeout-method thread > gpurun_out/b23_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc"; tail -1 gpurun_out/b23_$v.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for lib in $VS; do
    export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so
    timeout -k 10 300 python bench.py --config B --steps 20 --warmup 3 --no-cpu-baseline --no-hbm-probe > gpurun_out/b23_B_$lib.json 2> gpurun_out/b23_B_$lib.err || { tail -5 gpurun_out/b23_B_$lib.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b23_B_$lib.json'));print('B $lib', d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
  done
done
