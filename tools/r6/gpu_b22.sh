#!/bin/bash
# round 6 batch 22: affine Q2 quads in k_gather_lin, workgroups of 256 (product) / 128 / 192 items: quad parity
# tests on each variant library, then config B A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in q2quad_nt128 q2quad_nt192; do
  FEMASM_LIB=$PWD/abl/libfemasm_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deterministic.py -x -q -k "4-2 or 4-1" --timeout 120 --timeout-method thread > gpurun_out/b22_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc"; tail -1 gpurun_out/b22_$v.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for lib in new q2quad_nt128 q2quad_nt192; do
    if [ $lib = new ]; then unset FEMASM_LIB; else export FEMASM_LIB=$PWD/abl/libfemasm_$lib.so; fi
    timeout -k 10 300 python bench.py --config B --steps 20 --warmup 3 --no-cpu-baseline --no-hbm-probe > gpurun_out/b22_B_$lib.json 2> gpurun_out/b22_B_$lib.err || { tail -5 gpurun_out/b22_B_$lib.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b22_B_$lib.json'));print('B $lib', d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
  done
done
