#!/bin/bash
# Build timing-only ablation variants of libfemasm (-DFA_ABL=k) into abl/ and bench config E with
# each (FEMASM_LIB). Results are wrong by construction: bench only, never tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out abl
cd fem-libraries_amd/csrc
for k in ${ABL:-0 1 2 3 4}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -DFA_ABL=$k \
    ${EXTRA:-} -o ../../abl/libfemasm_abl$k.so femasm.hip &
done
wait
cd ../..
for k in ${ABL:-0 1 2 3 4}; do
  FEMASM_LIB=$PWD/abl/libfemasm_abl$k.so timeout -k 10 400 python bench.py --config ${CFG:-E} ${NARG:-} --steps 5 --warmup 2 \
    --no-cpu-baseline > gpurun_out/abl$k.json 2> gpurun_out/abl$k.err || { echo "abl $k failed"; tail -3 gpurun_out/abl$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abl$k.json'));print('abl$k', d['value'], d['roofline']['launch_ms'])"
done
