#!/bin/bash
# Per-phase shader-clock breakdown of the gather (FA_GATHER_TIMING build, config E by default).
set -o pipefail
export TMPDIR=/tmp
mkdir -p abl gpurun_out
(cd fem-libraries_amd/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics \
  -DFA_GATHER_TIMING=1 ${EXTRA:-} -o ../../abl/libt.so femasm.hip) || exit 1
FEMASM_LIB=$PWD/abl/libt.so timeout -k 10 300 python bench.py --config ${CFG:-E} --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/t.json 2> gpurun_out/t.err || { tail gpurun_out/t.err; exit 1; }
grep "gather timing" gpurun_out/t.err | tail -1
python -c "import json;d=json.load(open('gpurun_out/t.json'));print(d['value'], d['roofline']['launch_ms'])"
