#!/bin/bash
# Build compile-time variants of libfemasm into abl/ and bench each with FEMASM_LIB.
# (SKIP_BUILD=1: use the abl/ libraries built beforehand, e.g. in the CPU container)
# usage: VARIANTS="name:-DFLAG=1 -DX=2;name2:" CFG=E NARG="--n 120" bash tools/variants.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out abl
IFS=';' read -ra VS <<< "$VARIANTS"
cd fem-libraries_amd/csrc
[ -n "$SKIP_BUILD" ] || for v in "${VS[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics $flags \
    -o ../../abl/libfemasm_$name.so femasm.hip &
done
wait
cd ../..
for v in "${VS[@]}"; do
  name=${v%%:*}
  for cfg in ${CFG:-E}; do
    FEMASM_LIB=$PWD/abl/libfemasm_$name.so timeout -k 10 600 python bench.py --config $cfg ${NARG:-} --steps ${STEPS:-5} --warmup 2 \
      --no-cpu-baseline > gpurun_out/var_${name}_$cfg.json 2> gpurun_out/var_${name}_$cfg.err || { echo "$name failed"; tail -3 gpurun_out/var_${name}_$cfg.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/var_${name}_$cfg.json'));print('$name $cfg', d['value'], d['roofline']['launch_ms'])"
  done
done
