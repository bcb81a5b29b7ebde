#!/bin/bash
# neo-Hookean gather variants: small-mesh parity per prebuilt library, then config E-neo timing.
# VARIANTS="label:lib ..." (lib relative to the repo root; "default" = the in-tree build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $VARIANTS; do
  lab=${v%%:*}; lib=${v#*:}
  [ "$lib" = default ] && e=X=1 || e=FEMASM_LIB=$PWD/$lib
  env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_neohookean.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/neo_par_$lab.log 2>&1 || { echo "$lab parity failed"; tail -15 gpurun_out/neo_par_$lab.log; exit 1; }
  echo "$lab parity: $(tail -1 gpurun_out/neo_par_$lab.log)"
done
for rep in $(seq ${REPS:-1}); do
  for v in $VARIANTS; do
    lab=${v%%:*}; lib=${v#*:}
    [ "$lib" = default ] && e=X=1 || e=FEMASM_LIB=$PWD/$lib
    env $e timeout -k 10 300 python bench.py --config Eneo --steps ${STEPS:-3} --warmup 2 --no-cpu-baseline \
      > gpurun_out/neo_$lab.json 2> gpurun_out/neo_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/neo_$lab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/neo_$lab.json'));print('$lab', d['value'], d['roofline']['launch_ms'])"
  done
done
