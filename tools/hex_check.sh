#!/bin/bash
# Non-affine hexahedra (MFMA element kernel + block-store gather): parity tests, then config Dmfma.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x -p no:cacheprovider \
  -k "${K:-8 or Dmfma or hex or D}" --timeout 300 --timeout-method thread > gpurun_out/hex_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/hex_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-Dmfma}; do
  timeout -k 10 400 python bench.py --config $c --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/hex_$c.json 2> gpurun_out/hex_$c.err || { tail -5 gpurun_out/hex_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/hex_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
done
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/hexprof -o run --output-format csv -- python bench.py --config Dmfma --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/hexprof.log 2>&1 || exit 1
  find gpurun_out/hexprof -name "*kernel_stats.csv" -exec cat {} \;
fi
