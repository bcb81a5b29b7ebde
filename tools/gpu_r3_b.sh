#!/bin/bash
# round 3: new k_gather_lin parity (affine simplices) + E / C quick benches + AD damage tests + probe
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_parallel.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/b_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/b_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in E C; do
  timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/b_$c.json 2> gpurun_out/b_$c.err || { tail -5 gpurun_out/b_$c.err; exit 1; }
  FEMASM_LIN_GATHER=0 timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/b_${c}_old.json 2> gpurun_out/b_${c}_old.err || { tail -5 gpurun_out/b_${c}_old.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_$c.json'));o=json.load(open('gpurun_out/b_${c}_old.json'));print('$c new', d['value'], d['roofline']['launch_ms'], 'old', o['value'], o['roofline']['launch_ms'])"
done
timeout -k 10 180 python tools/probe/hbm_probe.py > gpurun_out/probe2.txt 2>&1; cat gpurun_out/probe2.txt
