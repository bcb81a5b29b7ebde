#!/bin/bash
# round 6 batch 6: device chunking -- plan tests, whole suite, setup phases, default bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plan_guards.py -x -q --timeout 240 --timeout-method thread > gpurun_out/b6_plan.log 2>&1
rc=$?; tail -3 gpurun_out/b6_plan.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6/gpu_suite.sh || exit 1
timeout -k 10 300 python tools/r6/setup_profile.py > gpurun_out/b6_setup.json 2> gpurun_out/b6_setup.err || { tail -5 gpurun_out/b6_setup.err; exit 1; }
cat gpurun_out/b6_setup.json
timeout -k 10 600 python bench.py > gpurun_out/b6_bench.json 2> gpurun_out/b6_bench.err || { tail -5 gpurun_out/b6_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b6_bench.json'));print('E', d['ms_per_step'], d['roofline']['frac'], d['setup_s'], d['setup']); e=d['eneo']; print('Eneo', e.get('ms_per_step'), e.get('setup_s'), e.get('setup'))"
