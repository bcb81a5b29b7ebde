#!/bin/bash
# round 6 batch 4: the whole GPU suite + smoke, then the default bench line (library warm-up, setup)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r6/gpu_suite.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/b4_bench.json 2> gpurun_out/b4_bench.err || { tail -5 gpurun_out/b4_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b4_bench.json'));print('E', d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['setup_s'], d['setup']); e=d['eneo']; print('Eneo', e.get('ms_per_step'), e.get('launch_ms'), e.get('setup_s')); print(d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
