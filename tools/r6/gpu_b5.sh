#!/bin/bash
# round 6 batch 5: LDS quarter arrays in k_plan_perm -- suite, setup phases, the E line's setup
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r6/gpu_suite.sh || exit 1
timeout -k 10 300 python tools/r6/setup_profile.py > gpurun_out/b5_setup.json 2> gpurun_out/b5_setup.err || { tail -5 gpurun_out/b5_setup.err; exit 1; }
cat gpurun_out/b5_setup.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b5_prof_setup -o setup -- python tools/r6/setup_profile.py > gpurun_out/b5_setup_prof.log 2>&1 || { tail -5 gpurun_out/b5_setup_prof.log; exit 1; }
f=$(find gpurun_out/b5_prof_setup -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/b5_setup_kernel_stats.csv; head -10 gpurun_out/b5_setup_kernel_stats.csv | cut -c1-140
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-eneo --no-cpu-baseline > gpurun_out/b5_bench.json 2> gpurun_out/b5_bench.err || { tail -5 gpurun_out/b5_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b5_bench.json'));print('E', d['ms_per_step'], d['setup_s'], d['setup'])"
