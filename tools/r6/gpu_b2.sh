#!/bin/bash
# round 6 batch 2: deterministic (prefetched block exponents), setup phases + kernel trace, HBM write
# probe variants, the default bench line of this build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_deterministic.py -x -q --timeout 240 --timeout-method thread > gpurun_out/b2_det.log 2>&1
rc=$?; tail -2 gpurun_out/b2_det.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --deterministic --no-eneo --no-cpu-baseline --no-hbm-probe > gpurun_out/b2_det_E.json 2> gpurun_out/b2_det_E.err || { tail -5 gpurun_out/b2_det_E.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b2_det_E.json'));print('det E', d['ms_per_step'], d['roofline']['launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b2_prof_setup -o setup -- python tools/r6/setup_profile.py > gpurun_out/b2_setup_prof.log 2>&1 || { tail -5 gpurun_out/b2_setup_prof.log; exit 1; }
grep '^{' gpurun_out/b2_setup_prof.log
f=$(find gpurun_out/b2_prof_setup -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/b2_setup_kernel_stats.csv; head -14 gpurun_out/b2_setup_kernel_stats.csv | cut -c1-160
timeout -k 10 300 python tools/probe/hbm_probe.py > gpurun_out/b2_hbm_probe.txt 2>&1 || { tail -5 gpurun_out/b2_hbm_probe.txt; exit 1; }
cat gpurun_out/b2_hbm_probe.txt | grep GiB
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b2_bench.json 2> gpurun_out/b2_bench.err || { tail -5 gpurun_out/b2_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b2_bench.json'));print('E', d['ms_per_step'], d['roofline']['launch_ms'], d['setup_s'], d['setup']); e=d['eneo']; print('Eneo', e.get('ms_per_step'), e.get('launch_ms'), e.get('setup_s'))"
