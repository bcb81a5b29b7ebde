#!/bin/bash
# neo-Hookean M gather: neo GPU tests, then E-neo bench with k_gather_neo and with k_gather's neo items
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_neohookean.py tests/test_gpu_configs.py tests/test_gpu_parallel.py -k "neo or Neo or neohookean" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/j_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/j_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  FEMASM_NEO_M=$v timeout -k 10 300 python bench.py --config Eneo --steps 4 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/j_Eneo$v.json 2> gpurun_out/j_Eneo$v.err || { tail -5 gpurun_out/j_Eneo$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/j_Eneo$v.json'));print('Eneo M=$v', d['value'], d['roofline']['launch_ms'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_j -o run --output-format csv -- python bench.py --config Eneo --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/prof_j.log 2>&1 || { tail -5 gpurun_out/prof_j.log; exit 1; }
f=$(find gpurun_out/prof_j -name "*kernel_stats.csv" | head -1); head -6 $f | cut -d, -f1-4 | cut -c1-150
find gpurun_out/prof_j -name "*kernel_trace.csv" -delete
for v in 30720 32768; do
  FEMASM_LIB=$PWD/abl/libfemasm_lds$v.so timeout -k 10 300 python bench.py --config E --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/j_Elds$v.json 2> gpurun_out/j_Elds$v.err || { tail -5 gpurun_out/j_Elds$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/j_Elds$v.json'));print('E lds $v', d['value'], d['roofline']['launch_ms'])"
done
timeout -k 10 300 python bench.py --config E --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/j_E.json 2> gpurun_out/j_E.err || { tail -5 gpurun_out/j_E.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/j_E.json'));print('E default', d['value'], d['roofline']['launch_ms'])"
