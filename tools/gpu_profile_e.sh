#!/bin/bash
# Profile set for the headline bench (config E): kernel-trace stats of `python bench.py` (no CPU
# baseline: its worker processes must not start under the profiler), then separate PMC passes of
# the assembly kernels -> traffic record. Large per-dispatch traces are deleted (stats kept).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
make -C fem-libraries_amd/csrc -j16 > gpurun_out/make.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_E -o run --output-format csv -- \
  python bench.py --no-cpu-baseline > gpurun_out/prof_E_bench.json 2> gpurun_out/prof_E_bench.err || exit $?
find gpurun_out/prof_E -name "*kernel_trace.csv" -delete
cat gpurun_out/prof_E_bench.json
bash tools/prof_passes.sh gpurun_out/pmcE 'k_gather|k_cell_records' -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $?
python tools/pmc_summary.py gpurun_out/pmcE > gpurun_out/pmcE_summary.txt || exit $?
python tools/pmc_summary.py gpurun_out/pmcE E:203 gpurun_out/traffic.json || exit $?
find gpurun_out/pmcE -name "*kernel_trace.csv" -delete
cat gpurun_out/pmcE_summary.txt gpurun_out/traffic.json
