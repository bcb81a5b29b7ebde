set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/prof_passes.sh gpurun_out/pmcE2 'k_gather|k_cell_records' -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
python tools/pmc_summary.py gpurun_out/pmcE2 > gpurun_out/pmcE2_summary.txt; cat gpurun_out/pmcE2_summary.txt
