#!/bin/bash
# E bench variance with / without the HBM probe, the HBM write-pattern probe, k_gather_lin ablations, LDS PMC of E
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python tools/probe/hbm_probe.py > gpurun_out/i_probe.txt 2>&1 || { tail -5 gpurun_out/i_probe.txt; exit 1; }
for r in a b; do
  for p in probe noprobe; do
    A=""; [ $p = noprobe ] && A="--no-hbm-probe"
    timeout -k 10 300 python bench.py --config E --steps 10 --warmup 2 --no-cpu-baseline $A > gpurun_out/i_E_$p$r.json 2> gpurun_out/i_E_$p$r.err || { tail -3 gpurun_out/i_E_$p$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/i_E_$p$r.json'));print('E $p$r', d['ms_per_step'], d['roofline']['launch_ms'])"
  done
done
bash tools/lin_ablate.sh || exit 1
bash tools/pmc_lin.sh E
