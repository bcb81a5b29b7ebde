#!/bin/bash
# Round 5: per-phase clocks of k_gather_neo (timing variant) and PMC passes of the E-neo and E launches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
FEMASM_LIB=$PWD/abl/libfemasm_neo_timing.so timeout -k 10 300 python bench.py --config Eneo --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/b_tn.out 2> gpurun_out/b_tn.err || { tail -5 gpurun_out/b_tn.err; exit 1; }
python - gpurun_out/b_tn.out <<'PY'
import sys
L = [l.split()[1:] for l in open(sys.argv[1]) if l.startswith('neo_timing')]
a, b = [list(map(int, x)) for x in L[-2:]]
d = [y - x for x, y in zip(a, b)]
n = d[5]
names = ['items', 'loads+B1', 'drain', 'B3', 'bottom']
tot = sum(d[:5])
print('wave-iterations', n, ' '.join(f'{k}={v / n:.0f}' for k, v in zip(names, d[:5])), 'total', f'{tot / n:.0f}', 'MHz', f'{100.0 * tot / max(d[6], 1):.0f}')
PY
for c in Eneo E; do
  bash tools/prof_passes.sh gpurun_out/pmc_$c 'k_gather|k_neo_records|k_cell_records' -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-probe || exit $?
  python tools/pmc_summary.py gpurun_out/pmc_$c > gpurun_out/pmc_$c.txt || exit $?
  find gpurun_out/pmc_$c -name "*.csv" ! -name "*counter_collection.csv" -delete
  cat gpurun_out/pmc_$c.txt
done
