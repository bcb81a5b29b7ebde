#!/bin/bash
# Round 5: per-phase clocks of k_gather_neo for timing-variant libraries (LIBS="neo_timing neo2+neo_timing")
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in ${LIBS:-neo_timing}; do
  FEMASM_LIB=$PWD/abl/libfemasm_$lib.so timeout -k 10 300 python bench.py --config Eneo --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe --no-eneo > gpurun_out/nt_$lib.out 2> gpurun_out/nt_$lib.err || { tail -5 gpurun_out/nt_$lib.err; exit 1; }
  python - gpurun_out/nt_$lib.out $lib <<'PY'
import sys
L = [l.split()[1:] for l in open(sys.argv[1]) if l.startswith('neo_timing')]
a, b = [list(map(int, x)) for x in L[-2:]]
d = [y - x for x, y in zip(a, b)]
n = d[5]
names = ['items', 'loads+B1', 'drain', 'B3', 'bottom']
tot = sum(d[:5])
print(sys.argv[2], 'wave-iterations', n, ' '.join(f'{k}={v / n:.0f}' for k, v in zip(names, d[:5])), 'total/iter', f'{tot / n:.0f}',
      'launch Gclk', ' '.join(f'{k}={v / 1e9:.2f}' for k, v in zip(names, d[:5])))
PY
done
