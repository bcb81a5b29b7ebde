#!/bin/bash
# per-phase clocks of k_gather_lin (abl/libfemasm_lin_timing.so) on configs E and C, default and deterministic
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-E C}; do
for d in ${DETS:-"" "--deterministic"}; do
  FEMASM_LIB=$PWD/abl/libfemasm_lin_timing.so timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe $d > gpurun_out/t_$c$d.out 2> gpurun_out/t_$c$d.err || { echo "$c $d failed"; tail -5 gpurun_out/t_$c$d.err; exit 1; }
  python - gpurun_out/t_$c$d.out "$c $d" <<'PY'
import sys, json
L = [l.split()[1:] for l in open(sys.argv[1]) if l.startswith('lin_timing')]
a, b = [list(map(int, x)) for x in L[-2:]]
d = [y - x for x, y in zip(a, b)]
n = d[7]
names = ['items', 'B1', 'xchg', 'stores', 'post', 'B3', 'bottom']
tot = sum(d[:7])
print(sys.argv[2], 'wave-iterations', n, 'clocks/iter', ' '.join(f'{k}={v / n:.0f}' for k, v in zip(names, d)), 'total', f'{tot / n:.0f}', 'MHz', f'{100.0 * tot / max(d[8], 1):.0f}')
js = [l for l in open(sys.argv[1]) if l.startswith('{')]
print(json.loads(js[-1])['roofline']['launch_ms'])
PY
done; done
