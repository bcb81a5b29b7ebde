#!/bin/bash
# cleaned library: full GPU suite, config benches, k_gather_lin ablations (default and deterministic)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_pytest_c.log 2>&1 || { tail -60 gpurun_out/gpu_pytest_c.log; exit 1; }
tail -3 gpurun_out/gpu_pytest_c.log
b() {  # name lib config extra
  L=""; [ "$2" != base ] && L="FEMASM_LIB=$PWD/abl/libfemasm_$2.so"
  env $L timeout -k 10 300 python bench.py --config $3 --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-hbm-probe $4 > gpurun_out/c_$1.json 2> gpurun_out/c_$1.err || { echo "bench $1 failed"; tail -5 gpurun_out/c_$1.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c_$1.json'));print('$1', d['value'], d['roofline']['launch_ms'])"
}
b E base E "" && b Edet base E --deterministic && b C base C "" && b Eneo base Eneo "" && b D base D "" && b Dmfma base Dmfma "" || exit 1
for v in lin_noadd lin_nostore lin_nozero lin_notab; do
  b E_$v $v E "" && b Edet_$v $v E --deterministic || exit 1
done
b E2 base E "" && b Edet2 base E --deterministic
