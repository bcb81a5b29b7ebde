#!/bin/bash
# neo records with u loaded once, 32 KB linear accumulator, 512-thread P1-tet gather: whole GPU suite,
# kernel stats of Eneo / E / C, C with 256 threads, PMC of the neo gather
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/l_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/l_pytest.log; [ $rc -eq 0 ] || exit $rc
CFGS="Eneo E C" STEPS=4 bash tools/prof_all.sh || exit 1
FEMASM_LIB=$PWD/abl/libfemasm_p1nt256.so timeout -k 10 300 python bench.py --config C --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-probe > gpurun_out/l_C256.json 2> gpurun_out/l_C256.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/l_C256.json'));print('C nt256', d['value'], d['roofline']['launch_ms'])"
bash tools/pmc_lin.sh Eneo
