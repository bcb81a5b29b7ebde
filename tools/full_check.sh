#!/bin/bash
# Round-end style check: the whole GPU suite, smoke(), and the default bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/full_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/full_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { tail -5 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/full_bench.json 2> gpurun_out/full_bench.err || { tail -5 gpurun_out/full_bench.err; exit 1; }
cat gpurun_out/full_bench.json
