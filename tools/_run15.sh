set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in "dyn1:FEMASM_GATHER_SCHED=dynamic" "dyn2:FEMASM_GATHER_GRID_MULT=2" "static:FEMASM_GATHER_SCHED=static"; do
  name=${v%%:*}; envs=${v#*:}
  for c in E C B; do
  env $envs timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/x.json 2> gpurun_out/x.err || { tail -5 gpurun_out/x.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/x.json'));print('$name $c', d['value'], d['roofline']['launch_ms'])"
  done
done
