#!/bin/bash
# Neo-Hookean GPU tests, then config E-neo under rocprofv3 kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider -k "neo or Neo" --timeout 300 \
  --timeout-method thread > gpurun_out/neo_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/neo_pytest.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/neoprof2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/neoprof2 -o run --output-format csv -- \
  python bench.py --config Eneo --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/neo.json 2> gpurun_out/neo.err \
  || { tail -5 gpurun_out/neo.err; exit 1; }
python3 - <<'PY'
import csv, glob, json
d = [json.loads(l) for l in open("gpurun_out/neo.json") if l.startswith("{")][-1]
print("Eneo", d["value"], d["ms_per_step"], d["roofline"]["launch_ms"])
for f in glob.glob("gpurun_out/neoprof2/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gather" in r["Name"] or "records" in r["Name"]:
            print(r["Name"][:40], float(r["AverageNs"]) / 1e6)
PY
