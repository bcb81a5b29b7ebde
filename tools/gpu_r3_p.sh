#!/bin/bash
# default-bench slowdown: the same E bench with and without the CPU-baseline worker pool
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
b() { timeout -k 10 600 python bench.py "$@" > gpurun_out/p_$n.json 2> gpurun_out/p_$n.err || { tail -3 gpurun_out/p_$n.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/p_$n.json'));print('$n', d['ms_per_step'], d['roofline']['launch_ms'])"; }
n=nocpu b --no-cpu-baseline
n=default b
n=aff0 b --cpu-all-affinity 0
n=nocpu2 b --no-cpu-baseline
