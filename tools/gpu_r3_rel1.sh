#!/bin/bash
# Release run 1/2 of the round-3 build: counter list, PMC traffic / flop records of E, E-neo, C
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_avail.txt 2>&1 || true
grep -ci mfma gpurun_out/rocprof_avail.txt || true
CFGS="E:203 Eneo:203 C:119" bash tools/gpu_traffic.sh > gpurun_out/traffic_rel1.txt 2>&1 || { tail -5 gpurun_out/traffic_rel1.txt; exit 1; }
tail -30 gpurun_out/traffic_rel1.txt
cp gpurun_out/traffic.json profiles/traffic.json
