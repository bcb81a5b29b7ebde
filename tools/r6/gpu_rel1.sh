#!/bin/bash
# Release run 1/2 of the round-6 build: PMC records (traffic, executed FP64, MFMA busy) of E, C, E-neo, D,
# Dmfma -> gpurun_out/traffic.json (keyed on the femasm.hip hash) and gpurun_out/pmc_<cfg>.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS="${CFGS:-E:203 C:119 Eneo:203 D:58 Dmfma:58 B:1000}" bash tools/gpu_traffic.sh > gpurun_out/traffic_rel1.txt 2>&1 || { tail -5 gpurun_out/traffic_rel1.txt; exit 1; }
tail -3 gpurun_out/traffic_rel1.txt | cut -c1-300
