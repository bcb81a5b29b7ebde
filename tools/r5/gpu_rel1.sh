#!/bin/bash
# Release run 1/2 of the round-5 build: PMC records (traffic, FP64, MFMA busy) of E, C, E-neo, D, Dmfma
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS="${CFGS:-E:203 C:119 Eneo:203 D:58 Dmfma:58}" bash tools/gpu_traffic.sh > gpurun_out/traffic_rel1.txt 2>&1 || { tail -5 gpurun_out/traffic_rel1.txt; exit 1; }
tail -5 gpurun_out/traffic_rel1.txt
