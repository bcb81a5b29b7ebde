#!/bin/bash
# round 6 batch 18: the chunk schedule probe (tools/probe/sched_probe.hip), shipped schedule vs tail stealing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 ./tools/probe/sched_probe 200 > gpurun_out/b18_sched.txt 2>&1; rc=$?; cat gpurun_out/b18_sched.txt; exit $rc
