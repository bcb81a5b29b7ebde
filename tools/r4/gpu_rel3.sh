#!/bin/bash
# Short release run: kernel stats of E and C, the whole GPU suite, smoke() and the default bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS="E C" bash tools/prof_all.sh > gpurun_out/prof_all_rel.txt 2>&1 || { tail -5 gpurun_out/prof_all_rel.txt; exit 1; }
grep -E "^(E|C) " gpurun_out/prof_all_rel.txt
bash tools/full_check.sh > gpurun_out/fc.txt 2>&1
rc=$?; tail -4 gpurun_out/fc.txt | cut -c1-400; exit $rc
