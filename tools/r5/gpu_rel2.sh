#!/bin/bash
# Release run 2/2 of the round-5 build: kernel stats of every config, the whole GPU suite, smoke()
# and the default bench line (tools/full_check.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS="E Eneo D Dq2 B C A Dmfma" bash tools/prof_all.sh > gpurun_out/prof_all_rel.txt 2>&1 || { tail -5 gpurun_out/prof_all_rel.txt; exit 1; }
grep -E "^(E|Eneo|D|Dq2|B|C|A|Dmfma) " gpurun_out/prof_all_rel.txt
bash tools/full_check.sh > gpurun_out/fc.txt 2>&1
rc=$?; tail -4 gpurun_out/fc.txt | cut -c1-400; exit $rc
