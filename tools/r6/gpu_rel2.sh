#!/bin/bash
# Release run 2/2 of the round-6 build: rocprofv3 kernel stats of every config, then the whole GPU suite,
# smoke() and the default bench line (tools/full_check.sh), then bench.py's N>1 path rehearsed with gloo
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS="E Eneo D Dq2 B C A Dmfma" bash tools/prof_all.sh > gpurun_out/prof_all_rel.txt 2>&1 || { tail -5 gpurun_out/prof_all_rel.txt; exit 1; }
grep -E "^(E|Eneo|D|Dq2|B|C|A|Dmfma) " gpurun_out/prof_all_rel.txt
bash tools/full_check.sh > gpurun_out/fc.txt 2>&1
rc=$?; tail -4 gpurun_out/fc.txt | cut -c1-400; [ $rc -eq 0 ] || exit $rc
FEMASM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 3 --warmup 1 --side 60 \
    > gpurun_out/rel_rehearse_2.json 2> gpurun_out/rel_rehearse_2.err || { tail -20 gpurun_out/rel_rehearse_2.err; exit 1; }
tail -1 gpurun_out/rel_rehearse_2.json | cut -c1-300
