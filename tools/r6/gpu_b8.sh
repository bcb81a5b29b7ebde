#!/bin/bash
# round 6 batch 8: device allocation timing of a 139 GB value array; N=2 gloo rehearsal of the bench's legs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/r6/alloc_probe.py > gpurun_out/b8_alloc.json 2> gpurun_out/b8_alloc.err || { tail -5 gpurun_out/b8_alloc.err; exit 1; }
cat gpurun_out/b8_alloc.json
FEMASM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 3 --warmup 1 --side 60 \
    > gpurun_out/b8_rehearse_2.json 2> gpurun_out/b8_rehearse_2.err || { tail -20 gpurun_out/b8_rehearse_2.err; exit 1; }
tail -1 gpurun_out/b8_rehearse_2.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['config']['parallelism']); print({k:(v.get('ms_per_step'), v.get('error')) for k,v in d['legs'].items()})"
