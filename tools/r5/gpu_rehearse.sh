#!/bin/bash
# Round 5: bench.py's N > 1 path on ONE GPU (ranks share cuda:0, gloo): the default ghost slabs at
# N = 2 and 4, and the RCCL-path exchange mode at N = 2 (side 60; the 8-GPU RCCL run is the driver's)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for run in "2 ghost" "4 ghost" "2 exchange"; do
  set -- $run; N=$1; mode=$2
  FEMASM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 3 --warmup 1 --side ${NMESH:-60} \
    --slab-mode $mode > gpurun_out/rehearse_${N}_$mode.json 2> gpurun_out/rehearse_${N}_$mode.err || { tail -20 gpurun_out/rehearse_${N}_$mode.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/rehearse_${N}_$mode.json'));print($N, '$mode', d['value'], d['ms_per_step'], d['config'].get('parallelism'), d['config'].get('slab_mode'))"
done
