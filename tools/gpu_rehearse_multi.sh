#!/bin/bash
# Rehearse bench.py's N > 1 path on ONE GPU: ranks share cuda:0 and exchange with gloo
# (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's). Checks the slab setup,
# split gather, async exchange, max-over-ranks timing and the JSON line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for N in 2 4; do
  FEMASM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 3 --warmup 1 --side ${NMESH:-60} \
    > gpurun_out/rehearse_$N.json 2> gpurun_out/rehearse_$N.err || { tail -20 gpurun_out/rehearse_$N.err; exit 1; }
  cat gpurun_out/rehearse_$N.json
done
