#!/bin/bash
# GPU session: slab tests (matrix for both forms, sharded residual), config Eneo bench at N=1,
# a 2-rank gloo rehearsal of the Eneo slab bench on one GPU (reduced side), headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parallel.py -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_par.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_par.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config Eneo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_Eneo.json 2> gpurun_out/bench_Eneo.err || { tail -5 gpurun_out/bench_Eneo.err; exit 1; }
cat gpurun_out/bench_Eneo.json; tail -2 gpurun_out/bench_Eneo.err
FEMASM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config Eneo --side 96 --steps 3 --warmup 1 \
  > gpurun_out/rehearse_Eneo2.json 2> gpurun_out/rehearse_Eneo2.err || { tail -5 gpurun_out/rehearse_Eneo2.err; exit 1; }
cat gpurun_out/rehearse_Eneo2.json
