#!/bin/bash
# round 6 batch 1: deterministic per-block scales (tests + E timing), setup phases, N>1 rehearsal (both legs)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_deterministic.py -x -q --timeout 240 --timeout-method thread > gpurun_out/b1_det.log 2>&1
rc=$?; tail -3 gpurun_out/b1_det.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/r6/setup_profile.py > gpurun_out/b1_setup.json 2> gpurun_out/b1_setup.err || { tail -5 gpurun_out/b1_setup.err; exit 1; }
cat gpurun_out/b1_setup.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b1_prof_setup -o setup -- python tools/r6/setup_profile.py > gpurun_out/b1_setup_prof.log 2>&1 || { tail -5 gpurun_out/b1_setup_prof.log; exit 1; }
f=$(find gpurun_out/b1_prof_setup -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/b1_setup_kernel_stats.csv; head -12 gpurun_out/b1_setup_kernel_stats.csv | cut -c1-150
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --deterministic --no-eneo --no-cpu-baseline --no-hbm-probe > gpurun_out/b1_det_E.json 2> gpurun_out/b1_det_E.err || { tail -5 gpurun_out/b1_det_E.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b1_det_E.json'));print('det E', d['ms_per_step'], d['roofline']['launch_ms'])"
for N in 2; do
FEMASM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 3 --warmup 1 --side 60 \
    > gpurun_out/b1_rehearse_$N.json 2> gpurun_out/b1_rehearse_$N.err || { tail -20 gpurun_out/b1_rehearse_$N.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b1_rehearse_$N.json'));print($N, d['value'], d['ms_per_step'], d['config']['parallelism']); print(json.dumps(d['legs']))"
done
