#!/bin/bash
# round 6 batch 3: deterministic with prefetched exponents; chunk visiting order variants (E linear)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
#timeout -k 10 300 python -u -m pytest tests/test_gpu_deterministic.py -x -q --timeout 240 --timeout-method thread > gpurun_out/b3_det.log 2>&1
#rc=$?; tail -2 gpurun_out/b3_det.log; [ $rc -eq 0 ] || exit $rc
#timeout -k 10 400 python bench.py --steps 5 --warmup 1 --deterministic --no-eneo --no-cpu-baseline --no-hbm-probe > gpurun_out/b3_det_E.json 2> gpurun_out/b3_det_E.err || { tail -5 gpurun_out/b3_det_E.err; exit 1; }
#python -c "import json;d=json.load(open('gpurun_out/b3_det_E.json'));print('det E', d['ms_per_step'], d['roofline']['launch_ms'], d['setup_s'], d['setup'])"
timeout -k 10 500 python tools/r6/order_variants.py 203 morton,row,deal16,deal1,deal64,morton > gpurun_out/b3_order.txt 2> gpurun_out/b3_order.err || { tail -5 gpurun_out/b3_order.err; exit 1; }
cat gpurun_out/b3_order.txt
timeout -k 10 400 python tools/overlap_probe.py --link-GBps 70 --cu-masks c1,s1,s2,s4 > gpurun_out/b3_overlap_E.json 2> gpurun_out/b3_overlap_E.err || { tail -5 gpurun_out/b3_overlap_E.err; exit 1; }
grep '^{"c1\|^{"s' gpurun_out/b3_overlap_E.err; python -c "import json;d=json.load(open('gpurun_out/b3_overlap_E.json'));print({k:d[k] for k in ('slab_assembly_ms','interior_alone_ms','interior_with_paced_ms','ghost_assembly_ms')})"
