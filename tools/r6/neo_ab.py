"""E-neo A/B in one process: the staged-record gather (fa_plan_cells lists) vs per-item record loads,
alternating, launch ms (HIP events). One JSON line per measurement."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from femasm import fem  # noqa: E402


def timed(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    st = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 203
    dev = torch.device("cuda", 0)
    m, V, a, bcs = bench.build_problem(n, dev, cfg=bench.CONFIGS["Eneo"])
    A = fem.create_matrix(a)
    p1 = fem.gather_plan(V, A, 0, a.kind)
    p0 = fem.gather_plan(V, A, 0, a.kind, stage=False)
    print(json.dumps({"staged_plan": bool(p1.ccell), "nchunks": int(p1.nchunks)}), flush=True)
    idx = None
    ref = None
    for rnd in range(2):
        for name, opt in (("staged", None), ("loaded", {"stage": False})):
            med, best = timed(lambda: fem.assemble_matrix(a, bcs=bcs, A=A, plan=opt))
            flat = A.data.view(-1)
            if idx is None:
                idx = torch.randint(0, flat.numel(), (1 << 22,), device=dev, generator=torch.Generator(dev).manual_seed(1))
                ref = flat[idx].clone()
            diff = float((flat[idx] - ref).abs().max() / ref.abs().max())
            print(json.dumps({"variant": name, "launch_ms_median": round(med, 3), "launch_ms_min": round(best, 3),
                              "max_rel_diff_sampled": diff}), flush=True)


if __name__ == "__main__":
    main()
