"""Config E linear, plan variants in one process (alternating, launch ms by HIP events): the slot map's
format (FA_PLAN_COMPACT 64-bit words per item vs 16-bit words) x the chunk visiting order (row vs
Morton). One JSON line per measurement; a sampled value check against the first variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from femasm import _lib, fem  # noqa: E402


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
    cfg = bench.CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "E"]
    dev = torch.device("cuda", 0)
    m, V, a, bcs = bench.build_problem(n, dev, cfg=cfg)
    A = fem.create_matrix(a)
    variants = {"compact_row": dict(order="positional", locality=False), "wide_row": dict(order="wide", locality=False),
                "compact_morton": dict(order="positional", locality=True), "wide_morton": dict(order="wide", locality=True)}
    for k, opt in variants.items():
        p = fem.gather_plan(V, A, 0, a.kind, **opt)
        print(json.dumps({"variant": k, "compact": bool(p.cell_flags & _lib.FA_PLAN_COMPACT), "nchunks": int(p.nchunks)}),
              flush=True)
    idx = ref = None
    for rnd in range(2):
        for k, opt in variants.items():
            med, best = timed(lambda: fem.assemble_matrix(a, bcs=bcs, A=A, plan=opt))
            flat = A.data.view(-1)
            if idx is None:
                idx = torch.randint(0, flat.numel(), (1 << 22,), device=dev, generator=torch.Generator(dev).manual_seed(1))
                ref = flat[idx].clone()
            diff = float((flat[idx] - ref).abs().max() / ref.abs().max())
            print(json.dumps({"variant": k, "launch_ms_median": round(med, 3), "launch_ms_min": round(best, 3),
                              "max_rel_diff_sampled": diff}), flush=True)


if __name__ == "__main__":
    main()
