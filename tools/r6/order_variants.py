"""Config E linear: the gather's chunk visiting order vs launch time (round 6). XCD x walks positions
[x per, (x + 1) per) of the visiting sequence (plan.corder). Variants: the default Morton order, row
order (corder NULL: contiguous row ranges per XCD), and row order dealt to the XCDs in blocks of G
chunks (every XCD writes near the others: one compact write frontier). One JSON line per variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from femasm import fem  # noqa: E402


def timed(fn, reps, warm=2):
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
    variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["morton", "row", "deal16", "deal1", "morton"]
    cfg = bench.CONFIGS[sys.argv[3] if len(sys.argv) > 3 else "E"]
    dev = torch.device("cuda", 0)
    m, V, a, bcs = bench.build_problem(n, dev, cfg=cfg)
    A = fem.create_matrix(a)
    # the plan assemble_matrix uses (default locality) has its visiting sequence swapped per variant;
    # the Morton sequence comes from the Morton plan (cached on V, so its memory stays alive)
    plan = fem.gather_plan(V, A, 0, a.kind)
    default = plan.corder
    morton = fem.gather_plan(V, A, 0, a.kind, locality="morton").corder
    nch = int(plan.nchunks)
    ref = None
    keep = []
    for var in variants:
        if var == "morton":
            plan.corder = morton
        elif var == "row":
            plan.corder = None
        elif var.startswith("deal"):
            g = int(var[4:])
            c = torch.arange(nch, device=dev, dtype=torch.int64)
            key = ((c // g) % 8) * nch + c
            seq = torch.argsort(key).to(torch.int32).contiguous()
            keep.append(seq)
            plan.corder = seq.data_ptr()
        else:
            raise SystemExit(f"unknown variant {var}")
        plan.chunk_desc = None  # the cached chunk arrays follow the old order: built per launch instead
        med, best = timed(lambda: fem.assemble_matrix(a, bcs=bcs, A=A), 10)
        flat = A.data.view(-1)
        if ref is None:
            idx = torch.randint(0, flat.numel(), (1 << 22,), device=dev, generator=torch.Generator(dev).manual_seed(1))
            ref = flat[idx].clone()
            diff = 0.0
        else:
            diff = float((flat[idx] - ref).abs().max() / ref.abs().max())
        print(json.dumps({"variant": var, "launch_ms_median": round(med, 3), "launch_ms_min": round(best, 3),
                          "nchunks": nch, "max_rel_diff_vs_first": diff}), flush=True)
    plan.corder = default
    plan.chunk_desc = None


if __name__ == "__main__":
    main()
