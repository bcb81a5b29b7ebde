"""Summarise rocprofv3 --pmc CSV passes (tools/prof_passes.sh) per kernel: mean per dispatch.
FETCH_SIZE / WRITE_SIZE are in KB; gfx950 FETCH_SIZE counts half of wide streaming reads
(MI355X_MICROARCH.md §HBM) -- both the raw and the x2-corrected values are printed."""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pass*", "*counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", row.get("Kernel-Name", "?"))[:60]
        acc[k][row["Counter_Name"]].append((row.get("Dispatch_Id"), float(row["Counter_Value"])))
for k, d in acc.items():
    print(k)
    for c, vals in sorted(d.items()):
        per = defaultdict(float)
        for did, v in vals:
            per[did] += v
        mean = sum(per.values()) / len(per)
        extra = ""
        if c == "FETCH_SIZE":
            extra = f"  (x2 corrected: {2 * mean / 1e6:.3f} GB)"
        if c == "WRITE_SIZE":
            extra = f"  ({mean / 1e6:.3f} GB)"
        print(f"  {c:24s} {mean:16.1f}{extra}  [{len(per)} dispatches]")


def counter_total(name, kernels=("k_gather", "k_cell_records")):
    """Sum over the launch's kernels of the per-dispatch mean of one counter, or None if not collected."""
    tot, seen = 0.0, False
    for k, d in acc.items():
        if not any(s in k for s in kernels) or name not in d:
            continue
        per = defaultdict(float)
        for did, v in d[name]:
            per[did] += v
        tot += sum(per.values()) / len(per)
        seen = True
    return tot if seen else None


def traffic_record(root, kernels=("k_gather", "k_cell_records")):
    """HBM bytes per assembly launch: sum over the launch's kernels of FETCH_SIZE x 2 + WRITE_SIZE (KB)."""
    tot = 0.0
    for k, d in acc.items():
        if not any(s in k for s in kernels):
            continue
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            if c not in d:
                continue
            per = defaultdict(float)
            for did, v in d[c]:
                per[did] += v
            mean = sum(per.values()) / len(per)
            tot += (2.0 if c == "FETCH_SIZE" else 1.0) * mean * 1e3
    return tot


if len(sys.argv) > 3:  # pmc_summary.py ROOT KEY OUT_JSON: record traffic for bench.py
    import json

    import hashlib

    key, out = sys.argv[2], sys.argv[3]
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fem-libraries_amd", "csrc", "femasm.hip")
    khash = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
    data = json.load(open(out)) if os.path.exists(out) else {}
    # keyed on the kernel source hash: bench.py refuses a record of another build of femasm.hip
    data[key] = {"bytes": traffic_record(root), "kernel_hash": khash,
                 "source": f"rocprofv3 --pmc passes in {root} (tools/prof_passes.sh)"}
    fl = counter_total("SQ_INSTS_VALU_FLOPS_FP64")
    if fl is not None:
        # SQ_INSTS_VALU_FLOPS_FP64 = 2 FMA + MUL + ADD per wave instruction (measured: it equals that
        # sum of the SQ_INSTS_VALU_*_F64 counters); x 64 lanes = the FP64 work issued to the VALU
        data[key]["fp64_flops"] = 64.0 * fl
        data[key]["fp64_flops_what"] = "64 x SQ_INSTS_VALU_FLOPS_FP64 (lane slots of the issued FP64 VALU instructions)"
    json.dump(data, open(out, "w"), indent=1)
