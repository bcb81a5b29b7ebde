"""Summarise rocprofv3 --pmc CSV passes (tools/prof_passes.sh) per kernel: mean per dispatch.
FETCH_SIZE / WRITE_SIZE are in KiB (tools/probe/fetch_calib.hip: a 4 GiB read gives FETCH_SIZE =
2 GiB / 1024 for 16-B, 80-B, u16 and u32 lane loads alike, a 4 GiB 16-B store stream WRITE_SIZE =
1.003 x 4 GiB / 1024); gfx950 FETCH_SIZE counts half of the bytes read (MI355X_MICROARCH.md §HBM):
both the raw and the x2-corrected values are printed."""
KIB = 1024.0
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
            extra = f"  (x2 corrected: {2 * mean * KIB / 1e9:.3f} GB)"
        if c == "WRITE_SIZE":
            extra = f"  ({mean * KIB / 1e9:.3f} GB)"
        print(f"  {c:24s} {mean:16.1f}{extra}  [{len(per)} dispatches]")


LAUNCH_KERNELS = ("k_gather", "k_cell_records", "k_rec_bcbits", "k_neo_records", "k_hex_mfma", "k_bc_diag")  # one assembly launch


def counter_total(name, kernels=LAUNCH_KERNELS):
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


def traffic_record(root, kernels=LAUNCH_KERNELS):
    """HBM bytes per assembly launch: sum over the launch's kernels of FETCH_SIZE x 2 + WRITE_SIZE (KiB)."""
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
            tot += (2.0 if c == "FETCH_SIZE" else 1.0) * mean * KIB
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
    mb = counter_total("SQ_VALU_MFMA_BUSY_CYCLES", ("k_hex_mfma",))
    ga = counter_total("GRBM_GUI_ACTIVE", ("k_hex_mfma",))
    if mb is not None and ga:
        # MFMA-busy cycles summed over the SIMDs / (the kernel's cycles per XCD x 1024 SIMDs)
        data[key]["mfma_busy"] = {"busy_cycles": mb, "gui_active": ga, "frac": mb / (ga / 8.0 * 1024.0),
                                  "kernel": "k_hex_mfma",
                                  "what": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)"}
        mops = counter_total("SQ_INSTS_VALU_MFMA_MOPS_F64", ("k_hex_mfma",))
        if mops is not None:
            data[key]["mfma_busy"]["mfma_fp64_flops"] = 512.0 * mops  # rocprofv3's MfmaFlopsF64
    json.dump(data, open(out, "w"), indent=1)
