"""Is the N = 8 exchange overlap affordable?

On ONE GPU, for the config-E slab of rank `--rank` of `--world` (side 203, 25-26 of the 203 cube
layers): time the interior-row gather of SlabProblem (fa_gather_rows over the rows between the two
interface planes) alone, then again while a device-to-device copy of the HBM footprint of one
boundary's transfer (the interface suffix the rank sends, ~0.28 GB) runs on a second stream, and the
same slab's ghost-mode assembly (its layers + the layer above, no exchange). HIP events on the
stream each kernel runs on. Writes one JSON line.

Round 5: also the same transfer PACED to one xGMI link direction (--link-GBps, --pieces copies separated
by spin kernels), whose duration matches the real exchange's, beside the interior rows.

usage: python tools/overlap_probe.py [--n 203] [--rank 3] [--world 8] [--reps 10] [--link-GBps 70]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))

import torch  # noqa: E402

from femasm.parallel import SlabProblem  # noqa: E402


def timed(fn, reps, stream):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=203)
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--form", default="linear")
    ap.add_argument("--link-GBps", dest="link_GBps", type=float, default=70.0,
                    help="paced transfer rate: one xGMI link direction (~153 GB/s per link both ways; ~64-76 GB/s one way)")
    ap.add_argument("--pieces", type=int, default=64)
    ap.add_argument("--cu-masks", default="",
                    help="round 6: comma list of CU masks for the interior rows / the transfer, e.g. c1,s1,s2,s4 "
                         "(c: bits 0..8k-1 left out, s: k bits of every 32-bit mask word)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {"n": args.n, "rank": args.rank, "world": args.world, "form": args.form}
    prob = SlabProblem(args.n, args.rank, args.world, dev, groups=[None] * (args.world - 1), form=args.form)
    sg = prob.split
    out["cells"] = prob.num_cells
    out["exchange_bytes_sent"] = prob.exchange_bytes
    out["exchange_bytes_recv"] = prob.exchange_recv_bytes
    cur = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    nbytes = max(prob.exchange_bytes, prob.exchange_recv_bytes)
    src = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    sg.prepare()
    for i in range(sg_n := len(sg.plans)):
        sg.rows(i)
    torch.cuda.synchronize()
    inner = prob.n_iface  # the interior range follows the interface planes

    # the copy alone (its own duration on the side stream)
    def copy():
        with torch.cuda.stream(side):
            dst.copy_(src)
    copy_ms, _ = timed(copy, args.reps, side)
    out["copy_alone_ms"] = copy_ms
    out["copy_GBps"] = 2 * nbytes / copy_ms / 1e6

    # full single-rank assembly (records + every range), interior alone, interior + concurrent copy
    def full():
        sg.prepare()
        for i in range(sg_n):
            sg.rows(i)
    out["slab_assembly_ms"], _ = timed(full, args.reps, cur)
    out["interior_alone_ms"], out["interior_alone_min_ms"] = timed(lambda: sg.rows(inner), args.reps, cur)

    def interior_with_copy():
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            dst.copy_(src)
        sg.rows(inner)
        cur.wait_stream(side)
    out["interior_with_copy_ms"], out["interior_with_copy_min_ms"] = timed(interior_with_copy, args.reps, cur)
    out["overlap_cost_ms"] = out["interior_with_copy_ms"] - out["interior_alone_ms"]

    # round 5: the transfer paced to an xGMI link's rate -- the same bytes in
    # `--pieces` device copies on the side stream, separated by spin kernels (torch.cuda._sleep) so
    # that the whole transfer lasts as long as `--link-GBps` would take, overlapping the interior rows
    cyc = 1 << 20
    sleep_ms, _ = timed(lambda: torch.cuda._sleep(cyc), 5, cur)
    cyc_per_ms = cyc / max(sleep_ms, 1e-6)
    target_ms = nbytes / (args.link_GBps * 1e6)
    piece = (src.numel() + args.pieces - 1) // args.pieces
    gap = max(int(cyc_per_ms * target_ms / args.pieces), 1)

    def paced():
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for k in range(args.pieces):
                dst[k * piece:(k + 1) * piece].copy_(src[k * piece:(k + 1) * piece])
                torch.cuda._sleep(gap)
    out["paced_target_ms"] = target_ms
    out["paced_alone_ms"], _ = timed(lambda: (paced(), cur.wait_stream(side)), args.reps, cur)

    def interior_with_paced():
        paced()
        sg.rows(inner)
        cur.wait_stream(side)
    out["interior_with_paced_ms"], out["interior_with_paced_min_ms"] = timed(interior_with_paced, args.reps, cur)

    def interior_then_wait_paced():  # the interior's own time while the paced transfer runs beside it
        paced()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        sg.rows(inner)
        e1.record(cur)
        cur.wait_stream(side)
        return e0, e1
    ts = []
    for _ in range(args.reps):
        e0, e1 = interior_then_wait_paced()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    out["interior_beside_paced_ms"] = statistics.median(ts)
    out["paced_pieces"], out["link_GBps"] = args.pieces, args.link_GBps

    # Round 6: the transfer given CUs of its own. The interior rows run on a stream
    # whose CU mask leaves k CUs per XCD out; the paced transfer runs on a stream masked to exactly those
    # CUs (hipExtStreamCreateWithCUMask). The mask's bit layout (which bit is which XCD's CU) is found by
    # timing: leaving out bits 0..7 vs one bit in every 32 -- the per-XCD work of the gather is fixed, so
    # an uneven mask shows as a ~1/3 slower XCD.
    if args.cu_masks:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
        hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        words = (ncu + 31) // 32

        def masked_stream(bits):
            arr = (ctypes.c_uint32 * words)()
            for b in bits:
                arr[b // 32] |= 1 << (b % 32)
            h = ctypes.c_void_p()
            rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), words, arr)
            if rc != 0:
                raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
            return torch.cuda.ExternalStream(h.value, device=dev)

        allb = set(range(ncu))
        res = {}
        for spec in args.cu_masks.split(","):
            layout, k = spec[0], int(spec[1:])  # 'c': bits 0..8k-1 left out; 's': k bits per 32-bit word
            out_bits = set(range(8 * k)) if layout == "c" else {w * 32 + j for w in range(words) for j in range(k)}
            out_bits &= allb
            s_int = masked_stream(sorted(allb - out_bits))
            s_xfer = masked_stream(sorted(out_bits))
            r = {"cus_left_out": len(out_bits)}

            def interior_masked():
                s_int.wait_stream(cur)
                with torch.cuda.stream(s_int):
                    sg.rows(inner)
                cur.wait_stream(s_int)
            r["interior_alone_ms"], _ = timed(interior_masked, args.reps, cur)

            def paced_on(stream):
                stream.wait_stream(cur)
                with torch.cuda.stream(stream):
                    for k2 in range(args.pieces):
                        dst[k2 * piece:(k2 + 1) * piece].copy_(src[k2 * piece:(k2 + 1) * piece])
                        torch.cuda._sleep(gap)

            def interior_with_paced_masked():
                paced_on(s_xfer)
                interior_masked()
                cur.wait_stream(s_xfer)
            r["interior_with_paced_ms"], r["interior_with_paced_min_ms"] = timed(interior_with_paced_masked, args.reps, cur)
            res[spec] = r
            print(json.dumps({spec: r}), file=sys.stderr, flush=True)
        out["cu_mask"] = res
    del prob, sg
    torch.cuda.empty_cache()
    ghost = SlabProblem(args.n, args.rank, args.world, dev, groups=[None] * (args.world - 1), form=args.form,
                        mode="ghost")
    ghost.assemble()
    torch.cuda.synchronize()
    out["ghost_cells"] = ghost.num_cells_assembled
    out["ghost_assembly_ms"], _ = timed(ghost.assemble, args.reps, cur)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
