"""LDS pass count of k_gather_lin's positional plan (P2 tetrahedra): for every chunk, 16-lane quarter
and column step, the largest number of the quarter's lanes whose block slot has the same residue mod
16 (the 64-bit LDS op serves each quarter on its own; lanes on one residue serialize). Compares the
plan's total with the per-quarter bound max(steps, max residue count) and with the unordered map.
usage: python tools/r4/plan_stats.py [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
import torch  # noqa: E402

from femasm import fem, mesh  # noqa: E402


def stats(n, order):
    dev = torch.device("cuda", 0)
    m = mesh.create_unit_cube(n, n, n, mesh.CellType.tetrahedron, device=dev)
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    a = fem.LinearElasticity(V, E=1.0, nu=0.3)
    A = fem.create_matrix(a)
    fem.gather_plan(V, A, 0, order=order)
    key = [k for k in V._plans][0]
    plan, rs, _, smap, eadj, _ = V._plans[key]
    ptr, _ = V.adjacency()
    NN, NSPLIT, NBG = 10, 2, 5
    words = smap.view(torch.int16).to(torch.int32) & 0xFFFF
    rsc = rs.cpu()
    ptrc = ptr.cpu()
    tot, lb, lanes_tot = 0, 0, 0
    global hist
    hist = {}
    nch = int(plan.nchunks)
    rsc = rsc[:nch + 1]
    a0s = ptrc[rsc[:-1]]
    nas = ptrc[rsc[1:]] - a0s
    w = words.view(-1, NN).cpu()
    for c in range(nch):
        a0, na = int(a0s[c]), int(nas[c])
        if na <= 0:
            continue
        e = w[a0:a0 + na]                                 # [na, NN] slot words by position
        items = e.view(na, NSPLIT, NBG).reshape(na * NSPLIT, NBG)
        res = (items & 1023) & 15                          # [lanes, steps]
        L = res.shape[0]
        pad = (-L) % 16
        if pad:
            res = torch.cat([res, torch.full((pad, NBG), -1, dtype=res.dtype)])
        q = res.view(-1, 16, NBG)                          # [quarters, 16, steps]
        oh = torch.zeros(q.shape[0], NBG, 17, dtype=torch.int32)
        idx = (q.permute(0, 2, 1) + 1).long()              # -1 -> 0 (padding)
        oh.scatter_add_(2, idx, torch.ones_like(idx, dtype=torch.int32))
        per_step = oh[:, :, 1:].amax(dim=2)                # [quarters, steps]
        tot += int(per_step.sum())
        cr = oh[:, :, 1:].sum(dim=1)                       # [quarters, 16] residue totals
        lb += int(torch.maximum(cr.amax(dim=1), torch.full((q.shape[0],), NBG)).sum())
        lanes_tot += L
        full = (q >= 0).all(dim=2).all(dim=1)  # quarters of 16 real lanes
        mc = cr.amax(dim=1)
        for k in range(q.shape[0]):
            if bool(full[k]):
                hist.setdefault(int(mc[k]), [0, 0])
                hist[int(mc[k])][0] += 1
                hist[int(mc[k])][1] += int(per_step[k].sum())
    return tot, lb, lanes_tot


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    for order in ("positional",):
        try:
            t, b, L = stats(n, order)
            print(f"n={n} order={order}: passes {t}  bound {b}  ratio {t / b:.3f}  lanes {L}")
            for mcv in sorted(hist):
                cnt, ps = hist[mcv]
                print(f"  full quarters with max residue count {mcv}: {cnt}  mean passes {ps / cnt:.2f}")
        except Exception as ex:  # noqa: BLE001
            print(f"order={order}: {ex}")
