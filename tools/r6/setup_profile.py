"""Config E setup, phase by phase (torch.cuda.synchronize around each): mesh, function space + dofmap,
bcs, adjacency, sparsity, plan chunks, slots, order, locality. Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from femasm import _lib, fem, mesh  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 203
    dev = torch.device("cuda", 0)
    torch.ones(1, device=dev)
    _lib.load()
    _wm, _wV, _wa, _wb = bench.build_problem(4, dev)  # the library's first launches (code object loading)
    fem.assemble_matrix(_wa, bcs=_wb)
    torch.cuda.synchronize()
    del _wm, _wV, _wa, _wb
    out = {}
    t = time.time()

    def mark(k):
        nonlocal t
        torch.cuda.synchronize()
        now = time.time()
        out[k] = round(now - t, 4)
        t = now
    m = mesh.create_box((1.0, 1.0, 1.0), (n, n, n), mesh.CellType.tetrahedron, device=dev)
    mark("mesh")
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    mark("space")
    _, V, a, bcs = bench.build_problem(n, dev)  # (rebuilds: the remaining pieces, E and bcs)
    torch.cuda.synchronize()
    t = time.time()
    marker, _ = fem._combine_bcs(V, bcs)
    mark("bcs_marker")
    V.adjacency()
    mark("adjacency")
    fm0, adj0 = V._fa_mesh(), V._fa_adjacency()
    indptr = torch.empty(V.num_nodes + 1, dtype=torch.int64, device=dev)
    nb = ctypes.c_int64(0)
    Lb = _lib.load()
    sh0 = _lib.stream_handle(dev)
    _lib.check(Lb.fa_sparsity_count(ctypes.byref(fm0), ctypes.byref(adj0), indptr.data_ptr(), ctypes.byref(nb), sh0), "count")
    mark("sparsity_count")
    indices = torch.empty(nb.value, dtype=torch.int32, device=dev)
    _lib.check(Lb.fa_sparsity_fill(ctypes.byref(fm0), ctypes.byref(adj0), indptr.data_ptr(), indices.data_ptr(), sh0), "fill")
    mark("sparsity_fill")
    V._pattern = (indptr, indices)
    A = fem.create_matrix(a)
    mark("matrix_alloc")
    L = _lib.load()
    fm, adj, fb = V._fa_mesh(), V._fa_adjacency(), fem._fa_bsr(A, 0)
    rs = torch.empty(A.parts[0][1] - A.parts[0][0] + 1, dtype=torch.int64, device=dev)
    plan = _lib.fa_plan()
    sh = _lib.stream_handle(dev)
    _lib.check(L.fa_plan_gather_form(ctypes.byref(fm), int(a.kind), ctypes.byref(adj), ctypes.byref(fb), rs.data_ptr(),
                                     ctypes.byref(plan), sh), "plan")
    mark("plan_chunks")
    smap = torch.empty(V.mesh.num_cells * V.nn * V.nn, dtype=torch.int16, device=dev)
    _lib.check(L.fa_plan_slots(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb), smap.data_ptr(),
                               ctypes.byref(plan), sh), "slots")
    mark("plan_slots")
    eadj = fem._plan_order(V, fm, adj, fb, plan, sh)
    mark("plan_order")
    corder = fem._plan_locality(V, fm, adj, plan, sh)
    mark("plan_locality")
    out["nchunks"] = int(plan.nchunks)
    out["total"] = round(sum(v for k, v in out.items() if k not in ("nchunks",)), 3)
    del eadj, corder
    print(json.dumps(out))


if __name__ == "__main__":
    main()
