"""Diagnostic: default (FP64) vs deterministic assembly on the P2-tet case that failed; prints the
worst rows and entries. usage: FEMASM_LIB=... python tools/r4/diag_default.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
import numpy as np, torch
from femasm import fem, mesh
from femasm.materials import e_range
dev = torch.device("cuda", 0)
for n in [(12, 11, 10), (6, 5, 4)]:
    m = mesh.create_unit_cube(*n, cell_type=-4, device=dev)
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    E = torch.tensor(e_range()[np.arange(m.num_cells) % 200], dtype=torch.float64, device=dev)
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    for bcs in ([], [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0, 0], right, V)]):
        Ad = fem.assemble_matrix(a, bcs=bcs, deterministic=True).data.clone()
        outs = []
        for r in range(3):
            A0 = fem.assemble_matrix(a, bcs=bcs)
            outs.append(A0.data.clone())
        ip = A0.indptr.cpu().numpy()
        for r, d in enumerate(outs):
            diff = (d - Ad).abs().reshape(-1)
            k = int(diff.argmax())
            blk = k // 9
            row = int(np.searchsorted(ip, blk, side="right") - 1)
            print(n, "bcs" if bcs else "nobc", "run", r, "maxdiff", float(diff.max()), "at value", k, "block", blk,
                  "row", row, "got", float(d.reshape(-1)[k]), "det", float(Ad.reshape(-1)[k]),
                  "nbad(>1e-9 rel)", int((diff > 1e-9 * Ad.abs().max()).sum()), "chunk-rows?", A0.num_block_rows)
        print("run-to-run default maxdiff", float((outs[0] - outs[1]).abs().max()), float((outs[0] - outs[2]).abs().max()))
