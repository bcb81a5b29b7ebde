"""Affine Q1 hexahedra (n^3 unit cube, linear elasticity, E per cell, nu 0.3, x = 0 / x = 1 bcs): launch
time of one assembly, median of 10 (round 6: k_gather_lin vs the tensor-factor gather; run once per
library with FEMASM_LIB). usage: python tools/r6/hex1_ab.py [n]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
import torch  # noqa: E402

from femasm import fem, mesh  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    dev = torch.device("cuda", 0)
    m = mesh.create_unit_cube(n, n, n, cell_type=mesh.CellType.hexahedron, device=dev)
    V = fem.functionspace(m, ("Lagrange", 1, (3,)))
    E = 1e6 * (1.0 + (torch.arange(m.num_cells, device=dev) % 200).to(torch.float64))
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0.0, 0.0], right, V)]
    A = fem.create_matrix(a)
    for _ in range(3):
        fem.assemble_matrix(a, bcs=bcs, A=A)
    st = torch.cuda.current_stream()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fem.assemble_matrix(a, bcs=bcs, A=A)
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    s = float(A.data.double().abs().sum())
    print(json.dumps({"lib": os.environ.get("FEMASM_LIB", "product"), "n": n, "cells": m.num_cells,
                      "ms_median": round(ts[5], 4), "ms_min": round(ts[0], 4), "abs_sum": s}), flush=True)


if __name__ == "__main__":
    main()
