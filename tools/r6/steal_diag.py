"""Round 6 diagnosis: repeated assemblies of the row-parts case of tests/test_gpu_deterministic.py
(P2 tets 4x3x3, max_part_bytes 8192), the value array filled with NaN before each run: per run, the
entries never written (NaN) and the entries that differ from run 0, with their row parts.
usage: python tools/r6/steal_diag.py [runs] [det 0/1] [part_bytes]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from femasm import fem, mesh  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    det = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
    pb = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
    dev = torch.device("cuda", 0)
    m = mesh.create_unit_cube(4, 3, 3, cell_type=-4, device=dev)
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    E = torch.linspace(1.0, 2.0, m.num_cells, dtype=torch.float64, device=dev)
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V)]
    A = fem.create_matrix(a, max_part_bytes=pb)
    bounds = [p[0] for p in A.parts] + [A.parts[-1][1]]
    ip = A.indptr.cpu().numpy()
    ref = None
    bad = 0
    for r in range(runs):
        A.data.fill_(float("nan"))
        fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=det)
        torch.cuda.synchronize()
        d = A.data.reshape(A.data.shape[0], -1).cpu().numpy()
        nanb = np.nonzero(np.isnan(d).any(axis=1))[0]
        if ref is None:
            ref = d.copy()
            diffb = np.zeros(0, dtype=np.int64)
        else:
            diffb = np.nonzero((d != ref).any(axis=1) & ~np.isnan(d).any(axis=1))[0]
        if len(nanb) or len(diffb):
            bad += 1
            rows = np.searchsorted(ip, nanb, side="right") - 1
            parts = np.searchsorted(bounds, rows, side="right") - 1
            print(f"run {r}: {len(nanb)} unwritten blocks (rows {sorted(set(rows.tolist()))[:12]}, parts "
                  f"{sorted(set(parts.tolist()))}), {len(diffb)} blocks differ from run 0", flush=True)
    print(f"det={det} parts={len(A.parts)} blocks={A.data.shape[0]}: {bad} of {runs} runs bad", flush=True)


if __name__ == "__main__":
    main()
