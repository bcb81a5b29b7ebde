"""The Newton driver over the GPU assembly: dolfinx NonlinearProblem +
NewtonSolver semantics (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:705-890) with GPU
F / J / CG, against the same Newton iteration run on the CPU with the oracle's F and J and a
direct sparse solve. Tolerances: the converged solutions agree to 1e-9 relative (the GPU Krylov
solve stops at ksp_rtol 1e-12, the CPU solve is direct, so the GPU may need one more Newton
step to push ||F|| below atol)."""
import numpy as np
import pytest
import scipy.sparse as sps
import scipy.sparse.linalg as spla
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _np(t):
    return None if t is None else t.cpu().numpy()


def test_bsr_mult_and_block_diag(oracle, dev):
    from femasm import fem, mesh

    m = mesh.create_unit_cube(3, 2, 2, mesh.CellType.tetrahedron, device=dev)
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
    A = fem.assemble_matrix(fem.LinearElasticity(V, E=E, nu=0.3))
    S = A.to_scipy()
    x = torch.linspace(-1, 1, V.num_dofs, dtype=torch.float64, device=dev)
    y = A.mult(x)
    ref = S @ _np(x)
    assert np.abs(_np(y) - ref).max() <= 1e-13 * np.abs(ref).max()
    D = _np(A.block_diagonal())
    Sd = S.toarray()
    for r in range(V.num_nodes):
        np.testing.assert_array_equal(D[r], Sd[3 * r:3 * r + 3, 3 * r:3 * r + 3])


def _oracle_newton(oracle, kind, ct, p, V, m, lam, mu, u0, marker, gv, f=None, d=None, rtol=1e-7, atol=5e-8,
                   max_it=10):
    """dolfinx NewtonSolver iteration on the CPU with the oracle's residual / tangent."""
    cells, geom, x = _np(V.dofmap), _np(m.cells), _np(m.x)
    bs = m.gdim
    indptr, indices = oracle.sparsity(cells, V.num_nodes)
    u = u0.copy()

    def F(u):
        b = oracle.assemble_residual(ct, p, cells, geom, x, lam, mu, u=u, f=f, d=d, kind=kind)
        b = oracle.apply_lifting(ct, p, cells, geom, x, lam, mu, b, marker, gv, x0=u, alpha=-1.0, u=u, d=d, kind=kind)
        b[marker != 0] = -(gv[marker != 0] - u[marker != 0])
        return b

    def J(u):
        if kind == 0:
            vals = oracle.assemble_elasticity(ct, p, cells, geom, x, lam, mu, indptr, indices, bc=marker)
        elif kind == 1:
            vals = oracle.assemble_damage(cells, geom, x, lam, mu, u, d, indptr, indices, bc=marker)
        else:
            vals = oracle.assemble_neohookean(ct, p, cells, geom, x, lam, mu, u, indptr, indices, bc=marker)
        return sps.bsr_matrix((vals, indices, indptr), shape=(V.num_dofs, V.num_dofs)).tocsr()

    b = F(u)
    it, r0, hist = 0, 0.0, [np.linalg.norm(b)]
    conv = hist[-1] < atol
    while not conv and it < max_it:
        dx = spla.spsolve(J(u).tocsc(), b)
        u -= dx
        it += 1
        b = F(u)
        if it == 1:
            r0 = np.linalg.norm(dx)
        hist.append(np.linalg.norm(b))
        conv = hist[-1] / r0 < rtol or hist[-1] < atol
    return u, it, conv, hist


def _bcs(fem, V, m, disp):
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    return [fem.dirichletbc(0.0, left, V), fem.dirichletbc([disp] + [0.0] * (m.gdim - 1), right, V)]


@pytest.mark.parametrize("kind,ct,p,n", [(0, -4, 2, (3, 2, 2)), (0, 3, 1, (8, 6)), (2, -4, 2, (3, 2, 2)),
                                         (2, 3, 2, (5, 4)), (2, 8, 1, (3, 2, 2)), (1, 3, 1, (10, 8))])
def test_newton_matches_oracle_newton(oracle, dev, kind, ct, p, n):
    from femasm import fem, mesh, nls

    m = (mesh.create_unit_square(*n, cell_type=ct, device=dev) if len(n) == 2
         else mesh.create_unit_cube(*n, cell_type=ct, device=dev))
    V = fem.functionspace(m, ("Lagrange", p, (m.gdim,)))
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
    u = fem.Function(V)
    f = torch.zeros(V.num_dofs, dtype=torch.float64, device=dev)
    f[1::m.gdim] = -1e3  # body force along y (the reference's f, asym_elasto_damage_model_symb_sym.py:310)
    d = None
    disp = 0.05 if kind == 2 else 1e-3
    if kind == 0:
        form = fem.LinearElasticity(V, E=E, nu=0.3, u=u, f=f)
    elif kind == 1:
        xn = V.tabulate_dof_coordinates()
        d = (0.6 * torch.exp(-20 * ((xn[:, 0] - 0.5) ** 2 + (xn[:, 1] - 0.5) ** 2))).contiguous()
        form = fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d, f=f)
    else:
        form = fem.NeoHookean(V, E=E, nu=0.3, u=u, f=f)
    bcs = _bcs(fem, V, m, disp)
    problem = nls.NonlinearProblem(form, u, bcs)
    solver = nls.NewtonSolver(None, problem)
    solver.rtol, solver.atol, solver.max_it = 1e-7, 5e-8, 10  # the reference's settings (:709-713)
    it, conv = solver.solve(u)
    assert conv
    marker, gv = fem._combine_bcs(V, bcs)
    lam, mu = oracle.lame(_np(E), 0.3)
    ku, kit, kconv, khist = _oracle_newton(oracle, kind, ct, p, V, m, lam, mu, np.zeros(V.num_dofs), _np(marker),
                                           _np(gv), f=_np(f), d=_np(d))
    assert kconv and kit <= it <= kit + 1, (it, kit, solver.history, khist)
    un = _np(u.x)
    assert np.abs(un - ku).max() <= 1e-9 * np.abs(ku).max()
    # the constrained dofs hold their prescribed values after the first update
    mk = _np(marker) != 0
    np.testing.assert_allclose(un[mk], _np(gv)[mk], rtol=0, atol=1e-14)
