"""Pins the CPU oracle (oracle/fa_oracle.c) before anything is compared against it.

The reference ships no assembly fixtures, so the oracle is pinned by:
the reference's own libc material table, SymPy exact integration, the rigid-body null
space, and a SymPy second derivative of the reference damage potential.
"""
import itertools
import math

import numpy as np
import pytest
import sympy as sp


def test_e_range_matches_reference_libc_table(oracle):
    # FEniCSx/mechanic2d/asym_elasto_damage_model.cc:533-545 — values quoted in SURVEY.md §8c
    E = oracle.e_range()
    assert E.shape == (200,)
    np.testing.assert_allclose(E[:3], [1.9321608e7, 7.0402010e7, 2.6005025e7], rtol=1e-8)
    assert E.min() >= 5e6 and E.max() <= 1e8


@pytest.mark.parametrize("ct,p", [(3, 1), (3, 2), (-4, 1), (-4, 2), (4, 1), (4, 2), (4, 3), (8, 1), (8, 2), (8, 3)])
def test_nodal_basis(oracle, ct, p):
    X = oracle.nodes(ct, p)
    v, g = oracle.tabulate(ct, p, X)
    np.testing.assert_allclose(v, np.eye(X.shape[0]), atol=1e-13)
    # partition of unity: gradients sum to zero at any point
    pts, _ = oracle.quadrature(ct, 4)
    v, g = oracle.tabulate(ct, p, pts)
    np.testing.assert_allclose(v.sum(1), 1.0, atol=1e-13)
    np.testing.assert_allclose(g.sum(1), 0.0, atol=1e-12)


def _ref_integral(ct, expo):
    if ct == 3:
        a, b = expo
        return sp.Rational(math.factorial(a) * math.factorial(b), math.factorial(a + b + 2))
    if ct == -4:
        a, b, c = expo
        return sp.Rational(math.factorial(a) * math.factorial(b) * math.factorial(c), math.factorial(a + b + c + 3))
    return sp.Mul(*[sp.Rational(1, e + 1) for e in expo])


@pytest.mark.parametrize("ct,m", [(3, 1), (3, 2), (3, 5), (-4, 1), (-4, 2), (-4, 4), (4, 4), (4, 6), (8, 4), (8, 6)])
def test_quadrature_exact(oracle, ct, m):
    pts, w = oracle.quadrature(ct, m)
    td = pts.shape[1]
    for expo in itertools.product(range(m + 1), repeat=td):
        if sum(expo) > m and ct in (3, -4):
            continue
        if max(expo) > m:
            continue
        num = (w * np.prod([pts[:, d] ** expo[d] for d in range(td)], axis=0)).sum()
        assert abs(num - float(_ref_integral(ct, expo))) < 1e-14


def _sympy_element_matrix(ct, p, xv, lam, mu):
    """Exact element stiffness on an affine simplex by SymPy: Lagrange basis from the
    oracle's node set (rational), integrals by the simplex monomial formula."""
    td = 2 if ct == 3 else 3
    X = [sp.symbols("X0:%d" % td)][0]
    nodes = oracle_nodes_rational(ct, p)
    mons = [m for m in itertools.product(range(p + 1), repeat=td) if sum(m) <= p]
    V = sp.Matrix([[sp.Mul(*[n[d] ** m[d] for d in range(td)]) for m in mons] for n in nodes])
    C = V.inv()
    phis = [sum(C[k, i] * sp.Mul(*[X[d] ** mons[k][d] for d in range(td)]) for k in range(len(mons))) for i in range(len(nodes))]
    xv = [[sp.nsimplify(c) for c in v] for v in xv]
    J = sp.Matrix([[xv[k + 1][i] - xv[0][i] for k in range(td)] for i in range(td)])
    Jinv = J.inv()
    detJ = abs(J.det())
    grads = [sp.Matrix([[sp.diff(ph, X[k]) for k in range(td)]]) * Jinv for ph in phis]
    nn = len(nodes)
    K = sp.zeros(nn * td, nn * td)
    for a in range(nn):
        for b in range(nn):
            for i in range(td):
                for j in range(td):
                    integrand = sp.expand(lam * grads[a][i] * grads[b][j] + mu * grads[a][j] * grads[b][i]
                                          + (mu * sum(grads[a][k] * grads[b][k] for k in range(td)) if i == j else 0))
                    poly = sp.Poly(integrand, *X)
                    val = sum(coef * _ref_integral(ct, mon) for mon, coef in poly.terms())
                    K[a * td + i, b * td + j] = val * detJ
    return np.array(K.evalf(30).tolist(), dtype=np.float64)


def oracle_nodes_rational(ct, p):
    if ct == 3:
        V = [(0, 0), (1, 0), (0, 1)]
        E = [(1, 2), (0, 2), (0, 1)]
    else:
        V = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1)]
        E = [(2, 3), (1, 3), (1, 2), (0, 3), (0, 2), (0, 1)]
    nodes = [tuple(sp.Integer(c) for c in v) for v in V]
    if p == 2:
        for a, b in E:
            nodes.append(tuple(sp.Rational(V[a][d] + V[b][d], 2) for d in range(len(V[0]))))
    return nodes


@pytest.mark.parametrize("ct,p", [(3, 1), (3, 2), (-4, 1), (-4, 2)])
def test_element_matrix_vs_sympy(oracle, ct, p):
    rng = np.random.default_rng(7)
    td = 2 if ct == 3 else 3
    xv = np.eye(td + 1, td, k=-1) + 0.2 * np.round(rng.uniform(-1, 1, (td + 1, td)), 2)
    lam, mu = 1.7, 0.9
    nn = oracle.lib().ora_num_nodes(ct, p)
    cells = np.arange(nn, dtype=np.int32)[None, :]
    geom = np.arange(td + 1, dtype=np.int32)[None, :]
    A = oracle.cell_matrices_elasticity(ct, p, cells, geom, xv, lam, mu)[0]
    Kx = _sympy_element_matrix(ct, p, xv.tolist(), sp.Rational(17, 10), sp.Rational(9, 10))
    np.testing.assert_allclose(A, Kx, rtol=1e-13, atol=1e-13 * np.abs(Kx).max())


@pytest.mark.parametrize("ct,p", [(3, 1), (3, 2), (-4, 1), (-4, 2), (4, 1), (4, 2), (4, 3), (8, 1), (8, 2), (8, 3)])
def test_rigid_body_null_space(oracle, ct, p):
    td = 2 if ct in (3, 4) else 3
    rng = np.random.default_rng(11)
    Xn = oracle.nodes(ct, p)
    nv = {3: 3, -4: 4, 4: 4, 8: 8}[ct]
    # an affine image of the reference cell (so higher-order nodes map consistently)
    Amap = np.eye(td) + 0.15 * rng.uniform(-1, 1, (td, td))
    xv = Xn[:nv] @ Amap.T + 0.3
    xn = Xn @ Amap.T + 0.3
    cells = np.arange(Xn.shape[0], dtype=np.int32)[None, :]
    geom = np.arange(nv, dtype=np.int32)[None, :]
    K = oracle.cell_matrices_elasticity(ct, p, cells, geom, xv, 2.0, 1.0)[0]
    np.testing.assert_allclose(K, K.T, atol=1e-12 * np.abs(K).max())
    modes = []
    for d in range(td):
        t = np.zeros_like(xn); t[:, d] = 1.0; modes.append(t.reshape(-1))
    rots = [(0, 1)] if td == 2 else [(0, 1), (0, 2), (1, 2)]
    for i, j in rots:
        r = np.zeros_like(xn); r[:, i] = -xn[:, j]; r[:, j] = xn[:, i]; modes.append(r.reshape(-1))
    for mvec in modes:
        assert np.abs(K @ mvec).max() < 1e-11 * np.abs(K).max()
    ev = np.linalg.eigvalsh(K)
    assert (ev > -1e-10 * ev.max()).all()
    assert (np.abs(ev) < 1e-10 * ev.max()).sum() == len(modes)


def _psi_sympy():
    """The reference damage potential (FEniCSx/mechanic2d/asym_ufl.py:37-51 = MFEM Potential,
    MFEM/mechanic2d/asym_elasto_damage_model.cc:100-155) in Voigt strains (e00, e11, gamma=2 e01),
    with the indicator alphas as symbols (piecewise constant where the signs do not change)."""
    e00, e11, gam, lam, mu, d, al, al1, al2 = sp.symbols("e00 e11 gamma lam mu d al al1 al2", real=True)
    e01 = gam / 2
    I1 = e00 + e11
    I2 = e01 * e01 - e00 * e11
    r = sp.sqrt(I1 * I1 + 4 * I2)
    ev1, ev2 = (I1 + r) / 2, (I1 - r) / 2
    psi = I1 * I1 * (1 - al * d) * lam / 2 + mu * ((1 - al1 * d) * ev1 ** 2 + (1 - al2 * d) * ev2 ** 2)
    return psi, (e00, e11, gam), (lam, mu, d, al, al1, al2), (ev1, ev2, I1)


@pytest.mark.parametrize("seed", range(6))
def test_damage_tangent_is_hessian_of_reference_potential(oracle, seed):
    """MFEM's hand-written tangent `hook` (restated in the oracle) equals the SymPy Hessian of the
    UFL potential psi; asym_stress equals its gradient. Pins rows a2-a4 of SURVEY §8."""
    psi, evars, pvars, (ev1, ev2, I1) = _psi_sympy()
    grad = [sp.diff(psi, v) for v in evars]
    hess = [[sp.diff(g, v) for v in evars] for g in grad]
    rng = np.random.default_rng(seed)
    lam, mu = 5.7e7, 3.8e7
    d = float(rng.uniform(0.05, 0.95))
    s = rng.normal(size=3) * 1e-3
    strain = np.array([s[0], s[1], s[2]])  # e00, e11, e01
    sub = {evars[0]: strain[0], evars[1]: strain[1], evars[2]: 2 * strain[2], pvars[0]: lam, pvars[1]: mu,
           pvars[2]: d}
    e1v, e2v, i1v = [float(x.subs(sub)) for x in (ev1, ev2, I1)]
    sub.update({pvars[3]: 1.0 if i1v >= 0 else 0.0, pvars[4]: 1.0 if e1v >= 0 else 0.0,
                pvars[5]: 1.0 if e2v >= 0 else 0.0})
    H = np.array([[float(h.subs(sub)) for h in row] for row in hess])
    G = np.array([float(g.subs(sub)) for g in grad])
    hook = oracle.damage_hook(strain, lam, mu, d)
    np.testing.assert_allclose(hook, H, rtol=1e-9, atol=1e-9 * np.abs(H).max())
    sig = oracle.damage_stress(strain, lam, mu, d, w=1.0)  # (s00, s11, s01)
    np.testing.assert_allclose(sig, G, rtol=1e-9, atol=1e-9 * np.abs(G).max())


def test_damage_law_linear_limit(oracle):
    """d = 0 gives the linear Hooke tangent (the bridge from the reference to the linear configs)."""
    lam, mu = 2.0, 1.5
    h = oracle.damage_hook(np.array([1e-3, -2e-3, 5e-4]), lam, mu, 0.0)
    np.testing.assert_array_equal(h, [[lam + 2 * mu, lam, 0], [lam, lam + 2 * mu, 0], [0, 0, mu]])


@pytest.mark.parametrize("gd", [2, 3])
def test_neo_hookean_tangent_is_hessian(oracle, gd):
    """The oracle's closed-form neo-Hookean tangent equals the SymPy Hessian of psi(F)."""
    Fs = sp.Matrix(gd, gd, lambda i, j: sp.Symbol(f"F{i}{j}", real=True))
    lam, mu = sp.Rational(17, 10), sp.Rational(9, 10)
    J = Fs.det()
    psi = mu / 2 * (sum(v ** 2 for v in Fs) + (1 if gd == 2 else 0) - 3) - mu * sp.log(J) + lam / 2 * sp.log(J) ** 2
    flat = list(Fs)
    H = sp.hessian(psi, flat)
    rng = np.random.default_rng(gd)
    Fn = np.eye(gd) + 0.1 * rng.uniform(-1, 1, (gd, gd))
    sub = {flat[k]: Fn.reshape(-1)[k] for k in range(gd * gd)}
    Hn = np.array(H.subs(sub).evalf(30).tolist(), dtype=np.float64)
    A = oracle.neo_tangent(Fn, 1.7, 0.9)
    np.testing.assert_allclose(A, Hn, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("gd", [2, 3])
def test_neo_hookean_stress_is_gradient(oracle, gd):
    """The oracle's first Piola stress equals the SymPy gradient of psi(F) (residual of config E)."""
    Fs = sp.Matrix(gd, gd, lambda i, j: sp.Symbol(f"F{i}{j}", real=True))
    lam, mu = sp.Rational(17, 10), sp.Rational(9, 10)
    J = Fs.det()
    psi = mu / 2 * (sum(v ** 2 for v in Fs) + (1 if gd == 2 else 0) - 3) - mu * sp.log(J) + lam / 2 * sp.log(J) ** 2
    flat = list(Fs)
    rng = np.random.default_rng(10 + gd)
    Fn = np.eye(gd) + 0.1 * rng.uniform(-1, 1, (gd, gd))
    sub = {flat[k]: Fn.reshape(-1)[k] for k in range(gd * gd)}
    Pn = np.array([float(sp.diff(psi, v).subs(sub).evalf(30)) for v in flat]).reshape(gd, gd)
    np.testing.assert_allclose(oracle.neo_stress(Fn, 1.7, 0.9), Pn, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("ct,deg", [(3, 2), (-4, 2)])
def test_neo_hookean_residual_tangent_consistent(oracle, ct, deg):
    """Assembled neo-Hookean residual r(u) and tangent K(u): K du matches the central difference
    of r (the Newton driver's consistency requirement), on a small perturbed mesh."""
    from femasm import mesh as fmesh
    from femasm import fem

    m = (fmesh.create_unit_square(2, 2, fmesh.CellType.triangle) if ct == 3
         else fmesh.create_unit_cube(1, 1, 2, fmesh.CellType.tetrahedron))
    V = fem.functionspace(m, ("Lagrange", deg, (m.gdim,)))
    cells = V.dofmap.cpu().numpy()
    xn = V.tabulate_dof_coordinates().cpu().numpy()
    geom = m.cells.cpu().numpy()
    x = m.x.cpu().numpy()
    rng = np.random.default_rng(4)
    u = 0.01 * rng.standard_normal(xn.shape[0] * m.gdim)
    du = rng.standard_normal(u.shape)
    lam, mu = 1.3, 0.7
    nn = cells.shape[1]
    Ae = oracle.assemble_neohookean(ct, deg, cells, geom, x, lam, mu, u, cell_matrices=True)
    Kdu = np.zeros_like(u)
    bs = m.gdim
    for c in range(cells.shape[0]):
        dofs = (cells[c][:, None] * bs + np.arange(bs)[None, :]).reshape(-1)
        Kdu[dofs] += Ae[c] @ du[dofs]
    h = 1e-6
    rp = oracle.assemble_residual(ct, deg, cells, geom, x, lam, mu, u=u + h * du, kind=2)
    rm = oracle.assemble_residual(ct, deg, cells, geom, x, lam, mu, u=u - h * du, kind=2)
    np.testing.assert_allclose((rp - rm) / (2 * h), Kdu, rtol=1e-6, atol=1e-7 * np.abs(Kdu).max())
    assert nn == cells.shape[1]
