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
