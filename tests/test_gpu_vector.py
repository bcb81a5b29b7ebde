"""GPU parity of the residual path: assemble_vector, apply_lifting, set_bc,
and the reference's setF sequence (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:817-845)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
RTOL = 1e-12


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _setup(oracle, ct, p, n, dev, seed=1):
    from femasm import fem, mesh

    m = mesh.create_unit_square(*n, cell_type=ct, device=dev) if len(n) == 2 else \
        mesh.create_unit_cube(*n, cell_type=ct, device=dev)
    V = fem.functionspace(m, ("Lagrange", p, (m.gdim,)))
    g = torch.Generator().manual_seed(seed)
    u = (1e-3 * (torch.rand(V.num_dofs, generator=g, dtype=torch.float64) - 0.5)).to(dev)
    f = (1e4 * (torch.rand(V.num_dofs, generator=g, dtype=torch.float64) - 0.5)).to(dev)
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
    return m, V, u, f, E


def _np(t):
    return None if t is None else t.cpu().numpy()


CASES = [(3, 1, (6, 5)), (3, 2, (4, 3)), (4, 1, (4, 3)), (4, 2, (3, 3)), (-4, 1, (2, 3, 2)), (-4, 2, (2, 2, 2)),
         (8, 1, (2, 2, 2)), (8, 2, (2, 1, 2))]


@pytest.mark.parametrize("ct,p,n", CASES)
def test_residual_matches_oracle(oracle, dev, ct, p, n):
    from femasm import fem

    m, V, u, f, E = _setup(oracle, ct, p, n, dev)
    L = fem.LinearElasticity(V, E=E, nu=0.3, u=u, f=f)
    b = fem.assemble_vector(L)
    lam, mu = oracle.lame(_np(E), 0.3)
    ref = oracle.assemble_residual(ct, p, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, u=_np(u), f=_np(f))
    assert np.abs(_np(b) - ref).max() <= RTOL * np.abs(ref).max()


def test_residual_damage_law(oracle, dev):
    from femasm import fem

    m, V, u, f, E = _setup(oracle, 3, 1, (9, 7), dev)
    g = torch.Generator().manual_seed(4)
    d = torch.rand(V.num_nodes, generator=g, dtype=torch.float64)
    d[d < 0.3] = 0.0
    d = d.to(dev)
    L = fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d, f=f)
    b = fem.assemble_vector(L)
    lam, mu = oracle.lame(_np(E), 0.3)
    ref = oracle.assemble_residual(3, 1, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, u=_np(u), f=_np(f), d=_np(d),
                                   kind=1)
    assert np.abs(_np(b) - ref).max() <= RTOL * np.abs(ref).max()


@pytest.mark.parametrize("ct,p,n", CASES)
def test_lifting_and_set_bc(oracle, dev, ct, p, n):
    """The reference's setF: b = F(u); apply_lifting(b, [J], [bcs], [u], -1); set_bc(b, bcs, u, -1)."""
    from femasm import fem

    m, V, u, f, E = _setup(oracle, ct, p, n, dev)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01] + [0.0] * (m.gdim - 1), right, V)]
    J = fem.LinearElasticity(V, E=E, nu=0.3, u=u, f=f)
    b = fem.assemble_vector(J)
    fem.apply_lifting(b, [J], [bcs], x0=[u], alpha=-1.0)
    fem.set_bc(b, bcs, x0=u, alpha=-1.0)
    marker, gv = fem._combine_bcs(V, bcs)
    lam, mu = oracle.lame(_np(E), 0.3)
    args = (ct, p, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu)
    ref = oracle.assemble_residual(*args, u=_np(u), f=_np(f))
    ref = oracle.apply_lifting(*args, ref, _np(marker), _np(gv), x0=_np(u), alpha=-1.0)
    mk = _np(marker).astype(bool)
    ref[mk] = -1.0 * (_np(gv)[mk] - _np(u)[mk])
    assert np.abs(_np(b) - ref).max() <= RTOL * np.abs(ref).max()


def test_lifting_damage_law(oracle, dev):
    from femasm import fem

    m, V, u, f, E = _setup(oracle, 3, 1, (8, 6), dev)
    g = torch.Generator().manual_seed(9)
    d = (torch.rand(V.num_nodes, generator=g, dtype=torch.float64) * 0.9).to(dev)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0.0], right, V)]
    J = fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d)
    b = torch.zeros(V.num_dofs, dtype=torch.float64, device=dev)
    fem.apply_lifting(b, [J], [bcs], x0=[u], alpha=-1.0)
    marker, gv = fem._combine_bcs(V, bcs)
    lam, mu = oracle.lame(_np(E), 0.3)
    ref = oracle.apply_lifting(3, 1, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, np.zeros(V.num_dofs),
                               _np(marker), _np(gv), x0=_np(u), alpha=-1.0, u=_np(u), d=_np(d), kind=1)
    assert np.abs(_np(b) - ref).max() <= RTOL * np.abs(ref).max()
