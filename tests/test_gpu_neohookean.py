"""GPU parity of the neo-Hookean tangent (BASELINE config E): device forward-over-forward AD vs the
oracle's closed-form tangent, through gather, scatter and the per-cell tabulation."""
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


def _setup(oracle, ct, p, n, dev, amp=0.05):
    from femasm import fem, mesh

    m = mesh.create_unit_square(*n, cell_type=ct, device=dev) if len(n) == 2 else \
        mesh.create_unit_cube(*n, cell_type=ct, device=dev)
    V = fem.functionspace(m, ("Lagrange", p, (m.gdim,)))
    xn = V.tabulate_dof_coordinates()
    # u = amp * (sin pi x, sin pi y[, sin pi z]) at the nodes (SURVEY §8d neo-Hookean state)
    u = (amp * torch.sin(torch.pi * xn)).reshape(-1).contiguous()
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
    a = fem.NeoHookean(V, E=E, nu=0.3, u=u)
    return m, V, a


def _np(t):
    return t.cpu().numpy()


CASES = [(3, 1, (5, 4)), (3, 2, (4, 3)), (-4, 1, (2, 3, 2)), (-4, 2, (2, 2, 3)), (4, 2, (3, 2)), (8, 1, (2, 2, 2))]


@pytest.mark.parametrize("method", ["gather", "scatter"])
@pytest.mark.parametrize("ct,p,n", CASES)
def test_neohookean_matrix(oracle, dev, ct, p, n, method):
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V)]
    A = fem.assemble_matrix(a, bcs=bcs, method=method)
    marker, _ = fem._combine_bcs(V, bcs)
    indptr, indices = oracle.sparsity(_np(V.dofmap), V.num_nodes)
    lam, mu = oracle.lame(_np(a.E), 0.3)
    ref = oracle.assemble_neohookean(ct, p, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, _np(a.u), indptr, indices,
                                     bc=_np(marker))
    assert np.abs(_np(A.data) - ref).max() <= RTOL * np.abs(ref).max()


@pytest.mark.parametrize("ct,p,n", CASES[:4])
def test_neohookean_cell_matrices(oracle, dev, ct, p, n):
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    Ae = _np(fem.tabulate_cells(a))
    lam, mu = oracle.lame(_np(a.E), 0.3)
    ref = oracle.assemble_neohookean(ct, p, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, _np(a.u),
                                     cell_matrices=True)
    assert np.abs(Ae - ref).max() <= RTOL * np.abs(ref).max()


def test_neohookean_reduces_to_linear_at_zero_state(oracle, dev):
    """At u = 0 (F = I) the neo-Hookean tangent is the linear-elasticity tangent."""
    from femasm import fem

    m, V, a = _setup(oracle, -4, 2, (2, 2, 2), dev, amp=0.0)
    A1 = fem.assemble_matrix(a)
    d1 = A1.data.clone()
    lin = fem.LinearElasticity(V, E=a.E, nu=0.3)
    A2 = fem.assemble_matrix(lin)
    assert ((A2.data - d1).abs().max() <= RTOL * d1.abs().max()).item()


@pytest.mark.parametrize("ct,p,n", CASES)
def test_residual_matches_oracle(oracle, dev, ct, p, n):
    """Neo-Hookean residual (first Piola stress by device AD) vs the oracle's closed form."""
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    b = fem.assemble_vector(a)
    lam, mu = oracle.lame(_np(a.E), 0.3)
    ref = oracle.assemble_residual(ct, p, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, u=_np(a.u), kind=2)
    assert np.abs(_np(b) - ref).max() <= RTOL * np.abs(ref).max()


@pytest.mark.parametrize("ct,p,n", CASES)
def test_lifting_matches_oracle(oracle, dev, ct, p, n):
    """apply_lifting with the neo-Hookean tangent at the state (dolfinx semantics, alpha = -1)."""
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc([0.02] + [0.0] * (m.gdim - 1), right, V)]
    b = torch.zeros(V.num_dofs, dtype=torch.float64, device=dev)
    fem.apply_lifting(b, [a], [bcs], x0=[a.u], alpha=-1.0)
    marker, gv = fem._combine_bcs(V, bcs)
    lam, mu = oracle.lame(_np(a.E), 0.3)
    ref = oracle.apply_lifting(ct, p, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, np.zeros(V.num_dofs),
                               _np(marker), _np(gv), x0=_np(a.u), alpha=-1.0, u=_np(a.u), kind=2)
    assert np.abs(ref).max() > 0
    assert np.abs(_np(b) - ref).max() <= RTOL * np.abs(ref).max()


@pytest.mark.parametrize("ct,p,n", [(3, 2, (4, 3)), (-4, 1, (2, 3, 2)), (-4, 2, (3, 2, 3))])
def test_neohookean_gather_with_bcs(oracle, dev, ct, p, n):
    """The neo-Hookean gather (k_gather_neo, M records) against the oracle with Dirichlet rows."""
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01] + [0.0] * (m.gdim - 1), right, V)]
    A = fem.assemble_matrix(a, bcs=bcs)
    marker, _ = fem._combine_bcs(V, bcs)
    indptr, indices = oracle.sparsity(_np(V.dofmap), V.num_nodes)
    lam, mu = oracle.lame(_np(a.E), 0.3)
    ref = oracle.assemble_neohookean(ct, p, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, _np(a.u), indptr, indices,
                                     bc=_np(marker))
    assert np.abs(_np(A.data) - ref).max() <= RTOL * np.abs(ref).max()


@pytest.mark.parametrize("order", ["steps", "none"])
def test_neohookean_needs_positional_plan(oracle, dev, order):
    """A plan without the positional order is refused, never assembled another way: up front by
    gather_plan (ValueError), and by the library itself (FA_E_ARG) when such a plan reaches
    fa_assemble_matrix through the C ABI."""
    import ctypes

    from femasm import _lib, fem

    m, V, a = _setup(oracle, -4, 2, (2, 2, 2), dev)
    with pytest.raises(ValueError, match="positional"):
        fem.assemble_matrix(a, plan=dict(order=order))
    A = fem.create_matrix(a)
    plan = fem.gather_plan(V, A, 0, _lib.FA_LINEAR_ELASTICITY, order=order)  # a linear-kind plan of that order
    L = _lib.load()
    rc = L.fa_assemble_matrix(ctypes.byref(V._fa_mesh()), ctypes.byref(fem._fa_form(a)), ctypes.byref(V._fa_adjacency()),
                              ctypes.byref(plan), None, 1.0, ctypes.byref(A._fa_bsr(0)), _lib.FA_GATHER,
                              _lib.stream_handle(dev))
    assert rc == -1 and "positional plan" in L.fa_last_error().decode()
