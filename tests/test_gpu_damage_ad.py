"""The reference's USE_AD damage tangent on the GPU (MFEM/mechanic2d/asym_elasto_damage_model.cc
built with -DUSE_AD, MFEM/mechanic2d/Makefile:8-9): the hook is the forward-over-forward AD Hessian
of the damage potential (:100-155, admfem.hpp:672-700) reordered to Voigt (:761-763), and the
stress its AD gradient (:158-204). fem.AsymDamage(..., tangent="ad") -> FA_ASYM_DAMAGE_AD.

Oracle: the hand tangent / stress restated in oracle/fa_oracle.c (:207-329, :766-881). The two
are the same derivatives of the same potential (the reference reports AD vs hand solutions equal
to 1e-15, doc.tex:2215-2220), so they must agree per row to the parity bar of 1e-12."""
import numpy as np
import pytest
import torch

from rowparity import assert_rows_close

pytestmark = pytest.mark.gpu
RTOL = 1e-12


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _np(t):
    return None if t is None else t.cpu().numpy()


def _state(oracle, n, dev, seed, dmin=0.3, amp=1e-3):
    from femasm import fem, mesh

    m = mesh.create_unit_square(*n, cell_type=mesh.CellType.triangle, device=dev)
    V = fem.functionspace(m, ("Lagrange", 1, (2,)))
    g = torch.Generator().manual_seed(seed)
    u = (amp * (torch.rand(V.num_dofs, generator=g, dtype=torch.float64) - 0.5)).to(dev)
    d = torch.rand(V.num_nodes, generator=g, dtype=torch.float64)
    d[d < dmin] = 0.0  # damaged and undamaged cells
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
    return m, V, u, d.to(dev), E


@pytest.mark.parametrize("method", ["gather", "scatter"])
@pytest.mark.parametrize("seed", [5, 11])
def test_ad_tangent_matrix_equals_hand_oracle(oracle, dev, method, seed):
    from femasm import fem

    m, V, u, d, E = _state(oracle, (9, 8), dev, seed)
    a = fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d, tangent="ad")
    assert a.kind == 3
    A = fem.assemble_matrix(a, method=method)
    cells = V.dofmap.cpu().numpy()
    indptr, indices = oracle.sparsity(cells, V.num_nodes)
    lam, mu = oracle.lame(_np(E), 0.3)
    ref = oracle.assemble_damage(cells, _np(m.cells), _np(m.x), lam, mu, _np(u), _np(d), indptr, indices)
    np.testing.assert_array_equal(A.indices.cpu().numpy(), indices)
    assert_rows_close(A.data.cpu().numpy(), ref, indptr, RTOL)


def test_ad_tangent_with_dirichlet(oracle, dev):
    from femasm import fem

    m, V, u, d, E = _state(oracle, (8, 9), dev, 7)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0.0], right, V)]
    A = fem.assemble_matrix(fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d, tangent="ad"), bcs=bcs)
    marker, _ = fem._combine_bcs(V, bcs)
    cells = V.dofmap.cpu().numpy()
    indptr, indices = oracle.sparsity(cells, V.num_nodes)
    lam, mu = oracle.lame(_np(E), 0.3)
    ref = oracle.assemble_damage(cells, _np(m.cells), _np(m.x), lam, mu, _np(u), _np(d), indptr, indices,
                                 bc=_np(marker), diag=1.0)
    assert_rows_close(A.data.cpu().numpy(), ref, indptr, RTOL)


@pytest.mark.parametrize("amp", [1e-3, 1.0])
def test_ad_element_matrices_equal_hand(oracle, dev, amp):
    """Cell by cell (fa_tabulate_cells): the AD hook's element matrices equal the hand tangent's on
    the device, per element row, over strains in tension, compression and mixed states."""
    from femasm import fem

    m, V, u, d, E = _state(oracle, (12, 11), dev, 3, dmin=0.1, amp=amp)
    Ah = fem.tabulate_cells(fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d)).cpu().numpy()
    Aa = fem.tabulate_cells(fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d, tangent="ad")).cpu().numpy()
    scale = np.abs(Ah).max(axis=2, keepdims=True)
    assert (np.abs(Aa - Ah) <= RTOL * scale).all(), float((np.abs(Aa - Ah) / scale).max())


def test_ad_residual_equals_hand_oracle(oracle, dev):
    from femasm import fem

    m, V, u, d, E = _state(oracle, (9, 7), dev, 4)
    f = (1e4 * (torch.rand(V.num_dofs, generator=torch.Generator().manual_seed(2), dtype=torch.float64) - 0.5)).to(dev)
    b = fem.assemble_vector(fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d, f=f, tangent="ad"))
    lam, mu = oracle.lame(_np(E), 0.3)
    ref = oracle.assemble_residual(3, 1, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, u=_np(u), f=_np(f), d=_np(d),
                                   kind=1)
    assert np.abs(_np(b) - ref).max() <= RTOL * np.abs(ref).max()


def test_ad_lifting_equals_hand_oracle(oracle, dev):
    from femasm import fem

    m, V, u, d, E = _state(oracle, (8, 6), dev, 9)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0.0], right, V)]
    J = fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d, tangent="ad")
    b = torch.zeros(V.num_dofs, dtype=torch.float64, device=dev)
    fem.apply_lifting(b, [J], [bcs], x0=[u], alpha=-1.0)
    marker, gv = fem._combine_bcs(V, bcs)
    lam, mu = oracle.lame(_np(E), 0.3)
    ref = oracle.apply_lifting(3, 1, _np(V.dofmap), _np(m.cells), _np(m.x), lam, mu, np.zeros(V.num_dofs),
                               _np(marker), _np(gv), x0=_np(u), alpha=-1.0, u=_np(u), d=_np(d), kind=1)
    assert np.abs(_np(b) - ref).max() <= RTOL * np.abs(ref).max()
