"""The HIP assembly on the product's own dofmaps, pinned without the oracle's inputs
(tests/test_dofmap_pin.py is the CPU side):

* rigid-body null space of the GPU-assembled global matrix: K r = 0 per row for the rigid modes at
  V.tabulate_dof_coordinates() (no bcs), through A.mult (fa_bsr_mult), every element family, with the
  structured and the generic numbering, on meshes with enough rows for several gather chunks;
* structured vs generic numbering: the two GPU matrices agree under the coordinate-matched node
  permutation;
* the reference's bc calls (locate_entities_boundary + locate_dofs_topological at dim 0,
  FEniCSx/mechanic2d/asym_elasto_damage_model.cc:627-638, :651-662) on P2 tetrahedra, assembled on the
  GPU and compared with the oracle given a marker the ORACLE derives from its own node coordinates."""
import numpy as np
import pytest
import torch

from rowparity import assert_rows_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _space(ct, p, n, dev, structured=True):
    from femasm import fem, mesh

    m = mesh.create_unit_square(*n, cell_type=ct, device=dev) if len(n) == 2 else \
        mesh.create_unit_cube(*n, cell_type=ct, device=dev)
    if not structured:
        m.structured = None
    return m, fem.functionspace(m, ("Lagrange", p, (m.gdim,)))


def _rigid_modes(x):
    n, td = x.shape
    modes = []
    for d in range(td):
        t = torch.zeros_like(x); t[:, d] = 1.0; modes.append(t.reshape(-1))
    for i, j in ([(0, 1)] if td == 2 else [(0, 1), (0, 2), (1, 2)]):
        r = torch.zeros_like(x); r[:, i] = -x[:, j]; r[:, j] = x[:, i]; modes.append(r.reshape(-1))
    return modes


CASES = [(3, 1, (40, 33), True), (3, 2, (30, 27), True), (3, 2, (30, 27), False), (-4, 1, (12, 11, 10), True),
         (-4, 2, (9, 8, 10), True), (-4, 2, (9, 8, 10), False), (4, 2, (31, 29), True), (4, 2, (31, 29), False),
         (8, 2, (7, 6, 8), True), (8, 2, (7, 6, 8), False), (8, 3, (5, 6, 5), True)]


@pytest.mark.parametrize("ct,p,n,structured", CASES)
def test_gpu_matrix_rigid_body_null_space(oracle, dev, ct, p, n, structured):
    from femasm import fem

    m, V = _space(ct, p, n, dev, structured)
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    A = fem.assemble_matrix(a)
    Aabs = fem.create_matrix(a)
    Aabs.data.copy_(A.data.abs())
    x = V.tabulate_dof_coordinates()
    for r in _rigid_modes(x):
        res = A.mult(r).abs()
        scale = Aabs.mult(r.abs()) + 1e-300
        worst = float((res / scale).max())
        assert worst <= 1e-12, f"K r != 0 on the GPU matrix: worst {worst:.2e}"


@pytest.mark.parametrize("ct,p,n", [(3, 2, (21, 17)), (-4, 2, (6, 7, 5)), (4, 2, (19, 16)), (8, 2, (5, 6, 4))])
def test_gpu_structured_and_generic_agree(oracle, dev, ct, p, n):
    from femasm import fem

    mats, xs = [], []
    for structured in (True, False):
        m, V = _space(ct, p, n, dev, structured)
        E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
        A = fem.assemble_matrix(fem.LinearElasticity(V, E=E, nu=0.3))
        mats.append(A.to_scipy())
        xs.append(V.tabulate_dof_coordinates().cpu().numpy())

    def order(x):
        return np.lexsort(np.round(x * 1e9).astype(np.int64).T[::-1])

    os_, og = order(xs[0]), order(xs[1])
    np.testing.assert_allclose(xs[0][os_], xs[1][og], atol=1e-14)
    td = xs[0].shape[1]
    ps = (os_[:, None] * td + np.arange(td)).reshape(-1)
    pg = (og[:, None] * td + np.arange(td)).reshape(-1)
    A = mats[0].tocsr()[ps][:, ps]
    B = mats[1].tocsr()[pg][:, pg]
    d = abs(A - B)
    assert d.max() <= 1e-12 * abs(A).max()


def test_reference_bc_calls_p2_against_oracle_marker(oracle, dev):
    """dim-0 selection (the reference's call) on P2 tetrahedra: the assembled rows equal the oracle's
    with the marker the oracle derives itself (vertex nodes on x = 0 / x = 1 by its node coordinates)."""
    from femasm import fem, mesh

    m, V = _space(-4, 2, (7, 6, 5), dev)
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    left = lambda x: torch.isclose(x[0], torch.zeros_like(x[0]))  # noqa: E731
    right = lambda x: torch.isclose(x[0], torch.ones_like(x[0]))  # noqa: E731
    bl = fem.locate_dofs_topological(V, 0, mesh.locate_entities_boundary(m, 0, left))
    br = fem.locate_dofs_topological(V, 0, mesh.locate_entities_boundary(m, 0, right))
    bcs = [fem.dirichletbc(0.0, bl, V), fem.dirichletbc([0.01, 0.0, 0.0], br, V)]
    A = fem.assemble_matrix(a, bcs=bcs)
    # the oracle's marker: vertex nodes (local < 4) whose oracle coordinate lies on a plane
    dm = V.dofmap.cpu().numpy().astype(np.int64)
    Xn = oracle.nodes(-4, 2)
    Psi = np.concatenate([1.0 - Xn.sum(1, keepdims=True), Xn], axis=1)
    xc = np.einsum("kv,cvd->ckd", Psi, m.x.cpu().numpy()[m.cells.cpu().numpy().astype(np.int64)])
    onp = (np.abs(xc[..., 0]) < 1e-12) | (np.abs(xc[..., 0] - 1.0) < 1e-12)
    onp[:, 4:] = False
    nodes = np.unique(dm[onp])
    marker = np.zeros(V.num_dofs, dtype=np.int8)
    for c in range(3):
        marker[nodes * 3 + c] = 1
    lam, mu = oracle.lame(E.cpu().numpy(), 0.3)
    ip, ix = oracle.sparsity(dm.astype(np.int32), V.num_nodes)
    ref = oracle.assemble_elasticity(-4, 2, dm.astype(np.int32), m.cells.cpu().numpy().astype(np.int32),
                                     m.x.cpu().numpy(), lam, mu, ip, ix, bc=marker)
    np.testing.assert_array_equal(A.indptr.cpu().numpy(), ip)
    np.testing.assert_array_equal(A.indices.cpu().numpy(), ix)
    assert_rows_close(A.data.cpu().numpy(), ref, ip, 1e-12)
    # and the selection is NOT the facet one at P2 (mid-edge nodes of the plane stay free)
    bf = fem.locate_dofs_geometrical(V, left)
    assert bl.numel() < bf.numel()
