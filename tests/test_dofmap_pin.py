"""The product's dofmaps and Dirichlet selections pinned independently of the product (VERDICT r4
"What's weak" 1): the GPU parity tests feed the oracle the product's own dofmap and bc marker, so a
wrong P2/P3 dofmap or bc selection would pass them. Here, on the CPU:

* every (cell, local node) of the product's dofmap maps to a global node whose coordinate, computed by
  the ORACLE from the cell's vertices and its own reference nodes (oracle.nodes), is the same from every
  cell that shares it, and equals V.tabulate_dof_coordinates();
* the global matrix the oracle assembles on the product's dofmap has the rigid-body null space:
  K r = 0 (per row, relative to sum_j |K_ij r_j|) for the rigid modes evaluated at the dof coordinates,
  for P1 / P2 triangles and tetrahedra, Q2 quadrilaterals, Q2 / Q3 hexahedra (GLL-warped at Q3), with
  the structured (lattice) and the generic (unstructured) numbering;
* the structured and the generic dofmaps give the same matrix under the coordinate-matched node
  permutation;
* locate_entities_boundary + locate_dofs_topological (the reference's own bc calls,
  FEniCSx/mechanic2d/asym_elasto_damage_model.cc:627-638, :651-662) select, with dolfinx closure
  semantics, the nodes the oracle's coordinates put on the plane: vertex nodes only at dim 0, every
  node on it at the facet dimension (= locate_dofs_geometrical)."""
import numpy as np
import pytest
import torch

from femasm import fem, mesh

CPU = torch.device("cpu")
NV = {3: 3, -4: 4, 4: 4, 8: 8}


def _space(ct, p, n, structured=True):
    m = mesh.create_unit_square(*n, cell_type=ct, device=CPU) if len(n) == 2 else \
        mesh.create_unit_cube(*n, cell_type=ct, device=CPU)
    if not structured:
        m.structured = None
    return m, fem.functionspace(m, ("Lagrange", p, (m.gdim,)))


def _geometry_basis(ct, X):
    """P1 / Q1 vertex basis at reference points (restated here, oracle side)."""
    if ct in (3, -4):
        return np.concatenate([1.0 - X.sum(1, keepdims=True), X], axis=1)
    td = X.shape[1]
    cols = []
    for b in range(1 << td):
        f = np.ones(X.shape[0])
        for d in range(td):
            f = f * (X[:, d] if (b >> d) & 1 else 1.0 - X[:, d])
        cols.append(f)
    return np.stack(cols, 1)


def _oracle_node_coords(oracle, ct, p, m, V):
    """[ncells, nn, gdim] node coordinates from each cell's vertices and the oracle's reference nodes."""
    Xn = oracle.nodes(ct, p)
    Psi = _geometry_basis(ct, Xn)  # [nn, nv]
    xv = m.x.numpy()[m.cells.numpy().astype(np.int64)]  # [nc, nv, gdim]
    return np.einsum("kv,cvd->ckd", Psi, xv)


CASES = [(3, 1, (5, 4), True), (3, 2, (4, 3), True), (3, 2, (4, 3), False), (-4, 1, (3, 2, 2), True),
         (-4, 2, (2, 3, 2), True), (-4, 2, (2, 3, 2), False), (4, 2, (4, 3), True), (4, 2, (4, 3), False),
         (8, 2, (2, 2, 3), True), (8, 2, (2, 2, 3), False), (8, 3, (2, 2, 2), True)]


@pytest.mark.parametrize("ct,p,n,structured", CASES)
def test_dofmap_consistent_with_oracle_coordinates(oracle, ct, p, n, structured):
    m, V = _space(ct, p, n, structured)
    xc = _oracle_node_coords(oracle, ct, p, m, V)
    dm = V.dofmap.numpy().astype(np.int64)
    assert dm.min() >= 0 and dm.max() < V.num_nodes
    assert np.unique(dm).size == V.num_nodes, "every node is used by some cell"
    xg = V.tabulate_dof_coordinates().numpy()
    err = np.abs(xc - xg[dm]).max()
    assert err < 1e-13, f"a cell's local node is numbered as a global node elsewhere ({err:.2e})"
    # distinct nodes have distinct coordinates (no two lattice positions merged)
    key = np.round(xg * 1e9).astype(np.int64)
    assert np.unique(key, axis=0).shape[0] == V.num_nodes


def _rigid_modes(x):
    n, td = x.shape
    modes = []
    for d in range(td):
        t = np.zeros_like(x); t[:, d] = 1.0; modes.append(t.reshape(-1))
    for i, j in ([(0, 1)] if td == 2 else [(0, 1), (0, 2), (1, 2)]):
        r = np.zeros_like(x); r[:, i] = -x[:, j]; r[:, j] = x[:, i]; modes.append(r.reshape(-1))
    return modes


def _oracle_matrix(oracle, ct, p, m, V, E=None):
    cells = V.dofmap.numpy().astype(np.int32)
    indptr, indices = oracle.sparsity(cells, V.num_nodes)
    Ev = np.full(m.num_cells, 7.0) if E is None else E
    lam, mu = oracle.lame(Ev, 0.3)
    vals = oracle.assemble_elasticity(ct, p, cells, m.cells.numpy().astype(np.int32), m.x.numpy(), lam, mu, indptr,
                                      indices)
    return oracle.bsr_to_dense(indptr, indices, vals, V.num_nodes)


@pytest.mark.parametrize("ct,p,n,structured", CASES)
def test_global_rigid_body_null_space(oracle, ct, p, n, structured):
    m, V = _space(ct, p, n, structured)
    E = oracle.e_range()[np.arange(m.num_cells) % 200]
    K = _oracle_matrix(oracle, ct, p, m, V, E)
    x = V.tabulate_dof_coordinates().numpy()
    for r in _rigid_modes(x):
        res = np.abs(K @ r)
        scale = np.abs(K) @ np.abs(r) + 1e-300
        assert (res <= 1e-12 * scale).all(), f"K r != 0: worst {np.max(res / scale):.2e}"


@pytest.mark.parametrize("ct,p,n", [(3, 2, (4, 3)), (-4, 2, (2, 2, 3)), (4, 2, (3, 4)), (8, 2, (2, 3, 2))])
def test_structured_and_generic_dofmaps_agree(oracle, ct, p, n):
    mats, xs = [], []
    for structured in (True, False):
        m, V = _space(ct, p, n, structured)
        E = oracle.e_range()[np.arange(m.num_cells) % 200]
        mats.append(_oracle_matrix(oracle, ct, p, m, V, E))
        xs.append(V.tabulate_dof_coordinates().numpy())
    # node permutation by coordinates: generic node g <-> structured node s
    def order(x):
        return np.lexsort(np.round(x * 1e9).astype(np.int64).T[::-1])
    os_, og = order(xs[0]), order(xs[1])
    np.testing.assert_allclose(xs[0][os_], xs[1][og], atol=1e-14)
    td = xs[0].shape[1]
    perm_s = (os_[:, None] * td + np.arange(td)).reshape(-1)
    perm_g = (og[:, None] * td + np.arange(td)).reshape(-1)
    A, B = mats[0][np.ix_(perm_s, perm_s)], mats[1][np.ix_(perm_g, perm_g)]
    assert np.abs(A - B).max() <= 1e-13 * np.abs(A).max()


@pytest.mark.parametrize("ct,p,n", [(3, 1, (5, 4)), (3, 2, (4, 3)), (-4, 1, (3, 2, 2)), (-4, 2, (2, 3, 2)),
                                    (4, 2, (3, 3)), (8, 2, (2, 2, 2)), (8, 3, (2, 2, 2))])
@pytest.mark.parametrize("structured", [True, False])
def test_bc_selection_topological_vs_oracle(oracle, ct, p, n, structured):
    if not structured and p == 3:
        pytest.skip("generic dofmap: degree <= 2")
    m, V = _space(ct, p, n, structured)
    on_left = lambda x: torch.isclose(x[0], torch.zeros_like(x[0]))  # noqa: E731
    xc = _oracle_node_coords(oracle, ct, p, m, V)  # [nc, nn, gdim]
    dm = V.dofmap.numpy().astype(np.int64)
    plane = np.abs(xc[..., 0]) < 1e-12
    want_all = np.unique(dm[plane])
    vert = np.zeros_like(plane)
    vert[:, :NV[ct]] = True
    want_vertex = np.unique(dm[plane & vert])
    # dim 0: the reference's call (vertex nodes only for P >= 2)
    verts = mesh.locate_entities_boundary(m, 0, on_left)
    got0 = fem.locate_dofs_topological(V, 0, verts).numpy()
    np.testing.assert_array_equal(got0, want_vertex)
    # facets: every node on the plane, as locate_dofs_geometrical
    facets = mesh.locate_entities_boundary(m, m.tdim - 1, on_left)
    gotf = fem.locate_dofs_topological(V, m.tdim - 1, facets).numpy()
    np.testing.assert_array_equal(gotf, want_all)
    np.testing.assert_array_equal(np.sort(fem.locate_dofs_geometrical(V, on_left).numpy()), want_all)
    if p >= 2:
        assert want_vertex.size < want_all.size
    if m.tdim == 3:  # edges of the plane: their vertices' and interior nodes (not the face interiors)
        edges = mesh.locate_entities_boundary(m, 1, on_left)
        ge = set(fem.locate_dofs_topological(V, 1, edges).numpy().tolist())
        assert set(want_vertex.tolist()) <= ge <= set(want_all.tolist())


def test_locate_entities_boundary_only_boundary():
    """Entities inside the domain are never returned, even when the marker accepts everything."""
    m, V = _space(-4, 1, (3, 3, 3))
    allv = mesh.locate_entities_boundary(m, 0, lambda x: torch.ones(x.shape[1], dtype=torch.bool))
    x = m.x[allv.to(torch.int64)]
    on_b = ((x < 1e-12) | (x > 1 - 1e-12)).any(1)
    assert bool(on_b.all()) and allv.numel() == 4 ** 3 - 2 ** 3
    f = mesh.locate_entities_boundary(m, 2, lambda x: torch.ones(x.shape[1], dtype=torch.bool))
    assert f.numel() == 6 * 3 * 3 * 2  # 2 triangles per boundary square
