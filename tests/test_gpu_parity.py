"""GPU parity: the HIP assembly path (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star: "global matrix within 1e-12 of reference"), per scalar row:
max_j |A_gpu[i, j] - A_oracle[i, j]| <= 1e-12 * max_j |A_oracle[i, j]| (tests/rowparity.py);
sparsity patterns must be identical.
"""
import os

import numpy as np
import pytest
import torch

from rowparity import assert_rows_close

pytestmark = pytest.mark.gpu

RTOL = 1e-12
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _mesh(ct, n, dev, perturb=0.0, structured=True):
    from femasm import mesh

    m = mesh.create_unit_square(*n, cell_type=ct, device=dev) if len(n) == 2 else \
        mesh.create_unit_cube(*n, cell_type=ct, device=dev)
    if perturb:
        g = torch.Generator().manual_seed(3)
        x = m.x.cpu()
        interior = ((x > 1e-9) & (x < 1 - 1e-9)).all(1)
        h = 1.0 / max(n)
        x[interior] += perturb * h * (torch.rand(x[interior].shape, generator=g, dtype=torch.float64) - 0.5)
        m.x = x.to(dev)
    if not structured:
        m.structured = None
    return m


def _E_cells(oracle, nc, dev):
    Er = oracle.e_range()
    return torch.tensor(Er[np.arange(nc) % 200], dtype=torch.float64, device=dev)


def _oracle_matrix(oracle, V, a, marker=None, diag=1.0):
    m = V.mesh
    cells = V.dofmap.cpu().numpy()
    geom = m.cells.cpu().numpy()
    x = m.x.cpu().numpy()
    indptr, indices = oracle.sparsity(cells, V.num_nodes)
    lam, mu = oracle.lame(a.E.cpu().numpy(), a.nu)
    bc = None if marker is None else marker.cpu().numpy()
    vals = oracle.assemble_elasticity(int(m.cell_type), V.degree, cells, geom, x, lam, mu, indptr, indices, bc=bc,
                                      diag=diag, qdeg=a.qdeg)
    return indptr, indices, vals


def _assert_close(A, ref_vals):
    assert_rows_close(A.data.cpu().numpy(), ref_vals, A.indptr.cpu().numpy(), RTOL)


CASES = [
    (3, 1, (8, 7)), (3, 2, (5, 4)),
    (4, 1, (5, 4)), (4, 2, (4, 5)), (4, 3, (3, 2)),
    (-4, 1, (3, 4, 2)), (-4, 2, (3, 2, 3)),
    (8, 1, (3, 2, 2)), (8, 2, (2, 2, 2)), (8, 3, (2, 1, 2)),
]


def _setup(oracle, ct, p, n, dev, **kw):
    from femasm import fem

    m = _mesh(ct, n, dev, **kw)
    V = fem.functionspace(m, ("Lagrange", p, (m.gdim,)))
    a = fem.form(fem.LinearElasticity(V, E=_E_cells(oracle, m.num_cells, dev), nu=0.3))
    return m, V, a


@pytest.mark.parametrize("ct,p,n", CASES)
def test_pattern_matches_oracle(oracle, dev, ct, p, n):
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    A = fem.create_matrix(a)
    indptr, indices = oracle.sparsity(V.dofmap.cpu().numpy(), V.num_nodes)
    np.testing.assert_array_equal(A.indptr.cpu().numpy(), indptr)
    np.testing.assert_array_equal(A.indices.cpu().numpy(), indices)


@pytest.mark.parametrize("method", ["gather", "scatter"])
@pytest.mark.parametrize("ct,p,n", CASES)
def test_assemble_matches_oracle(oracle, dev, ct, p, n, method):
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    A = fem.assemble_matrix(a, bcs=[], method=method)
    torch.cuda.synchronize()
    _, _, ref = _oracle_matrix(oracle, V, a)
    _assert_close(A, ref)


@pytest.mark.parametrize("method", ["gather", "scatter"])
@pytest.mark.parametrize("ct,p,n", CASES)
def test_assemble_with_dirichlet(oracle, dev, ct, p, n, method):
    """Reference bcs: x = 0 clamped, x = 1 prescribed (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:620-669)."""
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    imp = [0.01] + [0.0] * (m.gdim - 1)
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc(imp, right, V)]
    A = fem.assemble_matrix(a, bcs=bcs, method=method)
    marker, _ = fem._combine_bcs(V, bcs)
    _, _, ref = _oracle_matrix(oracle, V, a, marker=marker, diag=1.0)
    _assert_close(A, ref)
    # constrained rows are identity rows
    Ad = A.to_dense()
    rows = marker.cpu().numpy().astype(bool)
    np.testing.assert_array_equal(Ad[rows][:, rows], np.eye(rows.sum()))
    assert np.abs(Ad[rows][:, ~rows]).max(initial=0) == 0.0


@pytest.mark.parametrize("ct,p,n", [(-4, 2, (5, 4, 3)), (-4, 1, (6, 5, 4)), (4, 2, (7, 5)), (3, 2, (6, 5)),
                                    (8, 1, (4, 3, 3))])
def test_component_dirichlet(oracle, dev, ct, p, n):
    """Single-component constraints (x = 0: u_x only; y = 0: u_y only, overlapping at the corner):
    the records' per-dof bc bits (formed from the constrained dofs' side since round 6,
    k_rec_bcbits) zero exactly those rows / columns."""
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    x0 = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    y0 = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[1], torch.zeros_like(x[1])))
    bcs = [fem.dirichletbc(0.0, x0, V, components=[0]), fem.dirichletbc(0.0, y0, V, components=[1])]
    A = fem.assemble_matrix(a, bcs=bcs)
    marker, _ = fem._combine_bcs(V, bcs)
    assert 0 < int(marker.sum()) < 2 * V.num_nodes
    _, _, ref = _oracle_matrix(oracle, V, a, marker=marker, diag=1.0)
    _assert_close(A, ref)


@pytest.mark.parametrize("ct,p,n", [(4, 1, (4, 3)), (4, 2, (3, 3)), (8, 1, (2, 2, 2)), (8, 2, (2, 2, 1))])
@pytest.mark.parametrize("method", ["gather", "scatter"])
def test_non_affine_cells(oracle, dev, ct, p, n, method):
    """Perturbed interior vertices: bilinear/trilinear geometry with a Jacobian per quadrature point."""
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev, perturb=0.3)
    A = fem.assemble_matrix(a, method=method)
    _, _, ref = _oracle_matrix(oracle, V, a)
    _assert_close(A, ref)


@pytest.mark.parametrize("ct,p,n", [(3, 2, (4, 3)), (-4, 2, (2, 3, 2)), (4, 2, (3, 2)), (8, 2, (2, 2, 1))])
def test_generic_dofmap(oracle, dev, ct, p, n):
    """Unstructured (edge/face-based) node numbering, as for a Gmsh mesh."""
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev, structured=False)
    A = fem.assemble_matrix(a)
    _, _, ref = _oracle_matrix(oracle, V, a)
    _assert_close(A, ref)


@pytest.mark.parametrize("ct,p,n", CASES)
def test_tabulate_matches_oracle(oracle, dev, ct, p, n):
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    Ae = fem.tabulate_cells(a).cpu().numpy()
    lam, mu = oracle.lame(a.E.cpu().numpy(), a.nu)
    ref = oracle.cell_matrices_elasticity(int(ct), p, V.dofmap.cpu().numpy(), m.cells.cpu().numpy(),
                                          m.x.cpu().numpy(), lam, mu)
    err = np.abs(Ae - ref).max()
    assert err <= RTOL * np.abs(ref).max()


def test_reference_square_msh(oracle, dev):
    """The reference's own debug mesh (common/data/square.msh, 62 nodes / 98 triangles) with
    E = E_range[tag % 200] per physical tag (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:533-545)."""
    from femasm import fem, mesh

    m = mesh.read_gmsh(os.path.join(GOLDEN, "square.msh"), gdim=2, device=dev)
    assert (m.num_vertices, m.num_cells) == (62, 98)
    Er = oracle.e_range()
    E = torch.tensor(Er[m.cell_tags.cpu().numpy() % 200], device=dev)
    V = fem.functionspace(m, ("Lagrange", 1, (2,)))
    a = fem.LinearElasticity(V, E=E, nu=0.3, quadrature_degree=1)
    A = fem.assemble_matrix(a)
    _, _, ref = _oracle_matrix(oracle, V, a)
    _assert_close(A, ref)
    gold = np.load(os.path.join(GOLDEN, "square_p1_elasticity.npz"))
    np.testing.assert_array_equal(A.indices.cpu().numpy(), gold["indices"])
    assert_rows_close(A.data.cpu().numpy(), gold["data"], gold["indptr"], RTOL)


def test_reference_square_through_xdmf(oracle, dev, tmp_path):
    """The reference driver's input path (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:155-162,
    :543-545): mesh and cell tags read from an XDMF file (the square.msh mesh written with
    femasm.io), E from the tags, assembled on the GPU: the same matrix as the golden square.msh case."""
    from femasm import fem, io, materials, mesh

    g = mesh.read_gmsh(os.path.join(GOLDEN, "square.msh"), gdim=2)
    tags = io.MeshTags(2, torch.arange(g.num_cells, dtype=torch.int32), g.cell_tags, "square_cells")
    path = str(tmp_path / "square.xdmf")
    with io.XDMFFile(path, "w") as f:
        f.write_mesh(g, "square")
        f.write_meshtags(tags, g)
    with io.XDMFFile(path) as f:
        m = f.read_mesh("square", device=dev)
        t = f.read_meshtags(m, "square_cells")
    V = fem.functionspace(m, ("Lagrange", 1, (2,)))
    a = fem.LinearElasticity(V, E=materials.e_from_cell_tags(t, m.num_cells), nu=0.3, quadrature_degree=1)
    A = fem.assemble_matrix(a)
    gold = np.load(os.path.join(GOLDEN, "square_p1_elasticity.npz"))
    np.testing.assert_array_equal(A.indices.cpu().numpy(), gold["indices"])
    assert_rows_close(A.data.cpu().numpy(), gold["data"], gold["indptr"], RTOL)


@pytest.mark.parametrize("method", ["gather", "scatter"])
def test_damage_law_matches_oracle(oracle, dev, method):
    """Reference mechanic2d J with damage (MFEM hand tangent restated), random u and d."""
    from femasm import fem

    m = _mesh(3, (9, 8), dev)
    V = fem.functionspace(m, ("Lagrange", 1, (2,)))
    g = torch.Generator().manual_seed(5)
    u = (1e-3 * (torch.rand(V.num_dofs, generator=g, dtype=torch.float64) - 0.5)).to(dev)
    d = torch.rand(V.num_nodes, generator=g, dtype=torch.float64)
    d[d < 0.4] = 0.0  # mix of damaged and undamaged cells
    d = d.to(dev)
    E = _E_cells(oracle, m.num_cells, dev)
    a = fem.AsymDamage(V, E=E, nu=0.3, u=u, d=d)
    A = fem.assemble_matrix(a, method=method)
    cells = V.dofmap.cpu().numpy()
    indptr, indices = oracle.sparsity(cells, V.num_nodes)
    lam, mu = oracle.lame(E.cpu().numpy(), 0.3)
    ref = oracle.assemble_damage(cells, m.cells.cpu().numpy(), m.x.cpu().numpy(), lam, mu, u.cpu().numpy(),
                                 d.cpu().numpy(), indptr, indices)
    _assert_close(A, ref)


def test_gather_equals_scatter_larger(oracle, dev):
    """Both device algorithms agree on a mesh too large for the oracle to be quick."""
    from femasm import fem

    m, V, a = _setup(oracle, -4, 2, (12, 11, 10), dev)
    A1 = fem.assemble_matrix(a, method="gather")
    d1 = A1.data.clone()
    A2 = fem.assemble_matrix(a, method="scatter")
    scale = d1.abs().max()
    assert ((A2.data - d1).abs().max() <= RTOL * scale).item()
    # gather is run-to-run reproducible
    A3 = fem.assemble_matrix(a, method="gather")
    assert ((A3.data - d1).abs().max() <= 1e-15 * scale).item()


@pytest.mark.parametrize("method", ["gather", "scatter"])
@pytest.mark.parametrize("ct,p,n", [(-4, 2, (3, 3, 2)), (3, 1, (9, 6)), (8, 2, (2, 2, 2))])
def test_row_parts(oracle, dev, ct, p, n, method):
    """Values split into many row parts (each its own allocation, row window in fa_bsr)."""
    from femasm import fem

    m, V, a = _setup(oracle, ct, p, n, dev)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V)]
    A = fem.create_matrix(a, max_part_bytes=4096)
    assert len(A.parts) > 3
    fem.assemble_matrix(a, bcs=bcs, A=A, method=method)
    marker, _ = fem._combine_bcs(V, bcs)
    _, _, ref = _oracle_matrix(oracle, V, a, marker=marker)
    _assert_close(A, ref)
