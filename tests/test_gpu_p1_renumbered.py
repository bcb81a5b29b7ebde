"""P1 spaces whose node numbering is not the geometry's (FunctionSpace.from_dofmap: a permuted
vertex numbering). The fused P1 gather reads each vertex's coordinates by geometry node; its bc bits
come from the node pack when the dofmap is the geometry dofmap and per cell (k_cell_bcmask, read by
dof node) otherwise. The matrix of the renumbered space, permuted back, must equal the
geometry-numbered one, bc rows, columns and diagonal included (round 5: the round-4 fused path read
the bits by geometry node and marked the wrong rows; this test fails on it)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("ct,n", [(-4, (12, 11, 10)), (3, (40, 37))])
def test_renumbered_p1_space_equals_geometry_numbering(oracle, dev, ct, n):
    from femasm import fem, mesh

    m = mesh.create_unit_square(*n, cell_type=ct, device=dev) if len(n) == 2 else \
        mesh.create_unit_cube(*n, cell_type=ct, device=dev)
    gd = m.gdim
    V = fem.functionspace(m, ("Lagrange", 1, (gd,)))
    nv = V.num_nodes
    perm = torch.randperm(nv, generator=torch.Generator().manual_seed(7)).to(dev)
    V2 = fem.FunctionSpace.from_dofmap(m, 1, gd, perm[m.cells.to(torch.int64)], nv)
    assert V2.dofmap.data_ptr() != m.cells.data_ptr()  # the per-cell bc bits of the fused path
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], device=dev)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    assert left.numel() > 0 and right.numel() > 0
    mats = []
    for W, mp in ((V, lambda v: v), (V2, lambda v: perm[v.to(torch.int64)])):
        bcs = [fem.dirichletbc(0.0, mp(left), W), fem.dirichletbc([0.01] + [0.0] * (gd - 1), mp(right), W)]
        A = fem.assemble_matrix(fem.LinearElasticity(W, E=E, nu=0.3), bcs=bcs, diagonal=2.0)
        mats.append(A.to_scipy().tocsr())
    # row / column d of V2 is dof (perm[v], c) for dof (v, c) of V
    p = perm.cpu().numpy()
    idx = (p[:, None] * gd + np.arange(gd)).reshape(-1)
    B = mats[1][idx][:, idx]
    A = mats[0]
    assert (abs(A - B)).max() <= 1e-12 * abs(A).max()
    # the constrained rows: identity times the diagonal
    dofs = (left.cpu().numpy()[:, None] * gd + np.arange(gd)).reshape(-1)
    rows = A[dofs].toarray()
    np.testing.assert_array_equal(rows[np.arange(dofs.size), dofs], 2.0)
    assert np.count_nonzero(rows) == dofs.size
