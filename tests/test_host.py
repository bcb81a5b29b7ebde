"""Host-side logic of femasm.fem that needs no GPU: the Dirichlet marker cache."""
import torch

from femasm import fem, mesh


def _space():
    m = mesh.create_unit_cube(2, 2, 2, cell_type=mesh.CellType.tetrahedron, device=torch.device("cpu"))
    return fem.functionspace(m, ("Lagrange", 1, (3,)))


def test_bc_cache_sees_reassigned_g():
    """A bc whose g (or dofs) is replaced by a new tensor every step must not reuse an older step's
    combined values, even when the allocator hands the new tensor a freed tensor's storage."""
    V = _space()
    nodes = torch.arange(4)
    bc = fem.dirichletbc(0.0, nodes, V)
    for step in range(6):
        g = torch.zeros(V.num_dofs, dtype=torch.float64)
        g[bc.dofs] = float(step + 1)
        bc.g = g
        marker, gc = fem._combine_bcs(V, [bc])
        assert torch.equal(gc[bc.dofs], torch.full((bc.dofs.numel(),), float(step + 1), dtype=torch.float64))
        assert int(marker.sum()) == bc.dofs.numel()
        del g
    # an in-place edit of g also misses the cache
    bc.g[bc.dofs] = -7.0
    _, gc = fem._combine_bcs(V, [bc])
    assert float(gc[bc.dofs[0]]) == -7.0
    # new dofs tensor
    bc.dofs = bc.dofs[:3].clone()
    marker, _ = fem._combine_bcs(V, [bc])
    assert int(marker.sum()) == 3


def test_bc_cache_hits_unchanged_bcs():
    V = _space()
    bc = fem.dirichletbc(1.5, torch.arange(5), V)
    m1, g1 = fem._combine_bcs(V, [bc])
    m2, g2 = fem._combine_bcs(V, [bc])
    assert m1 is m2 and g1 is g2
    m3, g3 = fem._combine_bcs(V, [bc], with_g=False)
    assert g3 is None and torch.equal(m3, m1)
