"""GPU: the split gather (fa_gather_prepare + fa_gather_rows over row ranges, femasm.fem.SplitGather)
and the in-kernel slot search (gather_plan slots=False) against the CPU oracle. Bar as test_gpu_parity:
|A - A_oracle|_max <= 1e-12 |A_oracle|_max, identical patterns."""
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


def _problem(dev, oracle, ct_name, p, n):
    from femasm import fem, mesh

    ct = mesh.CellType[ct_name]
    m = mesh.create_unit_cube(n, n, n, cell_type=ct, device=dev) if ct in (mesh.CellType.tetrahedron,
                                                                           mesh.CellType.hexahedron) \
        else mesh.create_unit_square(n, n, cell_type=ct, device=dev)
    gd = m.gdim
    V = fem.functionspace(m, ("Lagrange", p, (gd,)))
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], dtype=torch.float64, device=dev)
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01] + [0.0] * (gd - 1), right, V)]
    marker, _ = fem._combine_bcs(V, bcs)
    cells = V.dofmap.cpu().numpy()
    indptr, indices = oracle.sparsity(cells, V.num_nodes)
    lam, mu = oracle.lame(E.cpu().numpy(), 0.3)
    ref = oracle.assemble_elasticity(int(ct), p, cells, m.cells.cpu().numpy(), m.x.cpu().numpy(), lam, mu, indptr,
                                     indices, bc=marker.cpu().numpy(), diag=1.0)
    return V, a, bcs, indptr, indices, ref


@pytest.mark.parametrize("ct,p,n", [("tetrahedron", 2, 5), ("tetrahedron", 1, 6), ("triangle", 2, 9),
                                    ("quadrilateral", 2, 7), ("hexahedron", 2, 3)])
def test_split_gather_ranges(dev, oracle, ct, p, n):
    from femasm import fem

    V, a, bcs, indptr, indices, ref = _problem(dev, oracle, ct, p, n)
    A = fem.create_matrix(a)
    A.parts[0][2].fill_(np.nan)  # every value must be written by exactly the planned ranges
    N = V.num_nodes
    cuts = [0, N // 5, N // 5 + 1, (2 * N) // 3, N]  # includes a one-row range
    ranges = list(zip(cuts[:-1], cuts[1:]))
    sg = fem.SplitGather(a, bcs, A, ranges)
    sg.prepare()
    for i in (2, 0, 3, 1):  # any order
        sg.rows(i)
    torch.cuda.synchronize()
    assert np.array_equal(A.indices.cpu().numpy(), indices)
    got = A.data.cpu().numpy()
    assert np.isfinite(got).all()
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err


@pytest.mark.parametrize("ct,p,n", [("tetrahedron", 2, 5), ("tetrahedron", 1, 6), ("triangle", 1, 12)])
def test_in_kernel_slot_search(dev, oracle, ct, p, n):
    from femasm import fem

    V, a, bcs, indptr, indices, ref = _problem(dev, oracle, ct, p, n)
    # the LDS-atomic gather's plan without a slot map (owner=False: triangles default to the owner plan)
    A = fem.assemble_matrix(a, bcs=bcs, plan=dict(slots=False, owner=False))
    plan_entry = next(iter(V.__dict__["_plans"].values()))
    assert plan_entry[3] is None, "slots=False must plan without a slot map"
    torch.cuda.synchronize()
    err = np.abs(A.data.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err


@pytest.mark.parametrize("order", ["positional", "steps", "none"])
@pytest.mark.parametrize("ct,p,n", [("tetrahedron", 2, 5), ("tetrahedron", 1, 6), ("triangle", 2, 9),
                                    ("triangle", 1, 12)])
def test_slot_order(dev, oracle, order, ct, p, n):
    """fa_plan_order's positional plan (default), its per-lane block order alone, and the plain slot map
    (gather_plan order "positional", "steps", "none") all give the oracle's matrix."""
    from femasm import fem

    V, a, bcs, indptr, indices, ref = _problem(dev, oracle, ct, p, n)
    A = fem.assemble_matrix(a, bcs=bcs, plan=dict(order=order, owner=False))
    plan = next(iter(V.__dict__["_plans"].values()))[0]
    assert (plan.slot_order > 0) == (order != "none")
    assert bool(plan.eadj) == (order == "positional")
    torch.cuda.synchronize()
    err = np.abs(A.data.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err


@pytest.mark.parametrize("locality", [True, False])
@pytest.mark.parametrize("ct,p,n", [("tetrahedron", 2, 5), ("hexahedron", 2, 4), ("triangle", 1, 12)])
def test_chunk_locality_order(dev, oracle, locality, ct, p, n):
    """fa_plan_locality: the gather visits its chunks in Morton order of their positions (default) or
    in row order (locality=False); the order is a permutation and the matrix is the oracle's."""
    from femasm import fem

    V, a, bcs, indptr, indices, ref = _problem(dev, oracle, ct, p, n)
    A = fem.assemble_matrix(a, bcs=bcs, plan=dict(locality=locality, owner=False))
    entry = next(iter(V.__dict__["_plans"].values()))
    plan, corder = entry[0], entry[5]
    if not locality or plan.nchunks <= 1:
        assert corder is None and not plan.corder
    else:
        assert plan.corder == corder.data_ptr()
        assert torch.equal(torch.sort(corder.cpu()).values, torch.arange(plan.nchunks, dtype=torch.int32))
    torch.cuda.synchronize()
    err = np.abs(A.data.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err


def test_split_gather_neo_needs_positional_plans(dev, oracle):
    """A neo-Hookean SplitGather without the positional plan fails at construction, with a message."""
    from femasm import fem, mesh

    m = mesh.create_unit_cube(2, 2, 2, cell_type=mesh.CellType.tetrahedron, device=dev)
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    u = torch.zeros(V.num_dofs, dtype=torch.float64, device=dev)
    a = fem.NeoHookean(V, E=1.0, nu=0.3, u=u)
    A = fem.create_matrix(a)
    with pytest.raises(ValueError, match="positional"):
        fem.SplitGather(a, [], A, [(0, V.num_nodes)], slots=False)


def test_split_gather_after_moving_vertices(dev, oracle):
    """Hexahedra: vertices moved in place after the SplitGather was planned (the mesh stops being
    affine); the next assembly is the oracle's matrix of the moved mesh."""
    from femasm import fem

    V, a, bcs, indptr, indices, _ = _problem(dev, oracle, "hexahedron", 2, 3)
    A = fem.create_matrix(a)
    N = V.num_nodes
    sg = fem.SplitGather(a, bcs, A, [(0, N // 2), (N // 2, N)])
    m = V.mesh
    x = m.x
    interior = ((x > 1e-9) & (x < 1 - 1e-9)).all(1)
    x[interior] += 0.05 * torch.sin(7.0 * x[interior])  # in place: same tensor, new version
    sg.prepare()
    sg.rows(0)
    sg.rows(1)
    torch.cuda.synchronize()
    marker, _ = fem._combine_bcs(V, bcs)
    lam, mu = oracle.lame(a.E.cpu().numpy(), 0.3)
    ref = oracle.assemble_elasticity(int(m.cell_type), 2, V.dofmap.cpu().numpy(), m.cells.cpu().numpy(),
                                     m.x.cpu().numpy(), lam, mu, indptr, indices, bc=marker.cpu().numpy(), diag=1.0)
    err = np.abs(A.data.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err
