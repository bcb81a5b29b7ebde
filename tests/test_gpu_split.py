"""GPU: the split gather (fa_gather_prepare + fa_gather_rows over row ranges, femasm.fem.SplitGather)
and the in-kernel slot search (FEMASM_SLOTS=0) against the CPU oracle. Bar as test_gpu_parity:
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
def test_in_kernel_slot_search(dev, oracle, monkeypatch, ct, p, n):
    from femasm import fem

    monkeypatch.setenv("FEMASM_SLOTS", "0")
    monkeypatch.setenv("FEMASM_CONTRIB", "0")  # the LDS-atomic gather's plan (triangles default to the owner plan)
    V, a, bcs, indptr, indices, ref = _problem(dev, oracle, ct, p, n)
    A = fem.assemble_matrix(a, bcs=bcs)
    plan_entry = next(iter(V.__dict__["_plans"].values()))
    assert plan_entry[3] is None, "FEMASM_SLOTS=0 must plan without a slot map"
    torch.cuda.synchronize()
    err = np.abs(A.data.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err


@pytest.mark.parametrize("order", ["pos", "1", "0"])
@pytest.mark.parametrize("ct,p,n", [("tetrahedron", 2, 5), ("tetrahedron", 1, 6), ("triangle", 2, 9),
                                    ("triangle", 1, 12)])
def test_slot_order(dev, oracle, monkeypatch, order, ct, p, n):
    """fa_plan_order's positional plan (default), its per-lane block order alone, and the plain slot map
    (FEMASM_SLOT_ORDER "pos", "1", "0") all give the oracle's matrix."""
    from femasm import fem

    monkeypatch.setenv("FEMASM_SLOT_ORDER", order)
    monkeypatch.setenv("FEMASM_CONTRIB", "0")  # the LDS-atomic gather's plan refinements
    V, a, bcs, indptr, indices, ref = _problem(dev, oracle, ct, p, n)
    A = fem.assemble_matrix(a, bcs=bcs)
    plan = next(iter(V.__dict__["_plans"].values()))[0]
    assert (plan.slot_order > 0) == (order != "0")
    assert bool(plan.eadj) == (order == "pos")
    torch.cuda.synchronize()
    err = np.abs(A.data.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err


@pytest.mark.parametrize("order", ["morton", "0"])
@pytest.mark.parametrize("ct,p,n", [("tetrahedron", 2, 5), ("hexahedron", 2, 4), ("triangle", 1, 12)])
def test_chunk_locality_order(dev, oracle, monkeypatch, order, ct, p, n):
    """fa_plan_locality: the gather visits its chunks in Morton order of their positions (default) or
    in row order (FEMASM_CHUNK_ORDER=0); the order is a permutation and the matrix is the oracle's."""
    from femasm import fem

    monkeypatch.setenv("FEMASM_CHUNK_ORDER", order)
    monkeypatch.setenv("FEMASM_CONTRIB", "0")  # the LDS-atomic gather's plan refinements
    V, a, bcs, indptr, indices, ref = _problem(dev, oracle, ct, p, n)
    A = fem.assemble_matrix(a, bcs=bcs)
    entry = next(iter(V.__dict__["_plans"].values()))
    plan, corder = entry[0], entry[5]
    if order == "0" or plan.nchunks <= 1:
        assert corder is None and not plan.corder
    else:
        assert plan.corder == corder.data_ptr()
        assert torch.equal(torch.sort(corder.cpu()).values, torch.arange(plan.nchunks, dtype=torch.int32))
    torch.cuda.synchronize()
    err = np.abs(A.data.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err
