"""GPU parity of the block-owner gather (k_gather_own, contribution plan fa_plan_contrib; the
default for triangles, gather_plan(owner=True) forces it for tetrahedra too) against the CPU oracle, with
the per-row 1e-12 bar of tests/rowparity.py.

Covers P1/P2 triangles and tetrahedra with and without the reference's Dirichlet sets
(FEniCSx/mechanic2d/asym_elasto_damage_model.cc:620-669), meshes of many chunks (lane segments
that end inside a block: the partial-sum atomics), unstructured numbering, cells with mu |J| < 0,
and agreement with the LDS-atomic gather."""
import numpy as np
import pytest
import torch

from rowparity import assert_rows_close
from test_gpu_parity import _E_cells, _mesh, _oracle_matrix

pytestmark = pytest.mark.gpu
RTOL = 1e-12


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture
def contrib():
    return dict(owner=True)


def _assemble(oracle, dev, ct, p, n, bcs_on, owner=True, **kw):
    from femasm import _lib, fem

    m = _mesh(ct, n, dev, **kw)
    V = fem.functionspace(m, ("Lagrange", p, (m.gdim,)))
    a = fem.form(fem.LinearElasticity(V, E=_E_cells(oracle, m.num_cells, dev), nu=0.3))
    bcs = []
    if bcs_on:
        left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
        right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
        bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01] + [0.0] * (m.gdim - 1), right, V)]
    A = fem.assemble_matrix(a, bcs=bcs, plan=dict(owner=owner))
    plan = fem.gather_plan(V, A, 0, _lib.FA_LINEAR_ELASTICITY, owner=owner)
    torch.cuda.synchronize()
    return V, a, bcs, A, plan


CASES = [(3, 1, (9, 7)), (3, 2, (6, 5)), (-4, 1, (4, 3, 5)), (-4, 2, (3, 4, 3)),
         (-4, 2, (10, 9, 8)), (3, 2, (40, 37))]


@pytest.mark.parametrize("bcs_on", [False, True])
@pytest.mark.parametrize("ct,p,n", CASES)
def test_owner_gather_matches_oracle(oracle, dev, contrib, ct, p, n, bcs_on):
    from femasm import fem

    V, a, bcs, A, plan = _assemble(oracle, dev, ct, p, n, bcs_on)
    assert plan.contrib, "the contribution plan was not built (the owner kernel did not run)"
    marker = fem._combine_bcs(V, bcs)[0] if bcs else None
    _, _, ref = _oracle_matrix(oracle, V, a, marker=marker, diag=1.0)
    assert_rows_close(A.data.cpu().numpy(), ref, A.indptr.cpu().numpy(), RTOL)


def test_owner_gather_unstructured_numbering(oracle, dev, contrib):
    V, a, bcs, A, plan = _assemble(oracle, dev, -4, 2, (4, 3, 4), True, structured=False, perturb=0.3)
    from femasm import fem

    assert plan.contrib
    _, _, ref = _oracle_matrix(oracle, V, a, marker=fem._combine_bcs(V, bcs)[0], diag=1.0)
    assert_rows_close(A.data.cpu().numpy(), ref, A.indptr.cpu().numpy(), RTOL)


def test_owner_gather_inverted_cells(oracle, dev, contrib):
    """Cells with negative mu |J| (E < 0 on some cells): the sign path of the kernel."""
    from femasm import fem

    m = _mesh(-4, (3, 3, 4), dev)
    V = fem.functionspace(m, ("Lagrange", 2, (m.gdim,)))
    E = _E_cells(oracle, m.num_cells, dev)
    E[::7] *= -1.0
    a = fem.form(fem.LinearElasticity(V, E=E, nu=0.3))
    A = fem.assemble_matrix(a, bcs=[], plan=contrib)
    from femasm import _lib

    assert fem.gather_plan(V, A, 0, _lib.FA_LINEAR_ELASTICITY, **contrib).contrib
    _, _, ref = _oracle_matrix(oracle, V, a)
    assert_rows_close(A.data.cpu().numpy(), ref, A.indptr.cpu().numpy(), RTOL)


@pytest.mark.parametrize("ct,p,n", [(-4, 2, (7, 6, 5)), (3, 1, (30, 20)), (3, 2, (12, 9))])
def test_owner_equals_lds_atomic_gather(oracle, dev, ct, p, n):
    out = {}
    for owner in (True, False):
        V, a, bcs, A, plan = _assemble(oracle, dev, ct, p, n, True, owner=owner)
        assert bool(plan.contrib) == owner
        out[owner] = (A.data.cpu().numpy(), A.indptr.cpu().numpy())
    assert_rows_close(out[True][0], out[False][0], out[False][1], 1e-13)


def test_contrib_plan_refuses_oversized_chunks(oracle, dev):
    """fa_plan_contrib checks the chunking: a plan whose chunks hold more than 256 adjacency entries
    (two chunks of half the rows each) is refused with FA_E_CAPACITY rather than overrunning the
    kernel's cell staging."""
    import ctypes

    from femasm import _lib, fem

    m = _mesh(-4, (6, 6, 6), dev)
    V = fem.functionspace(m, ("Lagrange", 1, (m.gdim,)))
    a = fem.form(fem.LinearElasticity(V, E=_E_cells(oracle, m.num_cells, dev), nu=0.3))
    A = fem.create_matrix(a)
    L = _lib.load()
    fm, adj, fb = V._fa_mesh(), V._fa_adjacency(), A._fa_bsr(0)
    rs = torch.empty(V.num_nodes + 1, dtype=torch.int64, device=dev)
    plan = _lib.fa_plan()
    sh = _lib.stream_handle(dev)
    _lib.check(L.fa_plan_gather(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb), rs.data_ptr(),
                                ctypes.byref(plan), sh), "fa_plan_gather")
    n = V.num_nodes
    rs[:3] = torch.tensor([0, n // 2, n], dtype=torch.int64, device=dev)
    plan.nchunks = 2
    plan.max_adj = int(V.adjacency()[0][n].item())
    assert plan.max_adj > 256
    buf = torch.empty(16, dtype=torch.uint8, device=dev)
    rc = L.fa_plan_contrib(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb), buf.data_ptr(), 16,
                           ctypes.byref(plan), sh)
    assert rc == -5 and not plan.contrib
