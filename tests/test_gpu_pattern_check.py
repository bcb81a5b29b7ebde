"""fa_check_pattern: the device-side validation of the sparsity pattern and the node -> cell
adjacency (both built with rocPRIM sorts / scans, code the library does not control), reachable
through fem.create_matrix(check=True) and FA_CHECK_ERRORS (assemble_matrix(check=True)).
A pattern built by the library passes for every element family; corrupted copies (an unsorted row,
a missing pair, an extra column, a broken indptr, a broken adjacency) fail with FA_E_PATTERN."""
import pytest
import torch

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
    return fem.functionspace(m, ("Lagrange", p, (m.gdim,)))


CASES = [(3, 1, (7, 5), True), (3, 2, (6, 5), True), (4, 2, (5, 4), True), (-4, 1, (4, 3, 5), True),
         (-4, 2, (3, 4, 3), True), (-4, 2, (3, 3, 2), False), (8, 2, (3, 2, 3), True), (8, 3, (2, 3, 2), True)]


@pytest.mark.parametrize("ct,p,n,structured", CASES)
def test_library_pattern_passes(dev, ct, p, n, structured):
    from femasm import fem

    V = _space(ct, p, n, dev, structured)
    a = fem.LinearElasticity(V, E=1.0, nu=0.3)
    A = fem.create_matrix(a, check=True)
    assert A.indices.numel() > 0


def _expect_bad(V, indptr, indices, what):
    from femasm import _lib, fem

    with pytest.raises(_lib.FemasmError, match=what):
        fem.check_pattern(V, indptr, indices)


def test_corrupted_patterns_fail(dev):
    from femasm import fem

    V = _space(-4, 2, (3, 2, 2), dev)
    a = fem.LinearElasticity(V, E=1.0, nu=0.3)
    A = fem.create_matrix(a)
    ip, ix = A.indptr.clone(), A.indices.clone()
    r = 37
    b0, b1 = int(ip[r]), int(ip[r + 1])
    # two columns of a row swapped: unsorted
    bad = ix.clone()
    bad[b0], bad[b0 + 1] = ix[b0 + 1], ix[b0]
    _expect_bad(V, ip, bad, "unsorted")
    # a column replaced by one no cell of the row needs (kept sorted): a missing pair and an extra column
    bad = ix.clone()
    far = int(ix[b1 - 1]) + 1
    if far < V.num_nodes:
        bad[b1 - 1] = far
        _expect_bad(V, ip, bad, "missing")
    # a column out of range
    bad = ix.clone()
    bad[b1 - 1] = V.num_nodes + 5
    _expect_bad(V, ip, bad, "out of range")
    # indptr not monotone
    bad_ip = ip.clone()
    bad_ip[r + 1] = bad_ip[r] - 1
    _expect_bad(V, bad_ip, ix, "indptr")
    # the block count does not match indptr[nnodes]
    _expect_bad(V, ip, ix[:-1], "indptr")
    # the library's own pattern, checked again, passes
    fem.check_pattern(V, ip, ix)


def test_corrupted_adjacency_fails(dev):
    from femasm import _lib, fem

    V = _space(-4, 1, (3, 3, 3), dev)
    a = fem.LinearElasticity(V, E=1.0, nu=0.3)
    A = fem.create_matrix(a)
    ptr, idx = V.adjacency()
    keep = idx.clone()
    try:
        idx[5], idx[6] = keep[6], keep[5]  # entries of one node out of order (or moved to another node)
        with pytest.raises(_lib.FemasmError, match="adjacency"):
            fem.check_pattern(V, A.indptr, A.indices)
    finally:
        idx.copy_(keep)
    fem.check_pattern(V, A.indptr, A.indices)


def test_check_errors_flag_validates_pattern(dev):
    """assemble_matrix(check=True) (FA_CHECK_ERRORS) refuses a corrupted pattern before assembling."""
    from femasm import _lib, fem

    V = _space(-4, 2, (2, 2, 2), dev)
    a = fem.LinearElasticity(V, E=1.0, nu=0.3)
    A = fem.create_matrix(a)
    fem.assemble_matrix(a, A=A, check=True)
    r = 11
    b0 = int(A.indptr[r])
    keep = A.indices[b0:b0 + 2].clone()
    try:
        A.indices[b0], A.indices[b0 + 1] = keep[1], keep[0]
        with pytest.raises(_lib.FemasmError, match="pattern check failed"):
            fem.assemble_matrix(a, A=A, check=True)
    finally:
        A.indices[b0:b0 + 2] = keep
