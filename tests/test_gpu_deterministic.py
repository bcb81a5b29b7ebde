"""Deterministic assembly mode (FA_DETERMINISTIC, SURVEY.md §5: a fixed-order mode whose values
are bit-identical run to run). The gather then sums every block in exact 64-bit fixed point, so
repeated assemblies must be torch.equal; the values must meet the per-row 1e-12 bar against the
CPU oracle and against the default (FP64-atomic, order-dependent) gather."""
import numpy as np
import pytest
import torch

from rowparity import RTOL, assert_rows_close, sampled_row_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _problem(oracle, ct, p, n, dev):
    from femasm import fem, mesh

    m = mesh.create_unit_square(*n, cell_type=ct, device=dev) if len(n) == 2 else \
        mesh.create_unit_cube(*n, cell_type=ct, device=dev)
    V = fem.functionspace(m, ("Lagrange", p, (m.gdim,)))
    E = torch.tensor(oracle.e_range()[np.arange(m.num_cells) % 200], dtype=torch.float64, device=dev)
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    vr = [0.01] + [0.0] * (m.gdim - 1)
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc(vr, right, V)]
    return m, V, a, bcs


def _oracle(oracle, V, a, bcs):
    from femasm import fem

    m = V.mesh
    marker, _ = fem._combine_bcs(V, bcs)
    cells = V.dofmap.cpu().numpy()
    ip, ix = oracle.sparsity(cells, V.num_nodes)
    lam, mu = oracle.lame(a.E.cpu().numpy(), a.nu)
    return oracle.assemble_elasticity(int(m.cell_type), V.degree, cells, m.cells.cpu().numpy(), m.x.cpu().numpy(),
                                      lam, mu, ip, ix, bc=marker.cpu().numpy(), diag=1.0)


# P1 / P2 tetrahedra (configs C, E) and triangles (config A), each with many chunks; affine Q1 / Q2
# quadrilaterals (config B's element) and Q1 hexahedra run the same gather since round 6
CASES = [(-4, 2, (12, 11, 10)), (-4, 1, (24, 23, 22)), (3, 1, (71, 71)), (3, 2, (40, 37)), (4, 2, (41, 37)),
         (4, 1, (63, 60)), (8, 1, (17, 16, 15))]


@pytest.mark.parametrize("ct,p,n", CASES)
def test_repeated_assemblies_bit_identical(oracle, dev, ct, p, n):
    from femasm import fem

    m, V, a, bcs = _problem(oracle, ct, p, n, dev)
    A = fem.create_matrix(a)
    runs = []
    for _ in range(3):
        A.data.fill_(float("nan"))  # nothing may survive from a previous run
        fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=True)
        runs.append(A.data.clone())
    assert torch.equal(runs[0], runs[1]) and torch.equal(runs[0], runs[2])
    # the same values from a fresh matrix and a fresh plan
    V.__dict__.pop("_plans", None)
    A2 = fem.assemble_matrix(a, bcs=bcs, deterministic=True)
    assert torch.equal(A2.data, runs[0])


@pytest.mark.parametrize("ct,p,n", CASES)
def test_deterministic_vs_oracle_and_default(oracle, dev, ct, p, n):
    from femasm import fem

    m, V, a, bcs = _problem(oracle, ct, p, n, dev)
    Ad = fem.assemble_matrix(a, bcs=bcs, deterministic=True)
    A0 = fem.assemble_matrix(a, bcs=bcs)
    ip = Ad.indptr.cpu().numpy()
    ref = _oracle(oracle, V, a, bcs)
    assert_rows_close(Ad.data.cpu().numpy(), ref, ip, RTOL, "deterministic vs oracle:")
    assert_rows_close(Ad.data.cpu().numpy(), A0.data.cpu().numpy(), ip, RTOL, "deterministic vs default:")


def test_deterministic_row_parts(oracle, dev):
    """Values split into many row parts (one plan per part)."""
    from femasm import fem

    m, V, a, bcs = _problem(oracle, -4, 2, (4, 3, 3), dev)
    A = fem.create_matrix(a, max_part_bytes=8192)
    assert len(A.parts) > 3
    fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=True)
    first = A.data.clone()
    fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=True)
    assert torch.equal(A.data, first)
    assert_rows_close(first.cpu().numpy(), _oracle(oracle, V, a, bcs), A.indptr.cpu().numpy(), RTOL)


def test_deterministic_split_gather(oracle, dev):
    """fa_gather_rows honours FA_PLAN_DETERMINISTIC (the slab path's split gather)."""
    from femasm import fem

    m, V, a, bcs = _problem(oracle, -4, 2, (6, 5, 4), dev)
    A = fem.create_matrix(a)
    nr = A.num_block_rows
    cuts = [0, nr // 3, nr // 3 + 7, nr]
    sg = fem.SplitGather(a, bcs, A, list(zip(cuts[:-1], cuts[1:])), deterministic=True)
    outs = []
    for _ in range(2):
        A.data.fill_(float("nan"))
        sg.prepare()
        for i in (2, 0, 1):
            sg.rows(i)
        outs.append(A.data.clone())
    assert torch.equal(outs[0], outs[1])
    assert_rows_close(outs[0].cpu().numpy(), _oracle(oracle, V, a, bcs), A.indptr.cpu().numpy(), RTOL)


def test_deterministic_unsupported_form_fails_loudly(oracle, dev):
    from femasm import _lib, fem, mesh

    m = mesh.create_unit_cube(2, 2, 2, cell_type=mesh.CellType.hexahedron, device=dev)
    m.x = m.x + 0.01 * torch.sin(7.0 * m.x)  # non-affine hexahedra: the MFMA element path
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    a = fem.LinearElasticity(V, E=1.0, nu=0.3)
    with pytest.raises(_lib.FemasmError, match="deterministic"):
        fem.assemble_matrix(a, deterministic=True)


@pytest.mark.parametrize("n", [203])
def test_config_e_deterministic_full_size(oracle, dev, n):
    """Config E (50.2 M P2 tets) in deterministic mode: two assemblies bit-identical, sampled rows
    against the oracle at the per-row bar."""
    from femasm import fem, mesh
    from femasm.materials import e_range

    m = mesh.create_unit_cube(n, n, n, mesh.CellType.tetrahedron, device=dev)
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    E = torch.tensor(e_range(), device=dev)[torch.arange(m.num_cells, device=dev) % 200]
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0.0, 0.0], right, V)]
    A = fem.create_matrix(a)
    fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=True)
    torch.cuda.synchronize()
    # a position-weighted checksum of the value bits (the 139 GB cannot be copied aside on one GPU)
    def sums():
        out, step = [], 1 << 26
        w = torch.arange(step, device=dev, dtype=torch.int64).remainder(251) + 1
        for _, _, d in A.parts:
            flat = d.reshape(-1).view(torch.int64)
            tot = 0
            for k in range(0, flat.numel(), step):
                x = flat[k:k + step]
                tot += int((x.remainder(1_000_003) * w[:x.numel()]).sum().item())
            out.append(tot)
        return out
    s1 = sums()
    fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=True)
    torch.cuda.synchronize()
    assert sums() == s1
    marker, _ = fem._combine_bcs(V, bcs)
    rel, nrows = sampled_row_parity(oracle, V, a, A, marker, nsample=1500)
    assert rel <= RTOL, f"sampled-row parity {rel:.2e} over {nrows} rows"


@pytest.mark.parametrize("contrast", [1e2, 1e4, 1e8])
def test_deterministic_high_contrast(oracle, dev, contrast):
    """A stiffness jump inside the chunks (E = 1 for x < 0.45, `contrast` beyond): rows of soft cells
    share chunks with rows of stiff cells. The fixed-point scale is per block (set by the cells adding
    into it, which all hold the block's row node), so every row meets the per-row 1e-12 bar at any
    contrast, as the default (FP64-atomic) gather does. (Rounds 4-5 used one scale per chunk: 6.8e-12
    at a contrast of 100.) Two deterministic runs are bit-identical."""
    from femasm import fem

    m, V, a, bcs = _problem(oracle, -4, 2, (12, 11, 10), dev)
    xc = m.x[m.cells.to(torch.int64)].mean(1)[:, 0]
    a.E = torch.where(xc < 0.45, torch.ones_like(xc), torch.full_like(xc, contrast)).contiguous()
    ref = _oracle(oracle, V, a, bcs)
    A = fem.assemble_matrix(a, bcs=bcs, deterministic=True)
    d1 = A.data.clone()
    A.data.fill_(float("nan"))
    fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=True)
    assert torch.equal(d1, A.data)
    B = fem.assemble_matrix(a, bcs=bcs)
    ip = A.indptr.cpu().numpy()
    assert_rows_close(B.data.cpu().numpy(), ref, ip, RTOL)  # the default gather
    assert_rows_close(A.data.cpu().numpy(), ref, ip, RTOL)


@pytest.mark.parametrize("contrast", [1e4])
def test_deterministic_high_contrast_p1(oracle, dev, contrast):
    """The same on P1 tetrahedra (the fused-records k_gather_lin)."""
    from femasm import fem

    m, V, a, bcs = _problem(oracle, -4, 1, (24, 23, 22), dev)
    xc = m.x[m.cells.to(torch.int64)].mean(1)[:, 0]
    a.E = torch.where(xc < 0.45, torch.ones_like(xc), torch.full_like(xc, contrast)).contiguous()
    ref = _oracle(oracle, V, a, bcs)
    A = fem.assemble_matrix(a, bcs=bcs, deterministic=True)
    assert_rows_close(A.data.cpu().numpy(), ref, A.indptr.cpu().numpy(), RTOL)


@pytest.mark.parametrize("ct,p,n", [(-4, 2, (12, 11, 10)), (4, 2, (41, 37)), (-4, 1, (24, 23, 22))])
def test_cached_chunk_arrays(oracle, dev, ct, p, n):
    """The plan's chunk arrays built once (fa_plan_chunk_desc, round 6) give the same bits as arrays
    rebuilt at the launch (plan.chunk_desc = NULL), in every visiting order."""
    from femasm import fem

    m, V, a, bcs = _problem(oracle, ct, p, n, dev)
    A = fem.create_matrix(a)
    for loc in ("row", "morton", "deal"):
        plan = fem.gather_plan(V, A, 0, a.kind, deterministic=True, locality=loc)
        assert plan.chunk_desc, "gather_plan builds the chunk arrays"
        fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=True, plan={"locality": loc})
        cached = A.data.clone()
        keep = plan.chunk_desc
        plan.chunk_desc = None
        A.data.fill_(float("nan"))
        fem.assemble_matrix(a, bcs=bcs, A=A, deterministic=True, plan={"locality": loc})
        plan.chunk_desc = keep
        assert torch.equal(A.data, cached), loc
