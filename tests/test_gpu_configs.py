"""Parity at every BASELINE.json configuration's own size, per-row bar (tests/rowparity.py).

  A  71 x 71 x 2 P1 triangles (reference J at d = 0, quadrature degree 1, reference bcs): the whole
     matrix against the committed fixture tests/golden/config_a_p1_elasticity.npz (oracle output,
     tests/golden/make_golden.py) -- identical pattern, every row within 1e-12.
  B  1000 x 1000 Q2 quadrilaterals, C 119^3 x 6 P1 tetrahedra, D 58^3 Q3 hexahedra (affine tensor
  gather) and the same with interior vertices moved (non-affine: the MFMA element path), D' 58^3 Q2
  hexahedra, E 203^3 x 6 P2 tetrahedra with the neo-Hookean AD tangent: sampled rows of
     the GPU matrix against the oracle assembling exactly the cells adjacent to those rows.
  (Config E with the linear form at full size: tests/test_gpu_fullsize.py.)

Material and bcs as the reference (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:533-545,
:620-669): E = E_range[cell % 200], nu = 0.3, x = 0 clamped, x = 1 prescribed.
"""
import os

import numpy as np
import pytest
import torch

from rowparity import RTOL, assert_rows_close, sampled_row_parity

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _free_memory():
    yield
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def _problem(ct, degree, n, dev, form="linear", qdeg=None, perturb=0.0):
    from femasm import fem, mesh
    from femasm.materials import e_range

    ct = mesh.CellType[ct]
    if mesh.GDIM[ct] == 2:
        m = mesh.create_unit_square(n, n, cell_type=ct, device=dev)
    else:
        m = mesh.create_unit_cube(n, n, n, cell_type=ct, device=dev)
    if perturb:  # interior vertices moved (as bench.py --config Dmfma): non-affine trilinear cells
        x = m.x
        s = torch.sin(torch.pi * x).prod(dim=1, keepdim=True)
        shift = torch.stack([torch.sin(2 * torch.pi * x[:, 0]), torch.cos(2 * torch.pi * x[:, 1]),
                             torch.sin(2 * torch.pi * x[:, 2] + 0.5)], dim=1)
        x += perturb / n * s * shift
    gd = m.gdim
    V = fem.functionspace(m, ("Lagrange", degree, (gd,)))
    E = torch.tensor(e_range(), dtype=torch.float64, device=dev)[torch.arange(m.num_cells, device=dev) % 200]
    if form == "neo":
        u = (1e-3 * torch.sin(torch.pi * V.tabulate_dof_coordinates())).reshape(-1).contiguous()
        a = fem.NeoHookean(V, E=E, nu=0.3, u=u, quadrature_degree=qdeg)
    else:
        a = fem.LinearElasticity(V, E=E, nu=0.3, quadrature_degree=qdeg)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01] + [0.0] * (gd - 1), right, V)]
    return m, V, a, bcs


def test_config_a_against_golden_fixture(dev):
    """Config A as the reference's mechanic2d J at d = 0 (P1 triangles, `dxx` degree 1)."""
    from femasm import fem

    m, V, a, bcs = _problem("triangle", 1, 71, dev, qdeg=1)
    assert m.num_cells == 10082 and V.num_dofs == 10368
    gold = np.load(os.path.join(GOLDEN, "config_a_p1_elasticity.npz"))
    marker, g = fem._combine_bcs(V, bcs)
    np.testing.assert_array_equal(marker.cpu().numpy(), gold["bc"])
    np.testing.assert_array_equal(g.cpu().numpy(), gold["g"])
    for method in ("gather", "scatter"):
        A = fem.assemble_matrix(a, bcs=bcs, method=method)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(A.indptr.cpu().numpy(), gold["indptr"])
        np.testing.assert_array_equal(A.indices.cpu().numpy(), gold["indices"])
        assert_rows_close(A.data.cpu().numpy(), gold["data"], gold["indptr"], what=f"config A ({method})")


CONFIGS = [
    # id, cell, degree, n, rows sampled, vertex perturbation (0: affine cells)
    ("B", "quadrilateral", 2, 1000, 1500, 0.0),
    ("C", "tetrahedron", 1, 119, 1500, 0.0),
    ("Dq2", "hexahedron", 2, 58, 400, 0.0),
    ("D", "hexahedron", 3, 58, 150, 0.0),
    ("Dmfma", "hexahedron", 3, 58, 100, 0.2),  # non-affine: MFMA element kernel + block gather
]


@pytest.mark.parametrize("cfg,ct,degree,n,nsample,perturb", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_config_full_size(oracle, dev, cfg, ct, degree, n, nsample, perturb):
    from femasm import fem

    m, V, a, bcs = _problem(ct, degree, n, dev, perturb=perturb)
    A = fem.create_matrix(a)
    assert int(A.indptr[-1]) == A.num_blocks
    fem.assemble_matrix(a, bcs=bcs, A=A)
    torch.cuda.synchronize()
    if ct == "hexahedron":  # the plan's affinity test picks the kernel: affine tensor gather or MFMA
        from femasm import _lib
        plan = fem.gather_plan(V, A, 0)
        assert bool(plan.cell_flags & _lib.FA_PLAN_AFFINE) == (perturb == 0.0)
    marker, _ = fem._combine_bcs(V, bcs)
    # rows on both bc planes and a chunk of consecutive rows are always in the sample
    x = V.tabulate_dof_coordinates()
    on_left = torch.nonzero(x[:, 0] == 0.0).flatten()[:8].cpu().tolist()
    on_right = torch.nonzero(x[:, 0] == 1.0).flatten()[-8:].cpu().tolist()
    mid = V.num_nodes // 2
    extra = on_left + on_right + list(range(mid, mid + 40))
    rel, nrows = sampled_row_parity(oracle, V, a, A, marker, nsample=nsample, extra=extra)
    assert rel <= RTOL, f"config {cfg}: per-row parity {rel:.2e} over {nrows} rows"
    for _, _, d in A.parts:
        flat = d.reshape(-1)
        for k in range(0, flat.numel(), 1 << 28):
            assert bool(torch.isfinite(flat[k:k + (1 << 28)]).all())


def test_config_e_neo_hookean_full_size(oracle, dev):
    """Config E physics: 203^3 x 6 P2 tetrahedra, neo-Hookean tangent by device AD at
    u = 1e-3 sin(pi x), quadrature degree 2, against the oracle's closed-form tangent."""
    from femasm import fem

    m, V, a, bcs = _problem("tetrahedron", 2, 203, dev, form="neo", qdeg=2)
    assert m.num_cells == 50_192_562
    A = fem.create_matrix(a)
    fem.assemble_matrix(a, bcs=bcs, A=A)
    torch.cuda.synchronize()
    marker, _ = fem._combine_bcs(V, bcs)
    rel, nrows = sampled_row_parity(oracle, V, a, A, marker, nsample=800, kind="neo")
    assert rel <= RTOL, f"config E neo-Hookean: per-row parity {rel:.2e} over {nrows} rows"
