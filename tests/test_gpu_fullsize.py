"""Full-size parity of the headline workload (config E's mesh, linear-elasticity J): sampled rows
of the GPU matrix against the CPU oracle assembling exactly the cells adjacent to those rows (so
the sampled rows are complete), per-row 1e-12 bar (tests/rowparity.py), plus size-independent
properties. Config E on one GPU allocates ~170 GB. The other configs: tests/test_gpu_configs.py."""
import pytest
import torch

from rowparity import sampled_row_parity

pytestmark = pytest.mark.gpu
RTOL = 1e-12


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("owner", [False, True], ids=["lds-atomic", "block-owner"])
@pytest.mark.parametrize("n", [203])
def test_config_e_p2_tet_full_size(oracle, dev, n, owner):
    """Config E mesh (203^3 x 6 = 50.2 M P2 tets, 202 M dofs) with the reference bcs, through the
    default LDS-atomic gather and through the block-owner gather (owner=True: ~4.9 M chunks of the
    contribution plan at full size)."""
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
    assert A.num_block_rows == (2 * n + 1) ** 3
    assert int(A.indptr[-1]) == A.num_blocks and bool((A.indptr[1:] >= A.indptr[:-1]).all())
    fem.assemble_matrix(a, bcs=bcs, A=A, plan=dict(owner=owner))
    torch.cuda.synchronize()
    marker, _ = fem._combine_bcs(V, bcs)
    rel, nrows = sampled_row_parity(oracle, V, a, A, marker, nsample=1500)
    assert rel <= RTOL, f"sampled-row parity {rel:.2e} over {nrows} rows"
    # values are finite everywhere
    for _, _, d in A.parts:
        flat = d.reshape(-1)
        for k in range(0, flat.numel(), 1 << 28):
            assert bool(torch.isfinite(flat[k:k + (1 << 28)]).all())
