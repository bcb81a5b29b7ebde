"""GPU: the uniform-nu affine-simplex gather (MAT_LINU: records s*Ji with s^2 = mu|J|, table
B = (lam/mu) Ahat + Ahat^T) against the CPU oracle, next to the general lam/mu kernel it replaces
for E-per-cell forms: forms given as lam/mu arrays, and cells with E < 0 (the
record's sign path). Bar as test_gpu_parity: |A - A_oracle|_max <= 1e-12 |A_oracle|_max."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
RTOL = 1e-12
CASES = [("tetrahedron", 2, 4), ("tetrahedron", 1, 6), ("triangle", 2, 8), ("triangle", 1, 10)]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _run(dev, oracle, ct_name, p, n, E_fn, use_lame, nu=0.3):
    from femasm import fem, mesh

    ct = mesh.CellType[ct_name]
    m = mesh.create_unit_cube(n, n, n, cell_type=ct, device=dev) if ct == mesh.CellType.tetrahedron \
        else mesh.create_unit_square(n, n, cell_type=ct, device=dev)
    gd = m.gdim
    V = fem.functionspace(m, ("Lagrange", p, (gd,)))
    E = E_fn(m.num_cells)
    lam, mu = oracle.lame(E, nu)
    if use_lame:
        a = fem.LinearElasticity(V, lam=torch.tensor(lam, device=dev), mu=torch.tensor(mu, device=dev))
    else:
        a = fem.LinearElasticity(V, E=torch.tensor(E, device=dev), nu=nu)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01] + [0.0] * (gd - 1), right, V)]
    A = fem.assemble_matrix(a, bcs=bcs)
    torch.cuda.synchronize()
    marker, _ = fem._combine_bcs(V, bcs)
    cells = V.dofmap.cpu().numpy()
    indptr, indices = oracle.sparsity(cells, V.num_nodes)
    ref = oracle.assemble_elasticity(int(ct), p, cells, m.cells.cpu().numpy(), m.x.cpu().numpy(), lam, mu, indptr,
                                     indices, bc=marker.cpu().numpy(), diag=1.0)
    assert np.array_equal(A.indices.cpu().numpy(), indices)
    err = np.abs(A.data.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= RTOL, err


@pytest.mark.parametrize("ct,p,n", CASES)
def test_uniform_nu_kernel(dev, oracle, ct, p, n):
    """E per cell with one nu: the uniform-nu kernels (the general lam / mu kernel: test_lame_arrays)."""
    _run(dev, oracle, ct, p, n, lambda nc: oracle.e_range()[np.arange(nc) % 200], use_lame=False)


@pytest.mark.parametrize("ct,p,n", CASES)
def test_lame_arrays(dev, oracle, ct, p, n):
    _run(dev, oracle, ct, p, n, lambda nc: oracle.e_range()[np.arange(nc) % 200], use_lame=True)


@pytest.mark.parametrize("ct,p,n", CASES[:2])
def test_negative_stiffness_cells(dev, oracle, ct, p, n):
    def E_fn(nc):
        E = oracle.e_range()[np.arange(nc) % 200].copy()
        E[::7] *= -1.0  # nonphysical, but the record's sign must carry it
        return E

    _run(dev, oracle, ct, p, n, E_fn, use_lame=False)
