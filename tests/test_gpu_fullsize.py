"""Full-size parity (BASELINE.json configs at their real sizes): sampled rows of the GPU matrix
against the CPU oracle assembling exactly the cells adjacent to those rows (so the sampled rows
are complete), plus size-independent properties. Config E on one GPU allocates ~170 GB."""
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


def sampled_row_parity(oracle, V, a, A, marker, nsample=2000, seed=0):
    """Max relative error over `nsample` random rows (relative to the global max |A| of the sample)."""
    m = V.mesh
    g = torch.Generator(device="cpu").manual_seed(seed)
    rows = torch.randint(0, V.num_nodes, (nsample,), generator=g).unique()
    ptr, idx = V.adjacency()
    ptr_h = ptr.cpu()
    segs = [idx[int(ptr_h[r]):int(ptr_h[r + 1])] for r in rows.tolist()]
    cells = torch.unique(torch.cat(segs).to(torch.int64) // V.nn)
    sub_nodes_glob = V.dofmap[cells].to(torch.int64)
    uniq, inv = torch.unique(sub_nodes_glob.reshape(-1), return_inverse=True)
    sub_cells = inv.reshape(sub_nodes_glob.shape).to(torch.int32).cpu().numpy()
    sub_geom_glob = m.cells[cells].to(torch.int64)
    vuniq, vinv = torch.unique(sub_geom_glob.reshape(-1), return_inverse=True)
    sub_geom = vinv.reshape(sub_geom_glob.shape).to(torch.int32).cpu().numpy()
    sub_x = m.x[vuniq].cpu().numpy()
    E = a.E[cells].cpu().numpy()
    lam, mu = oracle.lame(E, a.nu)
    bs = V.bs
    bc = None
    if marker is not None:
        dofs = (uniq[:, None] * bs + torch.arange(bs, device=uniq.device)[None, :]).reshape(-1)
        bc = marker[dofs].cpu().numpy()
    uniq_h = uniq.cpu().numpy()
    ip, ix = oracle.sparsity(sub_cells, len(uniq_h))
    vals = oracle.assemble_elasticity(int(m.cell_type), V.degree, sub_cells, sub_geom, sub_x, lam, mu, ip, ix, bc=bc,
                                      diag=1.0, qdeg=a.qdeg)
    loc = {int(gn): k for k, gn in enumerate(uniq_h)}
    gcols, gvals = A.row_blocks(rows.tolist())
    scale, err = 0.0, 0.0
    for r, gc, gv in zip(rows.tolist(), gcols, gvals):
        lr = loc[r]
        oc = uniq_h[ix[ip[lr]:ip[lr + 1]]]
        ov = vals[ip[lr]:ip[lr + 1]]
        assert np.array_equal(gc, oc), f"row {r}: pattern mismatch"
        scale = max(scale, float(np.abs(ov).max()))
        err = max(err, float(np.abs(gv - ov).max()))
    return err / scale, len(rows)


@pytest.mark.parametrize("n", [203])
def test_config_e_p2_tet_full_size(oracle, dev, n):
    """Config E mesh (203^3 x 6 = 50.2 M P2 tets, 202 M dofs) with the reference bcs."""
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
    fem.assemble_matrix(a, bcs=bcs, A=A)
    torch.cuda.synchronize()
    marker, _ = fem._combine_bcs(V, bcs)
    rel, nrows = sampled_row_parity(oracle, V, a, A, marker, nsample=1500)
    assert rel <= RTOL, f"sampled-row parity {rel:.2e} over {nrows} rows"
    # values are finite everywhere
    for _, _, d in A.parts:
        flat = d.reshape(-1)
        for k in range(0, flat.numel(), 1 << 28):
            assert bool(torch.isfinite(flat[k:k + (1 << 28)]).all())
