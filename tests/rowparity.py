"""Row-wise parity helpers for the GPU tests (test infrastructure: compares the HIP path with the
CPU oracle; never imported by the product package).

Bar (BASELINE.json north_star "global CSR entries match ... to 1e-12 relative"), applied per
scalar matrix row: for every row i, max_j |A_gpu[i, j] - A_ref[i, j]| <= 1e-12 * max_j |A_ref[i, j]|,
with identical sparsity patterns. A row of a soft cell (E spans 5e6 .. 1e8, a 20x range) is held to
its own scale, not to the largest entry of the matrix.
"""
from __future__ import annotations

import numpy as np
import torch

RTOL = 1e-12


def row_errors(got: np.ndarray, ref: np.ndarray, indptr: np.ndarray) -> tuple[float, int]:
    """Worst per-row relative error of BSR values [nb, bs, bs] sharing the pattern `indptr`.
    Returns (max over scalar rows of err_row / scale_row, index of that block row)."""
    bs = ref.shape[1]
    nrows = indptr.shape[0] - 1
    rows = np.repeat(np.arange(nrows), np.diff(indptr))
    d = np.abs(got - ref).max(axis=2)  # [nb, bs]: per block and scalar row i, max over columns
    s = np.abs(ref).max(axis=2)
    err = np.zeros((nrows, bs))
    scale = np.zeros((nrows, bs))
    np.maximum.at(err, rows, d)
    np.maximum.at(scale, rows, s)
    zero = scale == 0.0
    if np.any(err[zero] > 0.0):  # an all-zero reference row must be reproduced exactly
        r = int(np.argwhere(zero & (err > 0.0))[0][0])
        return float("inf"), r
    rel = np.where(zero, 0.0, err / np.where(zero, 1.0, scale))
    k = int(np.argmax(rel))
    return float(rel.reshape(-1)[k]), k // bs


def assert_rows_close(got: np.ndarray, ref: np.ndarray, indptr: np.ndarray, rtol: float = RTOL, what: str = ""):
    rel, r = row_errors(got, ref, indptr)
    assert rel <= rtol, f"{what} per-row parity {rel:.3e} > {rtol:g} (block row {r})"
    return rel


def submesh_of_rows(V, rows: torch.Tensor):
    """The cells adjacent to `rows` (node indices of V) renumbered into a self-contained sub-mesh.
    Assembling that sub-mesh gives those rows complete. Returns (cells [sub], node ids, sub dofmap,
    sub geometry dofmap, sub coordinates)."""
    m = V.mesh
    ptr, idx = V.adjacency()
    ptr_h = ptr.cpu()
    segs = [idx[int(ptr_h[r]):int(ptr_h[r + 1])] for r in rows.tolist()]
    cells = torch.unique(torch.cat(segs).to(torch.int64) // V.nn)
    glob = V.dofmap[cells].to(torch.int64)
    uniq, inv = torch.unique(glob.reshape(-1), return_inverse=True)
    sub_cells = inv.reshape(glob.shape).to(torch.int32).cpu().numpy()
    gv = m.cells[cells].to(torch.int64)
    vuniq, vinv = torch.unique(gv.reshape(-1), return_inverse=True)
    sub_geom = vinv.reshape(gv.shape).to(torch.int32).cpu().numpy()
    sub_x = m.x[vuniq].cpu().numpy()
    return cells, uniq, sub_cells, sub_geom, sub_x


def sample_rows(V, nsample: int, seed: int = 0, extra=()) -> torch.Tensor:
    """Random block rows plus the first / last rows and any `extra` rows (unique, sorted)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    rows = torch.randint(0, V.num_nodes, (nsample,), generator=g)
    fixed = torch.tensor([0, V.num_nodes - 1, *extra], dtype=torch.int64)
    return torch.unique(torch.cat([rows, fixed]))


def sampled_row_parity(oracle, V, a, A, marker, nsample=1500, seed=0, extra=(), kind="linear"):
    """Per-row parity of `nsample` random rows of the GPU matrix A against the oracle assembling
    exactly the cells adjacent to those rows (kind: "linear" elasticity or "neo" Hookean at the
    form's state u). Patterns must match row by row. Returns (worst per-row relative error, rows)."""
    m = V.mesh
    rows = sample_rows(V, nsample, seed, extra)
    cells, uniq, sub_cells, sub_geom, sub_x = submesh_of_rows(V, rows)
    if a.E is not None:
        lam, mu = oracle.lame(a.E[cells].cpu().numpy(), a.nu)
    else:
        lam, mu = a.lam[cells].cpu().numpy(), a.mu[cells].cpu().numpy()
    bs = V.bs
    dofs = (uniq[:, None] * bs + torch.arange(bs, device=uniq.device)[None, :]).reshape(-1)
    bc = None if marker is None else marker[dofs].cpu().numpy()
    uniq_h = uniq.cpu().numpy()
    ip, ix = oracle.sparsity(sub_cells, len(uniq_h))
    if kind == "neo":
        u = a.u[dofs].cpu().numpy()
        vals = oracle.assemble_neohookean(int(m.cell_type), V.degree, sub_cells, sub_geom, sub_x, lam, mu, u, ip, ix,
                                          bc=bc, diag=1.0, qdeg=a.qdeg)
    else:
        vals = oracle.assemble_elasticity(int(m.cell_type), V.degree, sub_cells, sub_geom, sub_x, lam, mu, ip, ix,
                                          bc=bc, diag=1.0, qdeg=a.qdeg)
    loc = {int(gn): k for k, gn in enumerate(uniq_h)}
    gcols, gvals = A.row_blocks(rows.tolist())
    got, ref, ptr = [], [], [0]
    for r, gc, gv in zip(rows.tolist(), gcols, gvals):
        lr = loc[r]
        oc = uniq_h[ix[ip[lr]:ip[lr + 1]]]
        assert np.array_equal(gc, oc), f"row {r}: pattern mismatch"
        got.append(gv)
        ref.append(vals[ip[lr]:ip[lr + 1]])
        ptr.append(ptr[-1] + len(gc))
    rel, _ = row_errors(np.concatenate(got), np.concatenate(ref), np.array(ptr))
    return rel, len(rows)
