"""Global sparse matrix in torch tensors — the dolfinx.la.MatrixCSR / PETSc BAIJ role.

Storage is block CSR with block size bs = gdim (dolfinx's blocked dofmap: dof = node*bs + comp):
``indptr`` int64 [nrows+1], ``indices`` int32 [nblocks] sorted per row, ``data`` float64
[nblocks, bs, bs] row-major blocks. For config E (202 M dofs) this keeps the index arrays at
7.7 GB instead of 69 GB for scalar CSR (SURVEY.md §7 "Memory").
"""
from __future__ import annotations

import numpy as np
import torch


class MatrixCSR:
    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor, bs: int, data: torch.Tensor | None = None):
        self.indptr = indptr
        self.indices = indices
        self.bs = int(bs)
        if data is None:
            data = torch.zeros((indices.shape[0], bs, bs), dtype=torch.float64, device=indices.device)
        self.data = data

    @property
    def num_block_rows(self) -> int:
        return int(self.indptr.shape[0] - 1)

    @property
    def num_blocks(self) -> int:
        return int(self.indices.shape[0])

    @property
    def shape(self):
        n = self.num_block_rows * self.bs
        return (n, n)

    @property
    def nnz(self) -> int:
        return self.num_blocks * self.bs * self.bs

    def zero(self):
        self.data.zero_()

    def to_scipy(self):
        """scipy.sparse.bsr_matrix on the host (test / debug helper)."""
        import scipy.sparse as sp

        return sp.bsr_matrix(
            (self.data.detach().cpu().numpy(), self.indices.cpu().numpy(), self.indptr.cpu().numpy()),
            shape=self.shape)

    def to_dense(self) -> np.ndarray:
        return self.to_scipy().toarray()

    def diagonal_block_slots(self) -> torch.Tensor:
        """Slot index of the diagonal block of every row (-1 if absent)."""
        rows = torch.repeat_interleave(torch.arange(self.num_block_rows, device=self.indices.device),
                                       self.indptr[1:] - self.indptr[:-1])
        hit = rows == self.indices.to(torch.int64)
        out = torch.full((self.num_block_rows,), -1, dtype=torch.int64, device=self.indices.device)
        out[rows[hit]] = torch.nonzero(hit).reshape(-1)
        return out

    def mult(self, x: torch.Tensor) -> torch.Tensor:
        """y = A x for a dof vector x [nrows*bs] (torch ops; used by the Newton driver)."""
        bs = self.bs
        xb = x.reshape(-1, bs)
        rows = torch.repeat_interleave(torch.arange(self.num_block_rows, device=x.device),
                                       self.indptr[1:] - self.indptr[:-1])
        contrib = torch.bmm(self.data, xb[self.indices.to(torch.int64)].unsqueeze(-1)).squeeze(-1)
        y = torch.zeros_like(xb)
        y.index_add_(0, rows, contrib)
        return y.reshape(-1)
