"""Global sparse matrix in torch tensors — the dolfinx.la.MatrixCSR / PETSc BAIJ role.

Storage is block CSR with block size bs = gdim (dolfinx's blocked dofmap: dof = node*bs + comp):
``indptr`` int64 [nrows+1], ``indices`` int32 [nblocks] sorted per row, ``data`` float64
[nblocks, bs, bs] row-major blocks. For config E (202 M dofs) this keeps the index arrays at
7.7 GB instead of 69 GB for scalar CSR (SURVEY.md §7 "Memory").
"""
from __future__ import annotations

import numpy as np
import torch


# Largest single values allocation by default (create_matrix(max_part_bytes=...) sets another);
# larger matrices are split into row parts (each assembled through the fa_bsr row window).
# Config E (138 GB) fits one part on a 288 GB MI355X.
MAX_PART_BYTES = 200 * (1 << 30)


class MatrixCSR:
    """Block-CSR matrix; values may be split into row parts (each its own allocation).

    ``parts``: list of (row_begin, row_end, data[indptr[row_end]-indptr[row_begin], bs, bs]).
    """

    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor, bs: int, data: torch.Tensor | None = None,
                 max_part_bytes: int = MAX_PART_BYTES, window: tuple | None = None):
        self.indptr = indptr
        self.indices = indices
        self.bs = int(bs)
        nrows = int(indptr.shape[0] - 1)
        if data is not None:
            self.parts = [(0, nrows, data)]
            return
        if window is not None:  # only rows [r0, r1) are held (a rank's rows)
            r0, r1 = int(window[0]), int(window[1])
            n = int(indptr[r1]) - int(indptr[r0])
            self.parts = [(r0, r1, torch.zeros((n, self.bs, self.bs), dtype=torch.float64, device=indices.device))]
            return
        block_bytes = 8 * self.bs * self.bs
        nb = int(indices.shape[0])
        cap = max(1, max_part_bytes // block_bytes)
        bounds = [0]
        if nb > cap:
            targets = torch.arange(cap, nb, cap, device=indptr.device, dtype=torch.int64)
            cuts = torch.searchsorted(indptr, targets, right=True) - 1
            bounds += sorted({int(c) for c in cuts.cpu().tolist() if 0 < int(c) < nrows})
        bounds.append(nrows)
        self.parts = []
        for r0, r1 in zip(bounds[:-1], bounds[1:]):
            n = int(indptr[r1]) - int(indptr[r0])
            self.parts.append((r0, r1, torch.zeros((n, self.bs, self.bs), dtype=torch.float64, device=indices.device)))

    @property
    def data(self) -> torch.Tensor:
        """All values [nblocks, bs, bs] (a concatenated copy when the matrix has several parts)."""
        if len(self.parts) == 1:
            return self.parts[0][2]
        return torch.cat([p[2] for p in self.parts])

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
        for _, _, d in self.parts:
            d.zero_()

    def to_scipy(self):
        """scipy.sparse.bsr_matrix on the host (test / debug helper)."""
        import scipy.sparse as sp

        return sp.bsr_matrix(
            (self.data.detach().cpu().numpy(), self.indices.cpu().numpy(), self.indptr.cpu().numpy()),
            shape=self.shape)

    def to_dense(self) -> np.ndarray:
        return self.to_scipy().toarray()

    def row_blocks(self, rows) -> tuple[list, list]:
        """Column indices and value blocks of the given block rows (host numpy), across parts."""
        ip = self.indptr
        out_c, out_v = [], []
        for r in rows:
            r = int(r)
            for r0, r1, d in self.parts:
                if r0 <= r < r1:
                    b, e = int(ip[r]), int(ip[r + 1])
                    base = int(ip[r0])
                    out_c.append(self.indices[b:e].cpu().numpy())
                    out_v.append(d[b - base:e - base].cpu().numpy())
                    break
        return out_c, out_v

    def diagonal_block_slots(self) -> torch.Tensor:
        """Slot index of the diagonal block of every row (-1 if absent)."""
        rows = torch.repeat_interleave(torch.arange(self.num_block_rows, device=self.indices.device),
                                       self.indptr[1:] - self.indptr[:-1])
        hit = rows == self.indices.to(torch.int64)
        out = torch.full((self.num_block_rows,), -1, dtype=torch.int64, device=self.indices.device)
        out[rows[hit]] = torch.nonzero(hit).reshape(-1)
        return out

    def _fa_bsr(self, part: int = 0):
        """The C-ABI view (fa_bsr) of one row part."""
        from . import _lib

        r0, r1, data = self.parts[part]
        b = _lib.fa_bsr()
        b.nrows = self.num_block_rows
        b.bs = self.bs
        b.nblocks = self.num_blocks
        b.indptr = self.indptr.data_ptr()
        b.indices = self.indices.data_ptr()
        b.data = data.data_ptr()
        b.row_begin = r0
        b.row_end = r1
        return b

    def mult(self, x: torch.Tensor, y: torch.Tensor | None = None) -> torch.Tensor:
        """y = A x for a dof vector x [nrows*bs] (HIP BSR SpMV, fa_bsr_mult, per row part)."""
        import ctypes

        from . import _lib

        L = _lib.load()
        if y is None:
            y = torch.empty_like(x)
        sh = _lib.stream_handle(x.device)
        for part in range(len(self.parts)):
            fb = self._fa_bsr(part)
            _lib.check(L.fa_bsr_mult(ctypes.byref(fb), x.data_ptr(), y.data_ptr(), sh), "fa_bsr_mult")
        return y

    def block_diagonal(self) -> torch.Tensor:
        """Diagonal blocks [nrows, bs, bs] (fa_bsr_block_diag; zeros where a row has none)."""
        import ctypes

        from . import _lib

        L = _lib.load()
        out = torch.empty((self.num_block_rows, self.bs, self.bs), dtype=torch.float64, device=self.indices.device)
        sh = _lib.stream_handle(out.device)
        for part in range(len(self.parts)):
            fb = self._fa_bsr(part)
            r0 = self.parts[part][0]
            _lib.check(L.fa_bsr_block_diag(ctypes.byref(fb), out[r0:].data_ptr(), sh), "fa_bsr_block_diag")
        return out
