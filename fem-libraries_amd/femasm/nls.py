"""Newton driver over the GPU assembly (the caller of the hot path).

Mirrors the reference's nonlinear solve — dolfinx ``fem.petsc.NonlinearProblem`` +
``nls.petsc.NewtonSolver`` (FEniCSx/mechanic2d/asym_elasto_damage_model_symb_sym.py:330-345;
C++: asym_elasto_damage_model.cc:705-714, 820-890) — with every operator on the GPU:

* ``NonlinearProblem.F`` = assemble_vector → apply_lifting(b, [J], [bcs], [x], -1) →
  set_bc(b, bcs, x, -1)  (the reference's ``setF``, :820-838);
* ``NonlinearProblem.J`` = assemble_matrix(J, bcs) with diagonal 1 (``setJ``, :847-862);
* the Newton iteration restates dolfinx's ``NewtonSolver::solve`` (dolfinx is a third-party
  dependency, not in /root/reference; v0.7-0.9 cpp/dolfinx/nls/NewtonSolver.cpp): F at the
  start; while not converged and it < max_it: J, solve J dx = F, x -= relaxation * dx, it += 1,
  F; residual0 = ||dx|| after the first update; convergence = the reference's own check
  (:870-890): ``||F|| / residual0 < rtol or ||F|| < atol``;
* the Krylov solve is conjugate gradients on the assembled BSR matrix (``fa_bsr_mult``) with a
  block-Jacobi preconditioner (``fa_bsr_block_diag``); ksp_rtol 1e-12 and max 2000 iterations as
  the reference sets (:717). The reference preconditions with BoomerAMG (:720-813), which is out
  of scope here: iteration counts differ, the converged solution does not.

Single GPU (the assembly's multi-GPU path is ``femasm.parallel``; a distributed Krylov solve is
not part of this module).
"""
from __future__ import annotations

import math

import torch

from . import fem
from .la import MatrixCSR


class NonlinearProblem:
    """F(u) = 0 with Jacobian J (dolfinx.fem.petsc.NonlinearProblem(F, u, bcs, J)).

    ``F`` and ``J`` are femasm forms (LinearElasticity / AsymDamage / NeoHookean) whose state
    ``u`` is this problem's ``u`` (the same storage: the driver updates it in place). ``J``
    defaults to ``F`` (the forms carry both the residual and its derivative).
    """

    def __init__(self, F, u: fem.Function, bcs=None, J=None):
        self.L = F
        self.a = J if J is not None else F
        self.u = u
        self.bcs = list(bcs or [])
        for frm in (self.L, self.a):
            if frm.u is None or frm.u.data_ptr() != u.x.data_ptr():
                raise ValueError("the forms' state u must be the problem's Function u (same storage)")
        self._A = None

    def form(self, x: torch.Tensor):
        """Called before F/J each iteration (the reference scatters ghosts here, :864-867)."""

    def F(self, x: torch.Tensor, b: torch.Tensor):
        b.zero_()
        fem.assemble_vector(self.L, b)
        fem.apply_lifting(b, [self.a], [self.bcs], x0=[x], alpha=-1.0)
        fem.set_bc(b, self.bcs, x, -1.0)

    def J(self, x: torch.Tensor, A: MatrixCSR):
        fem.assemble_matrix(self.a, bcs=self.bcs, diagonal=1.0, A=A)

    def matrix(self) -> MatrixCSR:
        if self._A is None:
            self._A = fem.create_matrix(self.a)
        return self._A


class KrylovSolver:
    """Preconditioned CG (PETSc KSPCG semantics: converged when the preconditioned residual norm
    falls below rtol times its initial value, or below atol; zero initial guess)."""

    def __init__(self, rtol: float = 1e-12, atol: float = 1e-50, max_it: int = 2000):
        self.rtol, self.atol, self.max_it = rtol, atol, max_it
        self.iterations = 0

    def set_operator(self, A: MatrixCSR):
        self.A = A
        D = A.block_diagonal()
        # rows without a diagonal block (none after assembly with bcs) keep identity
        eye = torch.eye(A.bs, dtype=D.dtype, device=D.device)
        bad = D.abs().sum((1, 2)) == 0
        D[bad] = eye
        self.Dinv = torch.linalg.inv(D)

    def _prec(self, r: torch.Tensor) -> torch.Tensor:
        bs = self.A.bs
        return torch.bmm(self.Dinv, r.reshape(-1, bs, 1)).reshape(-1)

    def solve(self, x: torch.Tensor, b: torch.Tensor) -> int:
        A = self.A
        x.zero_()
        r = b.clone()
        z = self._prec(r)
        p = z.clone()
        rz = torch.dot(r, z)
        znorm0 = float(torch.linalg.vector_norm(z))
        tol = max(self.rtol * znorm0, self.atol)
        Ap = torch.empty_like(b)
        it = 0
        if znorm0 <= tol:
            self.iterations = 0
            return 0
        while it < self.max_it:
            A.mult(p, Ap)
            alpha = rz / torch.dot(p, Ap)
            x.add_(alpha * p)
            r.sub_(alpha * Ap)
            z = self._prec(r)
            it += 1
            if float(torch.linalg.vector_norm(z)) <= tol:
                break
            rz_new = torch.dot(r, z)
            p.mul_(rz_new / rz).add_(z)
            rz = rz_new
        else:
            raise RuntimeError(f"CG did not converge in {self.max_it} iterations")
        self.iterations = it
        return it


class NewtonSolver:
    """dolfinx.nls.petsc.NewtonSolver restated (see module doc). Parameters default to dolfinx's
    (rtol 1e-9, atol 1e-10, max_it 50); the reference sets rtol 1e-7, atol 5e-8, max_it 10."""

    def __init__(self, comm=None, problem: NonlinearProblem | None = None):
        self.problem = problem
        self.rtol = 1e-9
        self.atol = 1e-10
        self.max_it = 50
        self.relaxation_parameter = 1.0
        self.error_on_nonconvergence = True
        self.report = False
        self.krylov_solver = KrylovSolver()
        self.residual = 0.0
        self.residual0 = 0.0
        self.iteration = 0
        self.krylov_iterations = 0
        self.history: list[float] = []

    def _converged(self, b: torch.Tensor) -> bool:
        # the reference's convergence check (asym_elasto_damage_model.cc:870-890)
        self.residual = float(torch.linalg.vector_norm(b))
        self.history.append(self.residual)
        rel = self.residual / self.residual0 if self.residual0 > 0 else math.inf
        if self.report:
            print(f"Newton iteration {self.iteration}: r (abs) = {self.residual:e} (tol = {self.atol}) "
                  f"r (rel) = {rel:e}(tol = {self.rtol})")
        return rel < self.rtol or self.residual < self.atol

    def solve(self, u: fem.Function) -> tuple[int, bool]:
        P = self.problem
        x = u.x
        if x.data_ptr() != P.u.x.data_ptr():
            raise ValueError("solve(u) must be called with the problem's u")
        b = torch.zeros_like(x)
        dx = torch.zeros_like(x)
        A = P.matrix()
        self.iteration = 0
        self.krylov_iterations = 0
        self.residual0 = 0.0
        self.history = []
        P.form(x)
        P.F(x, b)
        converged = self._converged(b)
        while not converged and self.iteration < self.max_it:
            P.J(x, A)
            self.krylov_solver.set_operator(A)
            self.krylov_iterations += self.krylov_solver.solve(dx, b)
            x.sub_(self.relaxation_parameter * dx)
            self.iteration += 1
            P.form(x)
            P.F(x, b)
            if self.iteration == 1:
                self.residual0 = float(torch.linalg.vector_norm(dx))
            converged = self._converged(b)
        if not converged and self.error_on_nonconvergence:
            raise RuntimeError(f"Newton solver did not converge in {self.iteration} iterations "
                               f"(residual {self.residual:e})")
        return self.iteration, converged
