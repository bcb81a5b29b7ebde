"""dolfinx.fem-shaped host API over the femasm C ABI.

Mirrors the calls the reference makes on its hot path (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:
``create_functionspace`` :275-285, ``Function`` / ``Constant`` :253-262, :506-546,
``locate_dofs_topological`` + ``DirichletBC`` :620-669, ``create_form`` :679-685,
``petsc::create_matrix`` :688, ``assemble_matrix`` + ``set_diagonal`` :847-862), with the
same argument meaning: bcs zero the rows/columns of constrained dofs and ``diagonal`` is
inserted on them. Mesh, dofmaps, coefficients and the global BSR matrix are torch tensors
on the GPU; every numeric step runs in hand-written HIP kernels (libfemasm.so). There is no
CPU fallback.
"""
from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .la import MatrixCSR
from .mesh import CellType, Mesh, NVERTS

from .mesh import EDGES as _EDGES, HEX_FACES as _HEX_FACES, REF_VERTS as _REF_VERTS  # basix sub-entities

_HEX_FACE_SPAN = ((0, 1, 2), (0, 1, 4), (0, 2, 4), (1, 3, 5), (2, 3, 6), (4, 5, 6))


def is_simplex(ct) -> bool:
    return CellType(ct) in (CellType.triangle, CellType.tetrahedron)


def num_nodes_of(ct, p: int) -> int:
    ct = CellType(ct)
    return {CellType.triangle: (p + 1) * (p + 2) // 2, CellType.tetrahedron: (p + 1) * (p + 2) * (p + 3) // 6,
            CellType.quadrilateral: (p + 1) ** 2, CellType.hexahedron: (p + 1) ** 3}[ct]


def element_info(ct, degree: int, qdeg: int | None = None) -> tuple[int, int]:
    """(nodes per cell, quadrature points) of the library's element tables (fa_element_info);
    qdeg None = the degree UFL estimates for the elasticity form."""
    nn, nq = ctypes.c_int32(0), ctypes.c_int32(0)
    _lib.check(_lib.load().fa_element_info(int(CellType(ct)), int(degree), -1 if qdeg is None else int(qdeg),
                                           ctypes.byref(nn), ctypes.byref(nq)), "fa_element_info")
    return nn.value, nq.value


def line_points(p: int) -> np.ndarray:
    """1-D node positions: equispaced (p <= 2) or GLL (p = 3; basix gll_warped)."""
    if p == 3:
        return np.array([0.0, 0.5 * (1 - 1 / np.sqrt(5)), 0.5 * (1 + 1 / np.sqrt(5)), 1.0])
    return np.linspace(0.0, 1.0, p + 1)


def node_lattice(ct, p: int) -> np.ndarray:
    """basix local node -> integer lattice position (units of 1/p of the cell) [nn, tdim].
    For tensor cells the entries are 1-D lattice indices (GLL positions at p = 3)."""
    ct = CellType(ct)
    V = np.array(_REF_VERTS[ct]) * p
    out = [tuple(v) for v in V]
    for a, b in _EDGES[ct]:
        for s in range(1, p):
            out.append(tuple(V[a] + s * (V[b] - V[a]) // p))
    if ct == CellType.quadrilateral:
        for i in range(1, p):
            for j in range(1, p):
                out.append((i, j))
    if ct == CellType.hexahedron:
        for f in _HEX_FACE_SPAN:
            for s in range(1, p):
                for t in range(1, p):
                    out.append(tuple(V[f[0]] + s * (V[f[1]] - V[f[0]]) // p + t * (V[f[2]] - V[f[0]]) // p))
        for i in range(1, p):
            for j in range(1, p):
                for k in range(1, p):
                    out.append((i, j, k))
    if is_simplex(ct) and p > 2:
        raise NotImplementedError("simplex degree > 2")
    return np.array(out, dtype=np.int64)


def reference_nodes(ct, p: int) -> np.ndarray:
    L = node_lattice(ct, p)
    if is_simplex(ct):
        return L.astype(np.float64) / p
    return line_points(p)[L]


def _geometry_basis(ct, X: np.ndarray) -> np.ndarray:
    """P1 / Q1 geometry basis values at reference points X [n, tdim] -> [n, nverts]."""
    ct = CellType(ct)
    if is_simplex(ct):
        return np.concatenate([1.0 - X.sum(1, keepdims=True), X], axis=1)
    cols = []
    for v in _REF_VERTS[ct]:
        f = np.ones(X.shape[0])
        for d, bit in enumerate(v):
            f = f * (X[:, d] if bit else 1.0 - X[:, d])
        cols.append(f)
    return np.stack(cols, 1)


class FunctionSpace:
    """Vector (bs = gdim) or scalar Lagrange space, or DG0 (per-cell) space."""

    def __init__(self, mesh: Mesh, family: str, degree: int, shape: tuple | None):
        self.mesh = mesh
        self.family = family
        self.degree = int(degree)
        self.bs = int(np.prod(shape)) if shape else 1
        self._adjacency = None
        self._pattern = None
        if family in ("DG", "Discontinuous Lagrange"):
            if degree != 0:
                raise NotImplementedError("only DG0 coefficient spaces")
            self.dofmap = torch.arange(mesh.num_cells, dtype=torch.int32, device=mesh.device).reshape(-1, 1)
            self.num_nodes = mesh.num_cells
            self.nn = 1
            return
        if family not in ("Lagrange", "P", "Q", "CG"):
            raise ValueError(f"unsupported family {family}")
        self.nn = num_nodes_of(mesh.cell_type, self.degree)
        if self.degree == 1:
            self.dofmap = mesh.cells
            self.num_nodes = mesh.num_vertices
        elif mesh.structured is not None:
            self.dofmap, self.num_nodes = _structured_dofmap(mesh, self.degree)
        else:
            self.dofmap, self.num_nodes = _generic_dofmap(mesh, self.degree)
        self._x = None

    @classmethod
    def from_dofmap(cls, mesh: Mesh, degree: int, bs: int, dofmap: torch.Tensor, num_nodes: int) -> "FunctionSpace":
        """A Lagrange space with a caller-supplied node numbering (e.g. a rank-local numbering
        of a slab of a larger mesh: femasm.parallel)."""
        V = cls.__new__(cls)
        V.mesh, V.family, V.degree, V.bs = mesh, "Lagrange", int(degree), int(bs)
        V.nn = num_nodes_of(mesh.cell_type, int(degree))
        V.dofmap = dofmap.to(torch.int32).contiguous()
        V.num_nodes = int(num_nodes)
        V._adjacency, V._pattern, V._x = None, None, None
        return V

    @property
    def num_dofs(self) -> int:
        return self.num_nodes * self.bs

    def tabulate_dof_coordinates(self) -> torch.Tensor:
        """Node coordinates [num_nodes, gdim] (the geometry map applied to the reference nodes)."""
        if self._x is None and self.mesh.structured is not None and self.degree > 1:
            self._x = _structured_node_coordinates(self.mesh, self.degree)
        if self._x is None:
            m = self.mesh
            X = reference_nodes(m.cell_type, self.degree)
            Psi = torch.tensor(_geometry_basis(m.cell_type, X), dtype=torch.float64, device=m.device)  # [nn, nv]
            xv = m.x[m.cells.to(torch.int64)]  # [nc, nv, gdim]
            xn = torch.einsum("kv,cvd->ckd", Psi, xv)
            out = torch.zeros((self.num_nodes, m.gdim), dtype=torch.float64, device=m.device)
            out[self.dofmap.to(torch.int64).reshape(-1)] = xn.reshape(-1, m.gdim)
            self._x = out
        return self._x

    # native objects -------------------------------------------------------------------
    def _fa_mesh(self) -> _lib.fa_mesh:
        m = self.mesh
        s = _lib.fa_mesh()
        s.cell_type = int(m.cell_type)
        s.degree = self.degree
        s.gdim = m.gdim
        s.nn = self.nn
        s.ncells = m.num_cells
        s.nnodes = self.num_nodes
        s.cells = self.dofmap.data_ptr()
        s.nv = NVERTS[m.cell_type]
        s.geom = m.cells.data_ptr()
        s.x = m.x.data_ptr()
        return s

    def adjacency(self):
        """Node -> cell adjacency (built once on the GPU: fa_build_adjacency)."""
        if self._adjacency is None:
            L = _lib.load()
            dev = self.mesh.device
            ptr = torch.empty(self.num_nodes + 1, dtype=torch.int64, device=dev)
            idx = torch.empty(self.mesh.num_cells * self.nn, dtype=torch.int32, device=dev)
            fm = self._fa_mesh()
            _lib.check(L.fa_build_adjacency(ctypes.byref(fm), ptr.data_ptr(), idx.data_ptr(), _lib.stream_handle(dev)),
                       "fa_build_adjacency")
            self._adjacency = (ptr, idx)
        return self._adjacency

    def _fa_adjacency(self) -> _lib.fa_adjacency:
        ptr, idx = self.adjacency()
        a = _lib.fa_adjacency()
        a.ptr = ptr.data_ptr()
        a.idx = idx.data_ptr()
        return a


def _structured_dofmap(mesh: Mesh, p: int, chunk: int = 1 << 22):
    """Lattice numbering of a structured mesh's degree-p nodes: node index of lattice point
    (I, J[, K]) is I + (p nx + 1)(J + (p ny + 1) K) — neighbours stay close in memory.
    Processed in cell chunks to bound temporaries (config E has 50 M cells)."""
    st = mesh.structured
    n = st["n"]
    tdim = len(n)
    dims = [p * k + 1 for k in n]
    vdims = [k + 1 for k in n]
    dev = mesh.device
    L = torch.tensor(node_lattice(mesh.cell_type, p), dtype=torch.int64, device=dev)  # [nn, tdim]
    out = torch.empty((mesh.num_cells, L.shape[0]), dtype=torch.int32, device=dev)
    simplex = is_simplex(mesh.cell_type)
    for c0 in range(0, mesh.num_cells, chunk):
        v = mesh.cells[c0:c0 + chunk].to(torch.int64)
        vlat = []
        for d in range(tdim):
            stride = int(np.prod(vdims[:d]))
            vlat.append((v // stride) % vdims[d])
        vlat = torch.stack(vlat, -1)  # [nc, nv, tdim]
        v0 = vlat[:, 0, :]
        nl = p * v0[:, None, :]
        if simplex:
            # node lattice = p v0 + sum_k L[node, k] (v_k - v0)   (L in units of 1/p)
            for k in range(tdim):
                nl = nl + L[None, :, k, None] * (vlat[:, k + 1, :] - v0)[:, None, :]
        else:
            nl = nl + L[None, :, :]
        idx = torch.zeros(nl.shape[:2], dtype=torch.int64, device=dev)
        for d in range(tdim - 1, -1, -1):
            idx = idx * dims[d] + nl[:, :, d]
        out[c0:c0 + chunk] = idx.to(torch.int32)
    return out.contiguous(), int(np.prod(dims))


def _structured_node_coordinates(mesh: Mesh, p: int) -> torch.Tensor:
    """Node coordinates of the lattice numbering (uniform box, GLL-graded inside cells at p = 3)."""
    st = mesh.structured
    n, lengths = st["n"], st["lengths"]
    r = torch.tensor(line_points(p), dtype=torch.float64, device=mesh.device)
    axes = []
    for k, Lk in zip(n, lengths):
        i = torch.arange(p * k + 1, device=mesh.device)
        cell, loc = torch.div(i, p, rounding_mode="floor"), i % p
        cell = torch.where(i == p * k, torch.full_like(cell, k - 1), cell)
        loc = torch.where(i == p * k, torch.full_like(loc, p), loc)
        axes.append((cell.to(torch.float64) + r[loc]) * (Lk / k))
    grids = torch.meshgrid(*reversed(axes), indexing="ij")
    return torch.stack([g.reshape(-1) for g in reversed(grids)], 1).contiguous()


def _generic_dofmap(mesh: Mesh, p: int):
    """Degree-2 numbering of an unstructured mesh: vertices, then one node per edge (and per
    hex face and quad/hex cell), edges identified by their sorted vertex pair."""
    if p != 2:
        raise NotImplementedError("unstructured meshes: degree <= 2 (Q3 needs a structured mesh)")
    ct = mesh.cell_type
    c = mesh.cells.to(torch.int64)
    nv = mesh.num_vertices
    parts = [c]
    E = torch.tensor(_EDGES[ct], dtype=torch.int64, device=c.device)
    ev = c[:, E]  # [nc, ne, 2]
    lo, hi = ev.min(-1).values, ev.max(-1).values
    key = lo * nv + hi
    uniq, inv = torch.unique(key.reshape(-1), return_inverse=True)
    parts.append(nv + inv.reshape(key.shape))
    nxt = nv + uniq.numel()
    if ct == CellType.hexahedron:
        F = torch.tensor(_HEX_FACES, dtype=torch.int64, device=c.device)
        fv = torch.sort(c[:, F], dim=-1).values  # [nc, 6, 4]
        fu, finv = torch.unique(fv.reshape(-1, 4), dim=0, return_inverse=True)
        parts.append(nxt + finv.reshape(fv.shape[:2]))
        nxt += fu.shape[0]
    if ct in (CellType.quadrilateral, CellType.hexahedron):
        parts.append(nxt + torch.arange(mesh.num_cells, device=c.device).reshape(-1, 1))
        nxt += mesh.num_cells
    return torch.cat(parts, 1).to(torch.int32).contiguous(), int(nxt)


def functionspace(mesh: Mesh, element) -> FunctionSpace:
    """dolfinx.fem.functionspace(mesh, ("Lagrange", p, (gdim,))) / ("DG", 0)."""
    family, degree = element[0], element[1]
    shape = element[2] if len(element) > 2 else None
    return FunctionSpace(mesh, family, degree, shape)


class Function:
    def __init__(self, V: FunctionSpace, name: str = "f", x: torch.Tensor | None = None):
        self.function_space = V
        self.name = name
        n = V.num_nodes * V.bs
        self.x = x if x is not None else torch.zeros(n, dtype=torch.float64, device=V.mesh.device)

    @property
    def array(self) -> torch.Tensor:
        return self.x

    def interpolate(self, fn):
        """Nodal interpolation: fn(x[gdim, n]) -> values [bs, n] (dolfinx convention)."""
        V = self.function_space
        xn = V.tabulate_dof_coordinates()
        vals = fn(xn.T)
        vals = torch.as_tensor(vals, dtype=torch.float64, device=xn.device).reshape(V.bs, -1)
        self.x = vals.T.contiguous().reshape(-1)


class Constant:
    def __init__(self, mesh_or_value, value=None):
        self.value = float(mesh_or_value if value is None else value)

    def __float__(self):
        return self.value


@dataclass
class DirichletBC:
    """Constrained dofs of V with their prescribed values (blocked dof = node*bs + comp)."""
    V: FunctionSpace
    dofs: torch.Tensor  # int64 dof indices
    g: torch.Tensor  # float64 [num_dofs] prescribed values (0 elsewhere)

    def marker(self) -> torch.Tensor:
        m = torch.zeros(self.V.num_dofs, dtype=torch.int8, device=self.dofs.device)
        m[self.dofs] = 1
        return m


def locate_dofs_geometrical(V: FunctionSpace, marker) -> torch.Tensor:
    """Nodes whose coordinates satisfy marker(x[gdim, n]); returns node indices (int64)."""
    xn = V.tabulate_dof_coordinates()
    return torch.nonzero(marker(xn.T), as_tuple=False).reshape(-1)


def _closure_nodes(ct, p: int, S) -> list:
    """Local nodes (basix order) in the closure of the reference sub-entity with local vertices S:
    simplices, barycentric coordinates of the vertices outside S vanish; tensor cells, the node lies
    on every coordinate plane all vertices of S share."""
    ct = CellType(ct)
    X = reference_nodes(ct, p)
    RV = np.array(_REF_VERTS[ct], dtype=np.float64)
    on = np.ones(X.shape[0], dtype=bool)
    if is_simplex(ct):
        lam = np.concatenate([1.0 - X.sum(1, keepdims=True), X], axis=1)  # [nn, nv]
        for v in range(RV.shape[0]):
            if v not in S:
                on &= np.abs(lam[:, v]) < 1e-12
    else:
        for d in range(RV.shape[1]):
            vals = {RV[v, d] for v in S}
            if len(vals) == 1:
                on &= np.abs(X[:, d] - vals.pop()) < 1e-12
    return [int(j) for j in np.nonzero(on)[0]]


def locate_dofs_topological(V: FunctionSpace, entity_dim: int, entities) -> torch.Tensor:
    """dolfinx.fem.locate_dofs_topological: the nodes (block dofs) in the closure of the given
    entities of dimension entity_dim (ids of femasm.mesh.entities; vertex indices for dim 0).
    Closure semantics as dolfinx: a vertex carries only its own node, an edge its vertices' and its
    interior nodes, a facet every node on it. The reference selects with entity_dim 0
    (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:637-638, :661-662), which for P >= 2 constrains
    the vertex nodes of the plane only. Returns sorted node indices (int64)."""
    from . import mesh as fmesh

    m = V.mesh
    ents = torch.as_tensor(entities, device=m.device).to(torch.int64).reshape(-1)
    _, cell_ents = fmesh.entities(m, entity_dim) if entity_dim < m.tdim else \
        (None, torch.arange(m.num_cells, device=m.device, dtype=torch.int64).reshape(-1, 1))
    nent = int(cell_ents.max()) + 1 if cell_ents.numel() else 0
    mark = torch.zeros(max(nent, int(ents.max()) + 1 if ents.numel() else 0), dtype=torch.bool, device=m.device)
    mark[ents] = True
    dm = V.dofmap.to(torch.int64)
    out = []
    for i, S in enumerate(fmesh.sub_entities(m.cell_type, entity_dim)):
        loc = torch.tensor(_closure_nodes(m.cell_type, V.degree, S), dtype=torch.int64, device=m.device)
        hit = mark[cell_ents[:, i]]
        if bool(hit.any()):
            out.append(dm[hit][:, loc].reshape(-1))
    if not out:
        return torch.zeros(0, dtype=torch.int64, device=m.device)
    return torch.unique(torch.cat(out))


def dirichletbc(value, nodes: torch.Tensor, V: FunctionSpace, components=None) -> DirichletBC:
    """Constrain all (or the given) components of `nodes` to `value` (a scalar or a bs-vector)."""
    bs = V.bs
    comps = list(range(bs)) if components is None else list(components)
    val = torch.as_tensor(value, dtype=torch.float64, device=nodes.device).reshape(-1)
    if val.numel() == 1:
        val = val.expand(bs)
    nodes = nodes.to(torch.int64)
    dofs = torch.cat([nodes * bs + c for c in comps]) if nodes.numel() else nodes
    g = torch.zeros(V.num_dofs, dtype=torch.float64, device=nodes.device)
    for c in comps:
        g[nodes * bs + c] = val[c]
    return DirichletBC(V, dofs, g)


def _bc_state(bc, with_g: bool):
    # the exact tensor objects a bc holds (weakly) and their in-place versions: a hit needs the same
    # objects at the same versions, so a reassigned bc.dofs / bc.g (even one the caching allocator
    # put at a freed tensor's address) or an edited one misses the cache
    st = [weakref.ref(bc), weakref.ref(bc.dofs), bc.dofs._version]
    if with_g:
        st += [weakref.ref(bc.g), bc.g._version]
    return st


def _bc_state_ok(st, bc, with_g: bool) -> bool:
    if st[0]() is not bc or st[1]() is not bc.dofs or st[2] != bc.dofs._version:
        return False
    return not with_g or (st[3]() is bc.g and st[4] == bc.g._version)


def _combine_bcs(V: FunctionSpace, bcs, with_g: bool = True):
    """(marker int8 [num_dofs], g f64 [num_dofs] or None) of a bcs list, cached on V per bcs set
    (a Newton loop assembles with the same bcs every iteration: the marker is built once, not in
    every timed assembly). with_g=False: the matrix assembly needs the marker only."""
    if not bcs:
        return None, None
    cache = V.__dict__.setdefault("_bc_cache", {})
    key = (with_g,) + tuple(id(bc) for bc in bcs)
    hit = cache.get(key)
    if hit is not None and all(_bc_state_ok(st, bc, with_g) for st, bc in zip(hit[2], bcs)):
        return hit[0], hit[1]
    marker = torch.zeros(V.num_dofs, dtype=torch.int8, device=V.mesh.device)
    g = torch.zeros(V.num_dofs, dtype=torch.float64, device=V.mesh.device) if with_g else None
    for bc in bcs:
        marker[bc.dofs] = 1
        if with_g:
            g[bc.dofs] = bc.g[bc.dofs]
    cache.pop(key, None)
    if len(cache) >= 8:  # a handful of bcs sets per space; drop the oldest
        cache.pop(next(iter(cache)))
    # weak references only (a bc refers to V: strong ones would make a cycle that keeps V's tensors
    # alive until a GC pass); a hit is checked against them, so a reused id cannot match
    cache[key] = (marker, g, [_bc_state(bc, with_g) for bc in bcs])
    return marker, g


# ---------------------------------------------------------------------------------- forms
class LinearElasticity:
    """J of the reference form with damage d = 0:
    inner(sigma(du), eps(v)) dx, sigma = lmbda tr(eps) I + 2 mu eps, mu = E/(2(1+nu)),
    lmbda = E nu/((1+nu)(1-2nu))  (FEniCSx/mechanic2d/asym_ufl.py:22-34, :78-83).
    E: DG0 Function / per-cell tensor / float; nu: Constant / float. Alternatively lam & mu per cell."""
    kind = _lib.FA_LINEAR_ELASTICITY

    def __init__(self, V: FunctionSpace, E=None, nu=0.3, lam=None, mu=None, quadrature_degree: int | None = None,
                 u=None, f=None):
        self.V = V
        nc = V.mesh.num_cells
        dev = V.mesh.device
        self.nu = float(nu)
        self.E = self.lam = self.mu = None
        if E is not None:
            self.E = _cellwise(E, nc, dev)
        else:
            self.lam, self.mu = _cellwise(lam, nc, dev), _cellwise(mu, nc, dev)
        self.qdeg = -1 if quadrature_degree is None else int(quadrature_degree)
        self.d = None
        # state (residual / nonlinear tangents) and body force, per dof; Functions or tensors
        self.u = None if u is None else (u.x if isinstance(u, Function) else u)
        self.f = None if f is None else (f.x if isinstance(f, Function) else f)


class AsymDamage(LinearElasticity):
    """The reference mechanic2d J: derivative of inner(sigma(u), eps(v)) dxx with the
    asymmetric tension/compression damage law, P1 triangles, one quadrature point
    (FEniCSx/mechanic2d/asym_ufl.py:36-81; MFEM/mechanic2d/asym_elasto_damage_model.cc:639-916).
    u: displacement Function, d: damage (P1 scalar Function or per-node tensor)."""
    kind = _lib.FA_ASYM_DAMAGE

    def __init__(self, V: FunctionSpace, E=None, nu=0.3, u=None, d=None, lam=None, mu=None, f=None,
                 tangent: str = "hand"):
        """tangent: "hand" (the reference's default build: eigen-decomposition tangent and stress,
        :207-329, :766-881) or "ad" (its USE_AD build: forward-over-forward AD of the damage
        potential, :100-204, :752-763)."""
        super().__init__(V, E=E, nu=nu, lam=lam, mu=mu, quadrature_degree=1, u=u, f=f)
        self.d = None if d is None else (d.x if isinstance(d, Function) else d)
        if tangent not in ("hand", "ad"):
            raise ValueError(f"tangent must be 'hand' or 'ad', not {tangent!r}")
        self.tangent = tangent
        if tangent == "ad":
            self.kind = _lib.FA_ASYM_DAMAGE_AD


class NeoHookean(LinearElasticity):
    """Compressible neo-Hookean tangent (BASELINE config E): psi = mu/2 (I_C - 3) - mu ln J +
    lmbda/2 (ln J)^2, F = I + grad u; J = derivative of the first Piola stress, taken on the
    GPU by forward-over-forward automatic differentiation of psi (the pattern of the reference's
    MFEM AD, MFEM/mechanic2d/autodiff/admfem.hpp:672-700). u: the state (required)."""
    kind = _lib.FA_NEO_HOOKEAN

    def __init__(self, V: FunctionSpace, E=None, nu=0.3, u=None, lam=None, mu=None, quadrature_degree=None, f=None):
        if u is None:
            raise ValueError("NeoHookean needs the state u")
        super().__init__(V, E=E, nu=nu, lam=lam, mu=mu, quadrature_degree=quadrature_degree, u=u, f=f)


def _cellwise(v, nc, dev):
    if isinstance(v, Function):
        v = v.x
    t = torch.as_tensor(v, dtype=torch.float64, device=dev)
    if t.numel() == 1:
        t = t.reshape(1).expand(nc)
    return t.contiguous()


def form(a):
    """dolfinx.fem.form analogue: forms are ready-made descriptors here (no code generation);
    returns the argument after validating it."""
    if not isinstance(a, LinearElasticity):
        raise TypeError("expected a femasm form descriptor (LinearElasticity, AsymDamage, ...)")
    return a


def _fa_form(a) -> _lib.fa_form:
    f = _lib.fa_form()
    f.kind = a.kind
    f.qdeg = a.qdeg
    f.E = _lib.ptr(a.E)
    f.nu = a.nu
    f.lam = _lib.ptr(a.lam)
    f.mu = _lib.ptr(a.mu)
    f.u = _lib.ptr(a.u)
    f.d = _lib.ptr(a.d)
    f.f = _lib.ptr(a.f)
    return f


def check_pattern(V: FunctionSpace, indptr: torch.Tensor, indices: torch.Tensor):
    """Validate a pattern of V and V's adjacency on the device (fa_check_pattern): sorted unique
    in-range columns, monotone indptr, exactly the node pairs of the cells. Raises FemasmError."""
    fm = V._fa_mesh()
    adj = V._fa_adjacency()
    _lib.check(_lib.load().fa_check_pattern(ctypes.byref(fm), ctypes.byref(adj), indptr.data_ptr(), indices.data_ptr(),
                                            int(indices.numel()), _lib.stream_handle(V.mesh.device)),
               "fa_check_pattern")


def sparsity_pattern(V: FunctionSpace):
    """The BSR pattern (indptr, indices) of V's cell node pairs, built on the GPU once and cached on V
    (dolfinx.fem.create_sparsity_pattern; create_matrix uses it)."""
    if V._pattern is None:
        L = _lib.load()
        dev = V.mesh.device
        fm = V._fa_mesh()
        adj = V._fa_adjacency()
        indptr = torch.empty(V.num_nodes + 1, dtype=torch.int64, device=dev)
        nb = ctypes.c_int64(0)
        sh = _lib.stream_handle(dev)
        _lib.check(L.fa_sparsity_count(ctypes.byref(fm), ctypes.byref(adj), indptr.data_ptr(), ctypes.byref(nb), sh),
                   "fa_sparsity_count")
        indices = torch.empty(nb.value, dtype=torch.int32, device=dev)
        _lib.check(L.fa_sparsity_fill(ctypes.byref(fm), ctypes.byref(adj), indptr.data_ptr(), indices.data_ptr(), sh),
                   "fa_sparsity_fill")
        V._pattern = (indptr, indices)
    return V._pattern


def create_matrix(a, max_part_bytes: int | None = None, check: bool = False) -> MatrixCSR:
    """Sparsity pattern of the bilinear form (all node pairs of every cell), built on the GPU
    (dolfinx.fem.petsc.create_matrix, FEniCSx/mechanic2d/asym_elasto_damage_model.cc:688), and the
    matrix's value array. check: validate the pattern and adjacency on the device (fa_check_pattern)."""
    V = a.V
    indptr, indices = sparsity_pattern(V)
    if check:
        check_pattern(V, indptr, indices)
    if max_part_bytes is None:
        return MatrixCSR(indptr, indices, V.bs)
    return MatrixCSR(indptr, indices, V.bs, max_part_bytes=max_part_bytes)


def _fa_bsr(A: MatrixCSR, part: int = 0) -> _lib.fa_bsr:
    return A._fa_bsr(part)


def _plan_order(V, fm, adj, fb, plan, sh, eadj=None, order: str = "positional", search: bool = False):
    """Bank-conflict-aware LDS order of the affine-simplex gather (fa_plan_order). order:
    "positional" (default) also balances which entries share a 16-lane quarter (one int32 per
    adjacency entry), "steps" orders each lane's blocks only, "none" keeps the plain slot map.
    search: also the alternating-path moves (FA_PLAN_ORDER_SEARCH: ~0.5 % faster assemblies on config E
    for a ~10x longer plan)."""
    if order not in ("positional", "steps", "none"):
        raise ValueError(f"unknown slot order {order!r}")
    if order == "none":
        return None
    if search:
        plan.cell_flags |= _lib.FA_PLAN_ORDER_SEARCH
    if order == "positional" and eadj is None:
        eadj = torch.empty(V.mesh.num_cells * V.nn, dtype=torch.int32, device=V.mesh.device)
    if order != "positional":
        eadj = None
    _lib.check(_lib.load().fa_plan_order(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb),
                                         eadj.data_ptr() if eadj is not None else None, ctypes.byref(plan), sh),
               "fa_plan_order")
    return eadj if plan.eadj else None


def _plan_locality(V, fm, adj, plan, sh, locality=True):
    """Chunk visiting order of the gather (the kernels' XCD x walks positions [x per, (x + 1) per) of
    it). True / "morton": fa_plan_locality, Morton order of the chunks' positions, so chunks that share
    cells run close in time on one XCD and the cells' records are re-read from its L2. "deal": row
    order dealt to the XCDs in pairs of chunks (chunk c to XCD (c // 2) mod 8): every XCD works in one
    compact window of the matrix at any time (the neo-Hookean gather, round 6: 62.1-62.2 vs 63.2-63.3 ms
    Morton on config E-neo, profiles/r6/order_variants_Eneo.txt). False / "row": row order, XCD x
    taking the contiguous eighth x of the chunks."""
    if locality in (False, "row") or plan.nchunks <= 1:
        return None
    if locality == "deal":
        nch = int(plan.nchunks)
        c = torch.arange(nch, device=V.mesh.device, dtype=torch.int64)
        corder = torch.argsort(((c // 2) % 8) * nch + c).to(torch.int32).contiguous()
        plan.corder = corder.data_ptr()
        return corder
    if locality not in (True, "morton"):
        raise ValueError(f"unknown chunk order {locality!r}")
    corder = torch.empty(plan.nchunks, dtype=torch.int32, device=V.mesh.device)
    _lib.check(_lib.load().fa_plan_locality(ctypes.byref(fm), ctypes.byref(adj), corder.data_ptr(),
                                            ctypes.byref(plan), sh), "fa_plan_locality")
    return corder if plan.corder else None


def _use_contrib(V, kind, owner) -> bool:
    """Block-owner gather (fa_plan_contrib) for linear elasticity on P1/P2 triangles and
    tetrahedra. owner=None (default) uses it for triangles, where it measured faster (config A
    0.136 vs 0.220 ms), and keeps the LDS-atomic gather for tetrahedra, where that one is faster
    (C 1.72 vs 2.07 ms, E 46.8 vs 53.1 ms); True / False force it."""
    if owner is False or kind != _lib.FA_LINEAR_ELASTICITY or V.degree not in (1, 2):
        return False
    if owner:
        return V.mesh.cell_type in (_lib.FA_TRIANGLE, _lib.FA_TETRAHEDRON)
    return V.mesh.cell_type == _lib.FA_TRIANGLE


def _plan_contrib(V, fm, adj, fb, rs, plan, sh):
    """Chunking + contribution plan of the block-owner gather; None (plan untouched) when a chunk
    cannot hold a row's entries (then the caller plans the LDS-atomic gather)."""
    L = _lib.load()
    rc = L.fa_plan_gather_contrib(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb), rs.data_ptr(),
                                  ctypes.byref(plan), sh)
    _lib.check(rc, "fa_plan_gather_contrib")
    if plan.nchunks == 0:
        return None
    nbytes = ctypes.c_int64(0)
    _lib.check(L.fa_plan_contrib_bytes(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb), ctypes.byref(plan),
                                       ctypes.byref(nbytes), sh), "fa_plan_contrib_bytes")
    buf = torch.empty(max(int(nbytes.value), 16), dtype=torch.uint8, device=V.mesh.device)
    rc = L.fa_plan_contrib(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb), buf.data_ptr(), buf.numel(),
                           ctypes.byref(plan), sh)
    if rc != _lib.FA_OK:
        if rc == -5:  # FA_E_CAPACITY: rows with more entries than a chunk holds
            return None
        _lib.check(rc, "fa_plan_contrib")
    return buf


def gather_plan(V: FunctionSpace, A: MatrixCSR, part: int = 0, kind: int = _lib.FA_LINEAR_ELASTICITY,
                deterministic: bool = False, owner: bool | None = None, slots: bool = True,
                order: str = "positional", locality: bool | None = None, search: bool = False):
    """Row-chunk plan of the gather kernel of a form kind for one row part of A's pattern (cached
    on V per options). Neo-Hookean forms get their own chunking (fa_plan_gather_form); the other
    kinds share one. deterministic: the LDS-atomic gather's plan (no contribution plan), for
    FA_DETERMINISTIC. owner: the block-owner contribution plan (None: for triangles). slots: the
    per-entry slot map (fa_plan_slots; False: the kernels search the pattern in LDS). order: the
    slot map's LDS order (_plan_order). search: the order's alternating-path moves (opt-in).
    locality: the chunk visiting order (_plan_locality: "morton" / True, "deal", "row" / False); None
    (default): "deal" for the neo-Hookean gather (62.1 vs 63.2 ms Morton on E-neo), "row" for the others
    (config E: 35.8 vs 36.3, 36.0 vs 36.2, 35.13 vs 35.29 ms Morton on three boxes; C 0.99 vs 1.01 ms;
    DESIGN.md §4)."""
    if deterministic and owner:
        raise ValueError("deterministic assembly runs the LDS-atomic gather: owner=True (block-owner plan) "
                         "cannot be combined with deterministic=True")
    neo = kind == _lib.FA_NEO_HOOKEAN
    if locality is None:
        locality = "deal" if neo else "row"
    if neo and not (slots and order == "positional"):
        raise ValueError("the neo-Hookean gather needs positional plans (slots=True, order='positional')")
    plans = V.__dict__.setdefault("_plans", {})
    contrib = _use_contrib(V, kind, owner) and not deterministic
    key = (A.indptr.data_ptr(), A.parts[part][0], A.parts[part][1], neo, contrib, slots, order, locality, search)
    if key not in plans:
        L = _lib.load()
        fm = V._fa_mesh()
        adj = V._fa_adjacency()
        fb = _fa_bsr(A, part)
        rs = torch.empty(A.parts[part][1] - A.parts[part][0] + 1, dtype=torch.int64, device=V.mesh.device)
        plan = _lib.fa_plan()
        sh = _lib.stream_handle(V.mesh.device)
        if contrib:
            buf = _plan_contrib(V, fm, adj, fb, rs, plan, sh)
            if buf is not None:
                plans[key] = (plan, rs, A.indptr, buf)
                return plan
        _lib.check(L.fa_plan_gather_form(ctypes.byref(fm), int(kind), ctypes.byref(adj), ctypes.byref(fb),
                                         rs.data_ptr(), ctypes.byref(plan), sh), "fa_plan_gather_form")
        smap = eadj = None
        # Per (adjacency entry, column node) block position in its row: no LDS search in the
        # kernel, for 2 B x nn^2 extra reads per cell. Measured with the interleaved-search
        # kernel: config E 64.5 -> 61.0 ms, C 2.22 -> 2.15 ms, Q2 quads +21 % (profiles/r1/
        # slots.md) -> on by default.
        if slots:
            smap = torch.empty(V.mesh.num_cells * V.nn * V.nn, dtype=torch.int16, device=V.mesh.device)
            _lib.check(L.fa_plan_slots(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb), smap.data_ptr(),
                                       ctypes.byref(plan), sh), "fa_plan_slots")
            # bank-balanced positional order of the LDS adds (affine-simplex elasticity and, with the
            # same column split, the neo-Hookean gather)
            eadj = _plan_order(V, fm, adj, fb, plan, sh, order=order, search=search)
        corder = _plan_locality(V, fm, adj, plan, sh, locality)
        # the gathers' chunk arrays in the visiting order, once per plan (fa_plan_chunk_desc; a launch
        # had rebuilt them: config E 0.21 ms of its ~35)
        cdesc = None
        if plan.nchunks > 0 and hasattr(L, "fa_plan_chunk_desc"):  # (an older measurement build lacks it)
            cdesc = torch.empty(3 * (int(plan.nchunks) + 1), dtype=torch.int64, device=V.mesh.device)
            _lib.check(L.fa_plan_chunk_desc(ctypes.byref(fm), ctypes.byref(adj), ctypes.byref(fb), ctypes.byref(plan),
                                            cdesc.data_ptr(), sh), "fa_plan_chunk_desc")
        plans[key] = (plan, rs, A.indptr, smap, eadj, corder, cdesc)
        V.__dict__.setdefault("_plan_xver", {})[key] = _coords_version(V.mesh)
    plan = plans[key][0]
    _recheck_affine(V, key, plan)
    return plan


def _coords_version(m) -> tuple:
    return (m.x.data_ptr(), m.x._version)


def _recheck_affine(V: FunctionSpace, key, plan):
    """The plan's FA_PLAN_AFFINE flag describes the coordinates it was planned on: the affine tensor
    gather builds each cell's Jacobian from three edges, so vertices moved in place since then
    (mesh.x is a public tensor) re-run the library's per-cell affinity check before assembling."""
    if V.mesh.cell_type not in (CellType.quadrilateral, CellType.hexahedron):
        return
    vers = V.__dict__.setdefault("_plan_xver", {})
    now = _coords_version(V.mesh)
    if vers.get(key) == now:
        return
    fm = V._fa_mesh()
    _lib.check(_lib.load().fa_plan_check_affine(ctypes.byref(fm), ctypes.byref(plan),
                                                _lib.stream_handle(V.mesh.device)), "fa_plan_check_affine")
    vers[key] = now


def assemble_matrix(a, bcs=None, diagonal: float = 1.0, A: MatrixCSR | None = None, method: str = "gather",
                    deterministic: bool = False, plan: dict | None = None, check: bool = False) -> MatrixCSR:
    """Assemble the bilinear form into a BSR matrix (dolfinx.fem.assemble_matrix + set_diagonal).

    bcs: list of DirichletBC — their rows and columns receive no cell contribution and their
    diagonal entries are set to `diagonal`. method: "gather" (row-gather, default) or
    "scatter" (element scatter with FP64 atomics; zeroes A first like MatZeroEntries).
    deterministic: bit-identical values run to run (FA_DETERMINISTIC: exact 64-bit fixed-point
    sums in the gather; linear elasticity with one Poisson ratio on affine simplices, affine Q1 / Q2
    quadrilaterals and Q1 hexahedra).
    plan: gather_plan options (owner, slots, order, locality). check: synchronise and raise if a
    kernel found a pattern entry missing (FA_CHECK_ERRORS).
    """
    V = a.V
    if method not in ("gather", "scatter"):
        raise ValueError(f"unknown method {method}")
    if deterministic and method != "gather":
        raise ValueError("deterministic assembly is a gather mode")
    if A is None:
        A = create_matrix(a)
    L = _lib.load()
    marker, _ = _combine_bcs(V, bcs, with_g=False)
    fm = V._fa_mesh()
    ff = _fa_form(a)
    sh = _lib.stream_handle(V.mesh.device)
    for part in range(len(A.parts)):
        fb = _fa_bsr(A, part)
        if method == "gather":
            adj = V._fa_adjacency()
            gp = gather_plan(V, A, part, a.kind, deterministic=deterministic, **(plan or {}))
            flags = _lib.FA_GATHER | (_lib.FA_DETERMINISTIC if deterministic else 0) | \
                (_lib.FA_CHECK_ERRORS if check else 0)
            rc = L.fa_assemble_matrix(ctypes.byref(fm), ctypes.byref(ff), ctypes.byref(adj), ctypes.byref(gp),
                                      _lib.ptr(marker), float(diagonal), ctypes.byref(fb), flags, sh)
        else:
            flags = _lib.FA_SCATTER | _lib.FA_ZERO_FIRST | (_lib.FA_CHECK_ERRORS if check else 0)
            rc = L.fa_assemble_matrix(ctypes.byref(fm), ctypes.byref(ff), None, None, _lib.ptr(marker),
                                      float(diagonal), ctypes.byref(fb), flags, sh)
        _lib.check(rc, "fa_assemble_matrix")
    A._keepalive = (marker, a)
    return A


class SplitGather:
    """fa_assemble_matrix(FA_GATHER) split into ``prepare()`` (per-cell records of all cells, once)
    and ``rows(i)`` (the rows of ``ranges[i]`` of one row part of A), via fa_gather_prepare /
    fa_gather_rows on a work buffer it owns. Each range is its own gather plan; every row of the
    part must be in exactly one range for a complete assembly. femasm.parallel uses it to start
    the interface exchange of a rank's slab while its interior rows assemble."""

    def __init__(self, a, bcs, A: MatrixCSR, ranges, part: int = 0, diagonal: float = 1.0,
                 deterministic: bool = False, slots: bool = True, order: str = "positional"):
        V = a.V
        if a.kind == _lib.FA_NEO_HOOKEAN and not (slots and order == "positional"):
            raise ValueError("the neo-Hookean gather needs positional plans (slots=True, order='positional')")
        L = _lib.load()
        self.L, self.a, self.A, self.diagonal = L, a, A, float(diagonal)
        self.marker, _ = _combine_bcs(V, bcs, with_g=False)
        self.fm, self.ff, self.adj = V._fa_mesh(), _fa_form(a), V._fa_adjacency()
        dev = V.mesh.device
        self.sh = _lib.stream_handle(dev)
        nbytes = ctypes.c_int64(0)
        _lib.check(L.fa_gather_work_bytes(ctypes.byref(self.fm), ctypes.byref(self.ff), ctypes.byref(nbytes)),
                   "fa_gather_work_bytes")
        self.work = torch.empty(max(int(nbytes.value), 16), dtype=torch.uint8, device=dev)
        pr0, pr1, data = A.parts[part]
        base = int(A.indptr[pr0])
        bs2 = A.bs * A.bs
        self.slots = None
        if slots:
            self.slots = torch.empty(V.mesh.num_cells * V.nn * V.nn, dtype=torch.int16, device=dev)
        self.subs, self.plans, self._keep = [], [], []
        self._xver = _coords_version(V.mesh)
        for r0, r1 in ranges:
            if not (pr0 <= r0 <= r1 <= pr1):
                raise ValueError(f"row range [{r0}, {r1}) outside part [{pr0}, {pr1})")
            fb = _fa_bsr(A, part)
            fb.row_begin, fb.row_end = r0, r1
            fb.data = data.data_ptr() + 8 * bs2 * (int(A.indptr[r0]) - base)
            rs = torch.empty(r1 - r0 + 1, dtype=torch.int64, device=dev)
            plan = _lib.fa_plan()
            if r1 > r0:
                _lib.check(L.fa_plan_gather_form(ctypes.byref(self.fm), int(a.kind), ctypes.byref(self.adj),
                                                 ctypes.byref(fb), rs.data_ptr(), ctypes.byref(plan), self.sh),
                           "fa_plan_gather_form")
            if deterministic:
                plan.cell_flags |= _lib.FA_PLAN_DETERMINISTIC
            self.subs.append(fb)
            self.plans.append(plan)
            self._keep.append(rs)
            if r1 > r0:
                self._keep.append(_plan_locality(V, self.fm, self.adj, plan, self.sh,  # (gather_plan's default)
                                                 locality="deal" if a.kind == _lib.FA_NEO_HOOKEAN else "row"))
        if self.slots is not None:
            # one slot map for all rows (fa_plan_slots writes every row), then each plan's order
            live = [i for i, (r0, r1) in enumerate(ranges) if r1 > r0]
            for i in live[:1]:
                _lib.check(L.fa_plan_slots(ctypes.byref(self.fm), ctypes.byref(self.adj), ctypes.byref(self.subs[i]),
                                           self.slots.data_ptr(), ctypes.byref(self.plans[i]), self.sh), "fa_plan_slots")
            self.eadj = None  # one positional entry buffer: the plans' entries are disjoint
            for i in live:
                self.plans[i].slots = self.slots.data_ptr()
                self.plans[i].slot_order = 0
                e = _plan_order(V, self.fm, self.adj, self.subs[i], self.plans[i], self.sh, self.eadj, order)
                self.eadj = e if e is not None else self.eadj

    def prepare(self):
        # the plans' FA_PLAN_AFFINE flags describe the coordinates they were planned on: vertices
        # moved in place since then re-run the library's per-cell affinity check (as gather_plan does)
        m = self.a.V.mesh
        now = _coords_version(m)
        if now != self._xver:
            self.fm = self.a.V._fa_mesh()  # mesh.x may be a new tensor
            if m.cell_type in (CellType.quadrilateral, CellType.hexahedron):
                for plan in self.plans:
                    _lib.check(self.L.fa_plan_check_affine(ctypes.byref(self.fm), ctypes.byref(plan), self.sh),
                               "fa_plan_check_affine")
            self._xver = now
        _lib.check(self.L.fa_gather_prepare(ctypes.byref(self.fm), ctypes.byref(self.ff), _lib.ptr(self.marker),
                                            self.work.data_ptr(), self.sh), "fa_gather_prepare")

    def rows(self, i: int):
        if self.plans[i].nchunks == 0:
            return
        _lib.check(self.L.fa_gather_rows(ctypes.byref(self.fm), ctypes.byref(self.ff), ctypes.byref(self.adj),
                                         ctypes.byref(self.plans[i]), _lib.ptr(self.marker), self.diagonal,
                                         self.work.data_ptr(), ctypes.byref(self.subs[i]), self.sh), "fa_gather_rows")


def tabulate_cells(a, c0: int = 0, ncells: int | None = None) -> torch.Tensor:
    """Element matrices [nc, nn*bs, nn*bs] (batched ffcx tabulate_tensor / AssembleElementGrad)."""
    V = a.V
    nc = V.mesh.num_cells - c0 if ncells is None else ncells
    nd = V.nn * V.bs
    Ae = torch.empty((nc, nd, nd), dtype=torch.float64, device=V.mesh.device)
    L = _lib.load()
    fm = V._fa_mesh()
    ff = _fa_form(a)
    _lib.check(L.fa_tabulate_cells(ctypes.byref(fm), ctypes.byref(ff), c0, nc, Ae.data_ptr(),
                                   _lib.stream_handle(V.mesh.device)), "fa_tabulate_cells")
    return Ae


def assemble_vector(L, b: torch.Tensor | None = None) -> torch.Tensor:
    """Residual of the form's constitutive law: b += int sigma(u):eps(v) dxx - int f.v dx
    (dolfinx.fem.assemble_vector of the reference F, FEniCSx/mechanic2d/asym_elasto_damage_model.cc:825;
    MFEM damIntegrator::AssembleElementVector :559-637). u, f are the form's `u` / `f` (None = 0)."""
    V = L.V
    if b is None:
        b = torch.zeros(V.num_dofs, dtype=torch.float64, device=V.mesh.device)
    Lb = _lib.load()
    fm = V._fa_mesh()
    ff = _fa_form(L)
    adj = V._fa_adjacency()
    _lib.check(Lb.fa_assemble_vector(ctypes.byref(fm), ctypes.byref(ff), ctypes.byref(adj), b.data_ptr(),
                                     _lib.stream_handle(V.mesh.device)), "fa_assemble_vector")
    return b


def apply_lifting(b: torch.Tensor, a: list, bcs: list, x0: list | None = None, alpha: float = 1.0, scale=None):
    """dolfinx apply_lifting: b -= alpha * A (g - x0) over constrained columns, with the cell
    matrices of a[0] (the reference calls it with alpha = -1, :827)."""
    if scale is not None:
        alpha = scale
    form_ = a[0]
    V = form_.V
    marker, g = _combine_bcs(V, bcs[0])
    if marker is None:
        return b
    x = None if not x0 else (x0[0].x if isinstance(x0[0], Function) else x0[0])
    Lb = _lib.load()
    fm = V._fa_mesh()
    ff = _fa_form(form_)
    adj = V._fa_adjacency()
    _lib.check(Lb.fa_apply_lifting(ctypes.byref(fm), ctypes.byref(ff), ctypes.byref(adj), b.data_ptr(),
                                   marker.data_ptr(), g.data_ptr(), _lib.ptr(x), float(alpha),
                                   _lib.stream_handle(V.mesh.device)), "fa_apply_lifting")
    return b


def set_bc(b: torch.Tensor, bcs: list, x0=None, alpha: float = 1.0, scale=None):
    """dolfinx set_bc: b[bc dofs] = alpha * (g - x0) (the reference: alpha = -1, x0 = u, :836)."""
    if scale is not None:
        alpha = scale
    if not bcs:
        return b
    V = bcs[0].V
    marker, g = _combine_bcs(V, bcs)
    x = None if x0 is None else (x0.x if isinstance(x0, Function) else x0)
    Lb = _lib.load()
    _lib.check(Lb.fa_set_bc(b.data_ptr(), b.numel(), marker.data_ptr(), g.data_ptr(), _lib.ptr(x), float(alpha),
                            _lib.stream_handle(V.mesh.device)), "fa_set_bc")
    return b
