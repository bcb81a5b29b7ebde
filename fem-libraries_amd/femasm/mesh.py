"""Meshes held in torch tensors — the dolfinx.mesh surface the reference uses.

Structured generators mirror dolfinx ``create_unit_square`` / ``create_unit_cube`` (the
synthetic inputs of BASELINE.json's configs) and the Gmsh 2.2 reader loads the
reference's own ``common/data/square.msh`` format (cell tags = physical groups, as
``gmshio``/MFEM read them: FEniCSx/mechanic2d/asym_elasto_damage_model.cc:152-162,
MFEM/mechanic2d/asym_elasto_damage_model.cc:1017-1020).

Reference-cell vertex orderings are basix's: triangle (0,0),(1,0),(0,1); tetrahedron adds
(0,0,1); quadrilateral (0,0),(1,0),(0,1),(1,1); hexahedron the tensor ordering v = i + 2j + 4k.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import IntEnum

import torch


class CellType(IntEnum):
    """dolfinx.mesh.CellType values."""
    triangle = 3
    quadrilateral = 4
    tetrahedron = -4
    hexahedron = 8


GDIM = {CellType.triangle: 2, CellType.quadrilateral: 2, CellType.tetrahedron: 3, CellType.hexahedron: 3}
NVERTS = {CellType.triangle: 3, CellType.quadrilateral: 4, CellType.tetrahedron: 4, CellType.hexahedron: 8}

# basix reference sub-entities: edges as vertex pairs, faces as vertex tuples (hexahedron faces in
# the face's own tensor order v0, v1, v2, v3; tetrahedron face i is opposite vertex i)
EDGES = {
    CellType.triangle: ((1, 2), (0, 2), (0, 1)),
    CellType.tetrahedron: ((2, 3), (1, 3), (1, 2), (0, 3), (0, 2), (0, 1)),
    CellType.quadrilateral: ((0, 1), (0, 2), (1, 3), (2, 3)),
    CellType.hexahedron: ((0, 1), (0, 2), (0, 4), (1, 3), (1, 5), (2, 3), (2, 6), (3, 7), (4, 5), (4, 6), (5, 7), (6, 7)),
}
HEX_FACES = ((0, 1, 2, 3), (0, 1, 4, 5), (0, 2, 4, 6), (1, 3, 5, 7), (2, 3, 6, 7), (4, 5, 6, 7))
TET_FACES = ((1, 2, 3), (0, 2, 3), (0, 1, 3), (0, 1, 2))
REF_VERTS = {
    CellType.triangle: ((0, 0), (1, 0), (0, 1)),
    CellType.tetrahedron: ((0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1)),
    CellType.quadrilateral: ((0, 0), (1, 0), (0, 1), (1, 1)),
    CellType.hexahedron: tuple((b & 1, (b >> 1) & 1, (b >> 2) & 1) for b in range(8)),
}


def sub_entities(ct, dim: int) -> tuple:
    """Local vertex tuples of a cell's sub-entities of dimension dim (basix numbering)."""
    ct = CellType(ct)
    tdim = GDIM[ct]
    if dim == 0:
        return tuple((v,) for v in range(NVERTS[ct]))
    if dim == tdim:
        return (tuple(range(NVERTS[ct])),)
    if dim == 1:
        return EDGES[ct]
    if dim == 2 and tdim == 3:
        return TET_FACES if ct == CellType.tetrahedron else HEX_FACES
    raise ValueError(f"no sub-entities of dimension {dim} for {ct.name}")


def _facet_edges(ct):
    """Edges of each facet of a 3-D cell, as local vertex pairs (hexahedron faces: the 4 sides, not
    the diagonals)."""
    if CellType(ct) == CellType.tetrahedron:
        return tuple(((f[0], f[1]), (f[0], f[2]), (f[1], f[2])) for f in TET_FACES)
    return tuple(((f[0], f[1]), (f[0], f[2]), (f[1], f[3]), (f[2], f[3])) for f in HEX_FACES)


@dataclass
class Mesh:
    cell_type: CellType
    x: torch.Tensor  # [nverts, gdim] float64 vertex coordinates
    cells: torch.Tensor  # [ncells, nverts_per_cell] int32 geometry / topology dofmap
    cell_tags: torch.Tensor | None = None  # [ncells] int32 physical tags (E per tag)
    structured: dict | None = field(default=None, repr=False)  # lattice info for fast dofmaps

    @property
    def gdim(self) -> int:
        return GDIM[self.cell_type]

    @property
    def tdim(self) -> int:
        return GDIM[self.cell_type]

    @property
    def num_cells(self) -> int:
        return int(self.cells.shape[0])

    @property
    def num_vertices(self) -> int:
        return int(self.x.shape[0])

    @property
    def device(self):
        return self.x.device

    def to(self, device) -> "Mesh":
        return Mesh(self.cell_type, self.x.to(device), self.cells.to(device),
                    None if self.cell_tags is None else self.cell_tags.to(device), self.structured)


def _lattice_vertices(n, lengths, device):
    axes = [torch.linspace(0.0, L, k + 1, dtype=torch.float64, device=device) for k, L in zip(n, lengths)]
    grids = torch.meshgrid(*reversed(axes), indexing="ij")  # slowest = last axis
    cols = [g.reshape(-1) for g in reversed(grids)]
    return torch.stack(cols, dim=1).contiguous()


def create_unit_square(nx: int, ny: int, cell_type: CellType = CellType.triangle, diagonal: str = "right",
                       device=None) -> Mesh:
    return create_rectangle((1.0, 1.0), (nx, ny), cell_type, diagonal, device)


def create_rectangle(lengths, n, cell_type: CellType = CellType.triangle, diagonal: str = "right", device=None) -> Mesh:
    """Structured rectangle [0,Lx]x[0,Ly] with nx*ny squares; triangles split each square along
    the diagonal from (i,j) to (i+1,j+1) ("right") or (i+1,j) to (i,j+1) ("left")."""
    nx, ny = n
    cell_type = CellType(cell_type)
    x = _lattice_vertices((nx, ny), lengths, device)
    i = torch.arange(nx, device=device, dtype=torch.int64)
    j = torch.arange(ny, device=device, dtype=torch.int64)
    J, I = torch.meshgrid(j, i, indexing="ij")
    v0 = (I + (nx + 1) * J).reshape(-1)
    v1, v2, v3 = v0 + 1, v0 + nx + 1, v0 + nx + 2
    if cell_type == CellType.quadrilateral:
        cells = torch.stack([v0, v1, v2, v3], 1)
    elif cell_type == CellType.triangle:
        if diagonal == "right":
            t = torch.stack([torch.stack([v0, v1, v3], 1), torch.stack([v0, v2, v3], 1)], 1)
        else:
            t = torch.stack([torch.stack([v0, v1, v2], 1), torch.stack([v1, v2, v3], 1)], 1)
        cells = t.reshape(-1, 3)
    else:
        raise ValueError(f"2-D cell type expected, got {cell_type}")
    return Mesh(cell_type, x, cells.to(torch.int32).contiguous(), None,
                dict(kind="rect", n=(nx, ny), lengths=tuple(lengths), diagonal=diagonal))


# Kuhn subdivision of a cube into 6 tetrahedra sharing the diagonal v0-v7 (dolfinx
# create_unit_cube(..., CellType.tetrahedron)); local cube vertex v = i + 2j + 4k.
KUHN_TETS = ((0, 1, 3, 7), (0, 1, 7, 5), (0, 5, 7, 4), (0, 3, 2, 7), (0, 6, 4, 7), (0, 2, 6, 7))


def create_unit_cube(nx: int, ny: int, nz: int, cell_type: CellType = CellType.tetrahedron, device=None) -> Mesh:
    return create_box((1.0, 1.0, 1.0), (nx, ny, nz), cell_type, device)


def create_box(lengths, n, cell_type: CellType = CellType.tetrahedron, device=None, z_range=None) -> Mesh:
    """Structured box with nx*ny*nz cubes (6 Kuhn tetrahedra or 1 hexahedron each).
    ``z_range=(k0, k1)`` builds only cube layers k0..k1-1 with the GLOBAL vertex numbering
    of the full box (used to shard the mesh by slabs)."""
    nx, ny, nz = n
    cell_type = CellType(cell_type)
    x = _lattice_vertices((nx, ny, nz), lengths, device)
    k0, k1 = (0, nz) if z_range is None else z_range
    i = torch.arange(nx, device=device, dtype=torch.int64)
    j = torch.arange(ny, device=device, dtype=torch.int64)
    k = torch.arange(k0, k1, device=device, dtype=torch.int64)
    K, J, I = torch.meshgrid(k, j, i, indexing="ij")
    sx, sy = 1, nx + 1
    sz = (nx + 1) * (ny + 1)
    base = (I + sx * 0 + sy * J + sz * K).reshape(-1)
    cv = [base + (b & 1) * sx + ((b >> 1) & 1) * sy + ((b >> 2) & 1) * sz for b in range(8)]
    if cell_type == CellType.hexahedron:
        cells = torch.stack(cv, 1)
    elif cell_type == CellType.tetrahedron:
        tets = [torch.stack([cv[a] for a in t], 1) for t in KUHN_TETS]
        cells = torch.stack(tets, 1).reshape(-1, 4)
    else:
        raise ValueError(f"3-D cell type expected, got {cell_type}")
    return Mesh(cell_type, x, cells.to(torch.int32).contiguous(), None,
                dict(kind="box", n=(nx, ny, nz), lengths=tuple(lengths), z_range=(k0, k1)))


_GMSH_TYPES = {2: CellType.triangle, 3: CellType.quadrilateral, 4: CellType.tetrahedron, 5: CellType.hexahedron}


def read_gmsh(path: str, gdim: int | None = None, device=None) -> Mesh:
    """Read a Gmsh 2.2 ASCII file (the format of the reference's common/data/square.msh).
    Keeps the highest-dimension cells; cell_tags are the physical groups. Vertex order is
    converted to basix's (Gmsh quads/hexes are counter-clockwise)."""
    with open(path) as fh:
        lines = [ln.strip() for ln in fh]
    i = lines.index("$Nodes")
    nnod = int(lines[i + 1])
    ids, coords = [], []
    for ln in lines[i + 2:i + 2 + nnod]:
        p = ln.split()
        ids.append(int(p[0]))
        coords.append([float(v) for v in p[1:4]])
    i = lines.index("$Elements")
    nel = int(lines[i + 1])
    elems = {}
    for ln in lines[i + 2:i + 2 + nel]:
        p = [int(v) for v in ln.split()]
        et, ntag = p[1], p[2]
        if et in _GMSH_TYPES:
            elems.setdefault(et, []).append((p[3], p[3 + ntag:]))
    et = max(elems, key=lambda t: GDIM[_GMSH_TYPES[t]] * 10 + (1 if t in (3, 5) else 0))
    ct = _GMSH_TYPES[et]
    g = gdim or GDIM[ct]
    used = sorted({n for _, ns in elems[et] for n in ns})
    remap = {old: new for new, old in enumerate(used)}
    pos = {nid: k for k, nid in enumerate(ids)}
    x = torch.tensor([coords[pos[n]][:g] for n in used], dtype=torch.float64)
    perm = {CellType.quadrilateral: [0, 1, 3, 2], CellType.hexahedron: [0, 1, 3, 2, 4, 5, 7, 6]}.get(ct)
    cells = []
    for _, ns in elems[et]:
        c = [remap[n] for n in ns]
        if perm:
            c = [c[k] for k in perm]
        cells.append(c)
    cells = torch.tensor(cells, dtype=torch.int32)
    tags = torch.tensor([t for t, _ in elems[et]], dtype=torch.int32)
    m = Mesh(ct, x, cells, tags, None)
    return m.to(device) if device is not None else m


def _unique_rows(t: torch.Tensor):
    """(unique sorted rows of an int64 tensor [n, k], inverse index [n])."""
    if t.shape[1] == 1:
        return torch.unique(t[:, 0], return_inverse=True)
    return torch.unique(t, dim=0, return_inverse=True)


def entities(mesh: Mesh, dim: int):
    """Topology of dimension dim (dolfinx mesh.topology.create_entities): (vertex tuples of the
    entities [ne, k] int64, each cell's entity ids [ncells, n_local] int64). Entities are numbered in
    the lexicographic order of their sorted vertex tuples; dim 0 entities are the vertices themselves
    (mesh.x rows). Cached on the mesh."""
    cache = mesh.__dict__.setdefault("_entities", {})
    if dim in cache:
        return cache[dim]
    c = mesh.cells.to(torch.int64)
    if dim == 0:
        ent = torch.arange(mesh.num_vertices, device=c.device, dtype=torch.int64).reshape(-1, 1)
        out = (ent, c)
    else:
        S = torch.tensor(sub_entities(mesh.cell_type, dim), dtype=torch.int64, device=c.device)  # [nl, k]
        tup = torch.sort(c[:, S], dim=-1).values  # [nc, nl, k]
        ent, inv = _unique_rows(tup.reshape(-1, S.shape[1]))
        out = (ent.reshape(-1, S.shape[1]), inv.reshape(c.shape[0], S.shape[0]))
    cache[dim] = out
    return out


def exterior_facets(mesh: Mesh) -> torch.Tensor:
    """Facet ids (entities(mesh, tdim - 1)) that belong to exactly one cell (dolfinx
    exterior_facet_indices on one process)."""
    _, cf = entities(mesh, mesh.tdim - 1)
    cnt = torch.bincount(cf.reshape(-1), minlength=int(cf.max()) + 1 if cf.numel() else 0)
    return torch.nonzero(cnt == 1, as_tuple=False).reshape(-1)


def locate_entities_boundary(mesh: Mesh, dim: int, marker) -> torch.Tensor:
    """dolfinx.mesh.locate_entities_boundary: the entities of dimension dim attached to an exterior
    facet (the facets themselves, or their edges / vertices) whose vertices ALL satisfy
    marker(x[gdim, n]). Returns sorted entity ids (int32) of entities(mesh, dim); for dim 0 these are
    vertex indices. The reference calls it with dim 0 (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:627-636,
    :651-660)."""
    tdim = mesh.tdim
    if not 0 <= dim < tdim:
        raise ValueError(f"boundary entities have dimension 0 .. {tdim - 1}, not {dim}")
    fverts, _ = entities(mesh, tdim - 1)
    ext = exterior_facets(mesh)
    dev = mesh.x.device
    if dim == tdim - 1:
        cand = ext
        cand_verts = fverts[ext]
    elif dim == 0:
        cand = torch.unique(fverts[ext].reshape(-1))
        cand_verts = cand.reshape(-1, 1)
    else:  # dim 1 of a 3-D mesh: the edges of the exterior facets
        # an exterior facet's vertices in its cell's local order give its edges (hexahedron faces:
        # the sides only); locate each exterior facet in one of its cells
        _, cf = entities(mesh, tdim - 1)
        c = mesh.cells.to(torch.int64)
        flat = cf.reshape(-1)
        is_ext = torch.zeros(fverts.shape[0], dtype=torch.bool, device=dev)
        is_ext[ext] = True
        hit = torch.nonzero(is_ext[flat], as_tuple=False).reshape(-1)
        cell, lf = hit // cf.shape[1], hit % cf.shape[1]
        FE = torch.tensor(_facet_edges(mesh.cell_type), dtype=torch.int64, device=dev)  # [nf, ne, 2]
        ev = c[cell[:, None, None], FE[lf]]  # [n, ne, 2]
        ev = torch.sort(ev.reshape(-1, 2), dim=-1).values
        everts, _ = entities(mesh, 1)
        # ids of these edges in entities(mesh, 1): search the sorted unique tuples
        key_all = everts[:, 0] * mesh.num_vertices + everts[:, 1]
        key = torch.unique(ev[:, 0] * mesh.num_vertices + ev[:, 1])
        cand = torch.searchsorted(key_all, key)
        cand_verts = everts[cand]
    ok = marker(mesh.x.T)
    ok = torch.as_tensor(ok, device=dev).to(torch.bool)
    keep = ok[cand_verts].all(dim=1)
    return cand[keep].to(torch.int32)


def locate_vertices(mesh: Mesh, marker) -> torch.Tensor:
    """Vertices whose coordinates satisfy marker(x) (x as [gdim, n], dolfinx convention)."""
    keep = marker(mesh.x.T)
    return torch.nonzero(keep, as_tuple=False).reshape(-1).to(torch.int32)
