"""XDMF mesh and mesh-tag files — the dolfinx.io.XDMFFile surface the reference reads its mesh with
(FEniCSx/mechanic2d/asym_elasto_damage_model.cc:155-162: ``read_mesh(..., "neper_dam")``,
``read_meshtags(mesh, "neper_dam_cells")`` / ``"neper_dam_facets"``; the cell tags set E per cell,
:543-545, the facet tags select the damaged edges, :363-367) and writes its output with (:549-560).

Layout as dolfinx writes it: a Uniform Grid named after the mesh (Topology + Geometry), and one
Uniform Grid per tag set (its own Topology of the tagged entities' vertices, the mesh's Geometry
by XInclude, and a cell-centred Attribute of the values). Heavy data: inline XML
(``XDMFFile.Encoding.ASCII``) and raw binary DataItems are read and XML is written. HDF5 heavy data
(dolfinx's default encoding) needs an HDF5 library, absent from this image (no h5py): such a file is
refused with a clear error, not misread. Vertex orders follow XDMF/VTK (quadrilaterals and hexahedra
counter-clockwise) and are converted to basix's on read, back on write.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass

import numpy as np
import torch

from .mesh import GDIM, NVERTS, CellType, Mesh, entities

_TOPO = {"Triangle": CellType.triangle, "Quadrilateral": CellType.quadrilateral,
         "Tetrahedron": CellType.tetrahedron, "Hexahedron": CellType.hexahedron}
_TOPO_NAME = {v: k for k, v in _TOPO.items()}
# entity topologies of the tag grids (facets of 2-D / 3-D cells, vertices)
_ENT = {"Polyvertex": 0, "PolyLine": 1, "Triangle": 2, "Quadrilateral": 2, "Tetrahedron": 3, "Hexahedron": 3}
# XDMF/VTK vertex order -> basix (the same permutation both ways)
_PERM = {CellType.quadrilateral: [0, 1, 3, 2], CellType.hexahedron: [0, 1, 3, 2, 4, 5, 7, 6]}


@dataclass
class MeshTags:
    """dolfinx.mesh.MeshTags: ``values[i]`` tags entity ``indices[i]`` of dimension ``dim``
    (entity ids as ``mesh.entities(mesh, dim)`` numbers them; cells for dim = tdim); indices sorted."""
    dim: int
    indices: torch.Tensor  # int32
    values: torch.Tensor  # int32
    name: str = "mesh_tags"

    def find(self, value: int) -> torch.Tensor:
        """Entities carrying ``value`` (dolfinx MeshTags::find)."""
        return self.indices[self.values == int(value)]


def _data_item(item: ET.Element, base: str) -> np.ndarray:
    dims = [int(d) for d in item.get("Dimensions", "").split()]
    fmt = item.get("Format", "XML")
    ntype = item.get("NumberType", item.get("DataType", "Float"))
    prec = int(item.get("Precision", "8" if ntype == "Float" else "4"))
    dt = {("Float", 8): np.float64, ("Float", 4): np.float32, ("Int", 4): np.int32, ("Int", 8): np.int64,
          ("UInt", 4): np.uint32, ("UInt", 8): np.uint64, ("Char", 1): np.int8, ("UChar", 1): np.uint8}.get((ntype, prec))
    if dt is None:
        raise ValueError(f"XDMF DataItem of type {ntype}/{prec} not supported")
    n = int(np.prod(dims)) if dims else None
    if fmt == "XML":
        a = np.array((item.text or "").split(), dtype=np.float64 if ntype == "Float" else np.int64).astype(dt)
    elif fmt == "Binary":
        path = (item.text or "").strip()
        path = path if os.path.isabs(path) else os.path.join(base, path)
        endian = {"Little": "<", "Big": ">"}.get(item.get("Endian", "Native"), "=")
        a = np.fromfile(path, dtype=np.dtype(dt).newbyteorder(endian), count=n if n else -1,
                        offset=int(item.get("Seek", "0"))).astype(dt)
    elif fmt == "HDF":
        raise NotImplementedError(
            f"XDMF heavy data in HDF5 ({(item.text or '').strip()}): no HDF5 library in this environment; "
            "write the file with XDMFFile.Encoding.ASCII (inline XML) instead")
    else:
        raise ValueError(f"XDMF DataItem format {fmt} not supported")
    if n is not None and a.size != n:
        raise ValueError(f"XDMF DataItem holds {a.size} values, Dimensions say {dims}")
    return a.reshape(dims) if dims else a


class XDMFFile:
    """dolfinx.io.XDMFFile(comm, path, mode) on one process: ``read_mesh(name)``,
    ``read_meshtags(mesh, name)``; ``write_mesh(mesh, name)``, ``write_meshtags(tags, mesh)`` (ASCII
    heavy data; the file is written on close / leaving the ``with`` block)."""

    def __init__(self, path: str, mode: str = "r"):
        if mode not in ("r", "w"):
            raise ValueError(f"mode {mode!r}: 'r' or 'w'")
        self.path, self.mode = path, mode
        self._base = os.path.dirname(os.path.abspath(path))
        self._grids = []
        if mode == "r":
            root = ET.parse(path).getroot()
            dom = root.find("Domain")
            if dom is None:
                raise ValueError(f"{path}: no XDMF Domain")
            self._dom = dom
            self._grid_list = dom.findall("Grid")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------------------------------- read
    def _grid(self, name: str) -> ET.Element:
        for g in self._grid_list:
            if g.get("Name") == name:
                return g
            for sub in g.findall("Grid"):  # a Collection of time steps / blocks: the first match
                if sub.get("Name") == name:
                    return sub
        raise KeyError(f"{self.path}: no Grid named {name!r} (have {[g.get('Name') for g in self._grid_list]})")

    def _geometry(self, g: ET.Element) -> np.ndarray:
        geo = g.find("Geometry")
        if geo is None:  # the tag grids include the mesh's geometry (xi:include): the first Geometry
            for other in self._grid_list:
                geo = other.find("Geometry")
                if geo is not None:
                    break
        if geo is None:
            raise ValueError(f"{self.path}: no Geometry")
        x = _data_item(geo.find("DataItem"), self._base).astype(np.float64)
        gt = geo.get("GeometryType", "XYZ")
        return x.reshape(-1, len(gt)) if gt in ("XY", "XYZ") else x

    def read_mesh(self, name: str = "mesh", device=None) -> Mesh:
        """The grid's cells and vertex coordinates (the cell tags stay None: ``read_meshtags``)."""
        g = self._grid(name)
        topo = g.find("Topology")
        ct = _TOPO.get(topo.get("TopologyType"))
        if ct is None:
            raise ValueError(f"{self.path}: topology {topo.get('TopologyType')} not supported")
        cells = _data_item(topo.find("DataItem"), self._base).astype(np.int64).reshape(-1, NVERTS[ct])
        x = self._geometry(g)
        gd = GDIM[ct]
        if x.shape[1] < gd:
            raise ValueError(f"{self.path}: {x.shape[1]}-D geometry for a {ct.name} mesh")
        if ct in _PERM:
            cells = cells[:, _PERM[ct]]
        m = Mesh(ct, torch.tensor(np.ascontiguousarray(x[:, :gd])), torch.tensor(cells.astype(np.int32)), None, None)
        return m.to(device) if device is not None else m

    def read_meshtags(self, mesh: Mesh, name: str) -> MeshTags:
        """Tags of the entities listed in grid ``name``: each tagged entity is found in
        ``mesh.entities(mesh, dim)`` by its vertex set (dolfinx read_meshtags)."""
        g = self._grid(name)
        topo = g.find("Topology")
        tt = topo.get("TopologyType")
        if tt not in _ENT:
            raise ValueError(f"{self.path}: tag topology {tt} not supported")
        dim = _ENT[tt]
        ev = _data_item(topo.find("DataItem"), self._base).astype(np.int64)
        npe = int(topo.get("NodesPerElement", "0") or 0)
        ev = ev.reshape(-1, npe) if npe else ev.reshape(ev.shape[0], -1)
        att = g.find("Attribute")
        if att is None:
            raise ValueError(f"{self.path}: tag grid {name!r} has no Attribute")
        vals = _data_item(att.find("DataItem"), self._base).astype(np.int64).reshape(-1)
        if vals.shape[0] != ev.shape[0]:
            raise ValueError(f"{self.path}: {ev.shape[0]} tagged entities, {vals.shape[0]} values")
        if dim > mesh.tdim:
            raise ValueError(f"{self.path}: {dim}-D tags on a {mesh.tdim}-D mesh")
        ents, _ = entities(mesh, dim) if dim < mesh.tdim else (mesh.cells.to(torch.int64), None)
        dev = mesh.x.device
        nv = mesh.num_vertices
        key_ent = torch.sort(ents.to(dev), dim=1).values
        key_tag = torch.sort(torch.tensor(ev, device=dev), dim=1).values
        if key_ent.shape[1] != key_tag.shape[1]:
            raise ValueError(f"{self.path}: tagged entities have {key_tag.shape[1]} vertices, the mesh's "
                             f"dimension-{dim} entities {key_ent.shape[1]}")
        # match sorted vertex tuples through one int64 key per tuple (mixed radix in the vertex count)
        def pack(k):
            out = torch.zeros(k.shape[0], dtype=torch.int64, device=dev)
            for c in range(k.shape[1]):
                out = out * nv + k[:, c]
            return out

        if nv ** key_ent.shape[1] >= 2 ** 63:
            raise ValueError("entity keys overflow int64")
        ke, kt = pack(key_ent), pack(key_tag)
        order = torch.argsort(ke)
        pos = torch.searchsorted(ke[order], kt)
        pos = pos.clamp(max=max(ke.numel() - 1, 0))
        found = ke[order][pos] == kt if ke.numel() else torch.zeros_like(kt, dtype=torch.bool)
        if not bool(found.all()):
            raise ValueError(f"{self.path}: {int((~found).sum())} tagged entities of {name!r} are not entities of the mesh")
        idx = order[pos]
        srt = torch.argsort(idx)
        return MeshTags(dim, idx[srt].to(torch.int32), torch.tensor(vals, device=dev)[srt].to(torch.int32), name)

    # ------------------------------------------------------------------------------------ write
    def write_mesh(self, mesh: Mesh, name: str = "mesh"):
        if self.mode != "w":
            raise ValueError("file opened for reading")
        ct = CellType(mesh.cell_type)
        cells = mesh.cells.cpu().numpy().astype(np.int64)
        if ct in _PERM:
            cells = cells[:, _PERM[ct]]
        self._mesh_name = name
        self._x = mesh.x.cpu().numpy()
        self._grids.append(("mesh", name, ct, cells, None))

    def write_meshtags(self, tags: MeshTags, mesh: Mesh):
        if self.mode != "w":
            raise ValueError("file opened for reading")
        dim = tags.dim
        if dim == mesh.tdim:
            ev = mesh.cells.cpu().numpy().astype(np.int64)[tags.indices.cpu().numpy()]
            ct = CellType(mesh.cell_type)
            if ct in _PERM:
                ev = ev[:, _PERM[ct]]
            tt = _TOPO_NAME[ct]
        else:
            ents, _ = entities(mesh, dim)
            ev = ents.cpu().numpy()[tags.indices.cpu().numpy()]
            tt = {0: "Polyvertex", 1: "PolyLine"}.get(dim)
            if tt is None:  # faces of 3-D cells: triangles or (hexahedra) quadrilaterals in VTK order
                tt = "Triangle" if ev.shape[1] == 3 else "Quadrilateral"
        self._grids.append(("tags", tags.name, tt, ev, tags.values.cpu().numpy()))

    @staticmethod
    def _item(parent, arr: np.ndarray, number: str):
        it = ET.SubElement(parent, "DataItem", Dimensions=" ".join(str(d) for d in arr.shape), Format="XML")
        if number == "Int":
            it.set("NumberType", "Int")
        else:
            it.set("Precision", "8")
        fmt = (lambda v: repr(float(v))) if number != "Int" else (lambda v: str(int(v)))
        rows = arr.reshape(arr.shape[0], -1)
        it.text = "\n" + "\n".join(" ".join(fmt(v) for v in r) for r in rows) + "\n"
        return it

    def close(self):
        if self.mode != "w" or not self._grids:
            return
        root = ET.Element("Xdmf", Version="3.0")
        root.set("xmlns:xi", "https://www.w3.org/2001/XInclude")
        dom = ET.SubElement(root, "Domain")
        for kind, name, ct, top, vals in self._grids:
            g = ET.SubElement(dom, "Grid", Name=name, GridType="Uniform")
            tname = _TOPO_NAME[ct] if kind == "mesh" else ct
            t = ET.SubElement(g, "Topology", TopologyType=tname, NumberOfElements=str(top.shape[0]),
                              NodesPerElement=str(top.shape[1]))
            self._item(t, top, "Int")
            geo = ET.SubElement(g, "Geometry", GeometryType="XY" if self._x.shape[1] == 2 else "XYZ")
            self._item(geo, self._x, "Float")
            if kind == "tags":
                a = ET.SubElement(g, "Attribute", Name=name, AttributeType="Scalar", Center="Cell")
                self._item(a, vals.reshape(-1, 1), "Int")
        ET.ElementTree(root).write(self.path, xml_declaration=True, encoding="utf-8")
        self._grids = []
