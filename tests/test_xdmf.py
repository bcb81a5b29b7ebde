"""XDMF mesh / mesh-tag files (femasm.io.XDMFFile), the reader the reference's C++ driver uses
(FEniCSx/mechanic2d/asym_elasto_damage_model.cc:155-162, cell tags -> E at :543-545, facet tags ->
damaged edges at :363-367). The reference ships no XDMF file (its data/neper_dam.xdmf is generated
outside the repository) and this image has no HDF5 library, so these tests pin the ASCII / binary
encodings: write -> read round trips on every cell type, the reference's own square.msh carried
through XDMF with its physical groups, a hand-written dolfinx-layout file (VTK vertex order,
xi:include'd geometry), and the refusal of HDF5 heavy data."""
import os

import numpy as np
import pytest
import torch

from femasm import io, materials, mesh

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _tags(dim, idx, vals, name):
    return io.MeshTags(dim, torch.as_tensor(idx, dtype=torch.int32), torch.as_tensor(vals, dtype=torch.int32), name)


@pytest.mark.parametrize("ct,n", [(3, (4, 3)), (4, (3, 2)), (-4, (2, 2, 1)), (8, (2, 1, 2))])
def test_round_trip(tmp_path, ct, n):
    m = mesh.create_unit_square(*n, cell_type=ct) if len(n) == 2 else mesh.create_unit_cube(*n, cell_type=ct)
    cell_vals = (np.arange(m.num_cells) * 7 + 3) % 11
    cells = _tags(m.tdim, np.arange(m.num_cells), cell_vals, "m_cells")
    fdim = m.tdim - 1
    ext = mesh.exterior_facets(m)
    facets = _tags(fdim, ext.numpy(), (np.arange(ext.numel()) % 5) + 1, "m_facets")
    path = str(tmp_path / "m.xdmf")
    with io.XDMFFile(path, "w") as f:
        f.write_mesh(m, "m")
        f.write_meshtags(cells, m)
        f.write_meshtags(facets, m)
    with io.XDMFFile(path, "r") as f:
        r = f.read_mesh("m")
        rc = f.read_meshtags(r, "m_cells")
        rf = f.read_meshtags(r, "m_facets")
    assert r.cell_type == m.cell_type
    assert torch.equal(r.x, m.x) and torch.equal(r.cells, m.cells)
    assert rc.dim == m.tdim and torch.equal(rc.indices, cells.indices) and torch.equal(rc.values, cells.values)
    assert rf.dim == fdim and torch.equal(rf.indices, facets.indices.sort().values)
    assert torch.equal(rf.values, facets.values[torch.argsort(facets.indices)])
    for v in range(1, 6):  # MeshTags.find, as the reference selects its damaged edges
        assert torch.equal(rf.find(v), facets.indices[facets.values == v].sort().values)


def test_square_msh_through_xdmf(tmp_path):
    """The reference's own mesh (common/data/square.msh) with its physical groups as cell tags:
    XDMF carries the same cells, and E per cell from the tags equals E from the Gmsh tags."""
    g = mesh.read_gmsh(os.path.join(GOLDEN, "square.msh"), gdim=2)
    tags = _tags(2, np.arange(g.num_cells), g.cell_tags.numpy(), "square_cells")
    path = str(tmp_path / "square.xdmf")
    with io.XDMFFile(path, "w") as f:
        f.write_mesh(g, "square")
        f.write_meshtags(tags, g)
    with io.XDMFFile(path, "r") as f:
        m = f.read_mesh("square")
        t = f.read_meshtags(m, "square_cells")
    assert torch.equal(m.cells, g.cells) and torch.allclose(m.x, g.x, rtol=0, atol=0)
    E = materials.e_from_cell_tags(t, m.num_cells)
    ref = torch.tensor(materials.e_range()[g.cell_tags.numpy() % 200])
    assert torch.equal(E, ref)


DOLFINX_STYLE = """<?xml version="1.0"?>
<!DOCTYPE Xdmf SYSTEM "Xdmf.dtd" []>
<Xdmf Version="3.0" xmlns:xi="https://www.w3.org/2001/XInclude">
  <Domain>
    <Grid Name="quads" GridType="Uniform">
      <Topology TopologyType="Quadrilateral" NumberOfElements="2" NodesPerElement="4">
        <DataItem Dimensions="2 4" NumberType="Int" Format="XML">
          0 1 4 3
          1 2 5 4
        </DataItem>
      </Topology>
      <Geometry GeometryType="XY">
        <DataItem Dimensions="6 2" Format="XML">
          0 0  1 0  2 0
          0 1  1 1  2 1
        </DataItem>
      </Geometry>
    </Grid>
    <Grid Name="quads_cells" GridType="Uniform">
      <xi:include xpointer="xpointer(/Xdmf/Domain/Grid[@GridType='Uniform'][1]/Geometry)" />
      <Topology TopologyType="Quadrilateral" NumberOfElements="2" NodesPerElement="4">
        <DataItem Dimensions="2 4" NumberType="Int" Format="XML">1 2 5 4 0 1 4 3</DataItem>
      </Topology>
      <Attribute Name="quads_cells" AttributeType="Scalar" Center="Cell">
        <DataItem Dimensions="2 1" NumberType="Int" Format="XML">17 9</DataItem>
      </Attribute>
    </Grid>
    <Grid Name="quads_facets" GridType="Uniform">
      <xi:include xpointer="xpointer(/Xdmf/Domain/Grid[@GridType='Uniform'][1]/Geometry)" />
      <Topology TopologyType="PolyLine" NumberOfElements="2" NodesPerElement="2">
        <DataItem Dimensions="2 2" NumberType="Int" Format="XML">2 5 3 0</DataItem>
      </Topology>
      <Attribute Name="quads_facets" AttributeType="Scalar" Center="Cell">
        <DataItem Dimensions="2 1" NumberType="Int" Format="XML">4 3</DataItem>
      </Attribute>
    </Grid>
  </Domain>
</Xdmf>
"""


def test_dolfinx_layout(tmp_path):
    """VTK (counter-clockwise) quadrilaterals become basix's tensor order; tag grids with the mesh's
    geometry by xi:include; tags listed out of cell order come back sorted by entity."""
    path = tmp_path / "quads.xdmf"
    path.write_text(DOLFINX_STYLE)
    with io.XDMFFile(str(path)) as f:
        m = f.read_mesh("quads")
        ct = f.read_meshtags(m, "quads_cells")
        ft = f.read_meshtags(m, "quads_facets")
    assert m.cell_type == mesh.CellType.quadrilateral
    assert m.cells.tolist() == [[0, 1, 3, 4], [1, 2, 4, 5]]  # basix: (0,0),(1,0),(0,1),(1,1)
    assert ct.indices.tolist() == [0, 1] and ct.values.tolist() == [9, 17]
    ev, _ = mesh.entities(m, 1)
    got = {tuple(ev[i].tolist()): int(v) for i, v in zip(ft.indices.tolist(), ft.values.tolist())}
    assert got == {(2, 5): 4, (0, 3): 3}


def test_binary_heavy_data(tmp_path):
    x = np.array([[0, 0], [1, 0], [0, 1]], dtype=np.float64)
    c = np.array([[0, 1, 2]], dtype=np.int32)
    x.tofile(tmp_path / "x.bin")
    c.tofile(tmp_path / "c.bin")
    (tmp_path / "t.xdmf").write_text(f"""<?xml version="1.0"?>
<Xdmf Version="3.0"><Domain><Grid Name="t" GridType="Uniform">
<Topology TopologyType="Triangle" NumberOfElements="1" NodesPerElement="3">
<DataItem Dimensions="1 3" NumberType="Int" Precision="4" Format="Binary" Endian="Little">c.bin</DataItem></Topology>
<Geometry GeometryType="XY"><DataItem Dimensions="3 2" Precision="8" Format="Binary" Endian="Little">x.bin</DataItem></Geometry>
</Grid></Domain></Xdmf>""")
    m = io.XDMFFile(str(tmp_path / "t.xdmf")).read_mesh("t")
    assert m.cells.tolist() == [[0, 1, 2]] and m.x.numpy().tolist() == x.tolist()


def test_hdf5_heavy_data_refused(tmp_path):
    (tmp_path / "h.xdmf").write_text("""<?xml version="1.0"?>
<Xdmf Version="3.0"><Domain><Grid Name="mesh" GridType="Uniform">
<Topology TopologyType="Triangle" NumberOfElements="2" NodesPerElement="3">
<DataItem Dimensions="2 3" NumberType="Int" Format="HDF">h.h5:/Mesh/mesh/topology</DataItem></Topology>
<Geometry GeometryType="XY"><DataItem Dimensions="4 2" Format="HDF">h.h5:/Mesh/mesh/geometry</DataItem></Geometry>
</Grid></Domain></Xdmf>""")
    with pytest.raises(NotImplementedError, match="HDF5"):
        io.XDMFFile(str(tmp_path / "h.xdmf")).read_mesh("mesh")


def test_unknown_entities_refused(tmp_path):
    m = mesh.create_unit_square(2, 2, cell_type=3)
    path = str(tmp_path / "m.xdmf")
    with io.XDMFFile(path, "w") as f:
        f.write_mesh(m, "m")
    txt = open(path).read()
    bad = txt.replace("</Domain>", """<Grid Name="bad" GridType="Uniform"><Topology TopologyType="PolyLine"
NumberOfElements="1" NodesPerElement="2"><DataItem Dimensions="1 2" NumberType="Int" Format="XML">0 8</DataItem>
</Topology><Attribute Name="bad" Center="Cell"><DataItem Dimensions="1 1" NumberType="Int" Format="XML">1</DataItem>
</Attribute></Grid></Domain>""")
    open(path, "w").write(bad)
    with io.XDMFFile(path) as f:
        r = f.read_mesh("m")
        with pytest.raises(ValueError, match="not entities of the mesh"):
            f.read_meshtags(r, "bad")
