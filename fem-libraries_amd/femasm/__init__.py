"""femasm — MI355X-native element-stiffness assembly (the hot path of SalzmanA/fem-libraries).

Submodules mirror the reference's dolfinx surface: ``mesh`` (meshes in torch tensors),
``fem`` (function spaces, forms, Dirichlet BCs, create_matrix / assemble_matrix), ``la``
(the BSR global matrix), ``io`` (XDMF meshes and mesh tags). Numerics run in libfemasm.so
(hand-written HIP for gfx950).
"""
from . import fem, io, la, mesh  # noqa: F401
from ._lib import FemasmError, load  # noqa: F401

__version__ = "0.1.0"
