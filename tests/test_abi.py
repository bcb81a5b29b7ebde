"""CPU checks of the drop-in boundary: libfemasm.so loads and exports every entry point that
include/femasm.h declares (no compute calls: no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "femasm.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fa_[a-z_]+)\s*\(", txt)))


def test_header_declares_boundary():
    names = declared_functions()
    for n in ["fa_assemble_matrix", "fa_tabulate_cells", "fa_sparsity_count", "fa_sparsity_fill",
              "fa_build_adjacency", "fa_assemble_vector", "fa_apply_lifting", "fa_set_bc", "fa_last_error"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from femasm import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libfemasm.so not built (run __graft_entry__.build())")
    L = ctypes.CDLL(_lib.LIB_PATH)
    for n in declared_functions():
        assert hasattr(L, n), n
    assert set(declared_functions()) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"


def test_missing_library_fails_loudly(tmp_path):
    from femasm import _lib

    with pytest.raises(_lib.FemasmError):
        _lib._lib = None
        try:
            _lib.load(str(tmp_path / "nope.so"))
        finally:
            _lib._lib = None


def test_version_and_element_info():
    from femasm import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libfemasm.so not built")
    L = _lib.load()
    assert L.fa_version() >= 100
    nn, nq = ctypes.c_int32(), ctypes.c_int32()
    assert L.fa_element_info(-4, 2, -1, ctypes.byref(nn), ctypes.byref(nq)) == 0
    assert (nn.value, nq.value) == (10, 4)
    assert L.fa_element_info(8, 3, -1, ctypes.byref(nn), ctypes.byref(nq)) == 0
    assert (nn.value, nq.value) == (64, 64)
    assert L.fa_element_info(-4, 5, -1, ctypes.byref(nn), ctypes.byref(nq)) == -2
    assert b"unsupported" in L.fa_last_error()


@pytest.mark.parametrize("ct,p,denom", [(3, 1, 2), (3, 2, 6), (-4, 1, 6), (-4, 2, 30), (4, 1, 12), (4, 2, 180),
                                         (8, 1, 72)])
def test_simplex_reference_tensors_pack(ct, p, denom):
    """The P1/P2 triangle and tetrahedron, Q1/Q2 quadrilateral and Q1 hexahedron default rules give
    reference tensors that are exactly N / D (small integers): the packed table the k_gather_lin
    kernels read (affine quadrilaterals and Q1 hexahedra since round 6). A rounding drift past pack_ahat's tolerance
    would silently route them to the slower generic gather."""
    from femasm import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libfemasm.so not built")
    L = _lib.load()
    D, amax = ctypes.c_int32(-1), ctypes.c_double(0.0)
    assert L.fa_element_table_info(ct, p, -1, ctypes.byref(D), ctypes.byref(amax)) == 0
    assert D.value == denom, (ct, p, D.value)
    assert amax.value > 0.0
    assert L.fa_element_table_info(8, 2, -1, ctypes.byref(D), None) == 0 and D.value == 0  # Q2 hexahedra: none
    assert L.fa_element_table_info(4, 3, -1, ctypes.byref(D), None) == 0 and D.value == 0  # Q3: |N| too large


def test_library_reads_no_environment():
    """The product library's results and accepted arguments depend on its arguments only: its
    source reads no environment variable and the built library names none of the former tuning
    switches (FEMASM_*); measurement variants are built out of tree (tools/r4/variant.py)."""
    from femasm import _lib

    src = open(os.path.join(ROOT, "fem-libraries_amd", "csrc", "femasm.hip")).read()
    assert "getenv" not in src and "FEMASM_" not in src
    if os.path.exists(_lib.LIB_PATH):
        assert b"FEMASM_" not in open(_lib.LIB_PATH, "rb").read()
    # nor does the host package (FEMASM_LIB, the library path, aside)
    pkg = os.path.join(ROOT, "fem-libraries_amd", "femasm")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            txt = open(os.path.join(pkg, f)).read()
            names = set(re.findall(r"FEMASM_[A-Z_]+", txt)) - {"FEMASM_LIB"}
            assert not names and "os.environ" not in txt.replace('os.environ.get("FEMASM_LIB")', ""), f


def test_python_constants_match_header():
    """Every FA_* integer constant the host package defines equals the header's #define (or enum
    value) of the same name: the ctypes layer passes them to the library as plain integers."""
    from femasm import _lib

    txt = open(HEADER).read()
    hdr = {m.group(1): int(m.group(2), 0)
           for m in re.finditer(r"#define\s+(FA_[A-Z0-9_]+)\s+\(?(-?(?:0x[0-9A-Fa-f]+|\d+))\)?", txt)}
    hdr.update({m.group(1): int(m.group(2), 0) for m in re.finditer(r"\b(FA_[A-Z0-9_]+)\s*=\s*(-?(?:0x[0-9A-Fa-f]+|\d+))", txt)})
    py = {k: v for k, v in vars(_lib).items() if k.startswith("FA_") and isinstance(v, int)}
    assert py, "no FA_ constants in femasm._lib"
    missing = sorted(k for k in py if k not in hdr)
    assert not missing, f"not in include/femasm.h: {missing}"
    for k, v in py.items():
        assert hdr[k] == v, f"{k}: header {hdr[k]}, femasm._lib {v}"
