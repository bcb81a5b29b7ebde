"""ctypes binding of the femasm C ABI (include/femasm.h) — libfemasm.so built for gfx950.

There is no fallback: if the shared library is missing, importing a compute entry point
raises. All pointers passed are device pointers of torch tensors; streams are torch's
current HIP stream.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libfemasm.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

FA_OK = 0
FA_TRIANGLE, FA_QUADRILATERAL, FA_TETRAHEDRON, FA_HEXAHEDRON = 3, 4, -4, 8
FA_LINEAR_ELASTICITY, FA_ASYM_DAMAGE, FA_NEO_HOOKEAN, FA_ASYM_DAMAGE_AD = 0, 1, 2, 3
FA_GATHER, FA_SCATTER, FA_ZERO_FIRST, FA_DETERMINISTIC, FA_CHECK_ERRORS = 0x0, 0x1, 0x2, 0x4, 0x8
FA_PLAN_AFFINE, FA_PLAN_DETERMINISTIC, FA_PLAN_ORDER_SEARCH, FA_PLAN_NEO = 0x1, 0x2, 0x4, 0x8


class FemasmError(RuntimeError):
    pass


class fa_mesh(ctypes.Structure):
    _fields_ = [
        ("cell_type", ctypes.c_int32),
        ("degree", ctypes.c_int32),
        ("gdim", ctypes.c_int32),
        ("nn", ctypes.c_int32),
        ("ncells", ctypes.c_int64),
        ("nnodes", ctypes.c_int64),
        ("cells", ctypes.c_void_p),
        ("nv", ctypes.c_int32),
        ("_pad", ctypes.c_int32),
        ("geom", ctypes.c_void_p),
        ("x", ctypes.c_void_p),
    ]


class fa_form(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("qdeg", ctypes.c_int32),
        ("E", ctypes.c_void_p),
        ("nu", ctypes.c_double),
        ("lam", ctypes.c_void_p),
        ("mu", ctypes.c_void_p),
        ("u", ctypes.c_void_p),
        ("d", ctypes.c_void_p),
        ("f", ctypes.c_void_p),
    ]


class fa_bsr(ctypes.Structure):
    _fields_ = [
        ("nrows", ctypes.c_int64),
        ("bs", ctypes.c_int32),
        ("_pad", ctypes.c_int32),
        ("nblocks", ctypes.c_int64),
        ("indptr", ctypes.c_void_p),
        ("indices", ctypes.c_void_p),
        ("data", ctypes.c_void_p),
        ("row_begin", ctypes.c_int64),
        ("row_end", ctypes.c_int64),
    ]


class fa_adjacency(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("idx", ctypes.c_void_p)]


class fa_plan(ctypes.Structure):
    _fields_ = [
        ("nchunks", ctypes.c_int64),
        ("row_start", ctypes.c_void_p),
        ("max_blocks", ctypes.c_int32),
        ("max_adj", ctypes.c_int32),
        ("slots", ctypes.c_void_p),
        ("slot_order", ctypes.c_int32),
        ("cell_flags", ctypes.c_int32),
        ("eadj", ctypes.c_void_p),
        ("corder", ctypes.c_void_p),
        ("contrib", ctypes.c_void_p),
        ("chunk_desc", ctypes.c_void_p),
    ]


# exported symbols with their signatures; tests check every one against include/femasm.h
P = ctypes.c_void_p
I32, I64, D = ctypes.c_int32, ctypes.c_int64, ctypes.c_double
SIGNATURES = {
    "fa_last_error": (ctypes.c_char_p, []),
    "fa_version": (ctypes.c_int, []),
    "fa_element_info": (ctypes.c_int, [I32, I32, I32, P, P]),
    "fa_element_table_info": (ctypes.c_int, [I32, I32, I32, P, P]),
    "fa_plan_chunk_desc": (ctypes.c_int, [P, P, P, P, P, P]),
    "fa_build_adjacency": (ctypes.c_int, [P, P, P, P]),
    "fa_sparsity_count": (ctypes.c_int, [P, P, P, P, P]),
    "fa_sparsity_fill": (ctypes.c_int, [P, P, P, P, P]),
    "fa_check_pattern": (ctypes.c_int, [P, P, P, P, I64, P]),
    "fa_plan_gather": (ctypes.c_int, [P, P, P, P, P, P]),
    "fa_plan_gather_form": (ctypes.c_int, [P, I32, P, P, P, P, P]),
    "fa_plan_slots": (ctypes.c_int, [P, P, P, P, P, P]),
    "fa_plan_order": (ctypes.c_int, [P, P, P, P, P, P]),
    "fa_plan_locality": (ctypes.c_int, [P, P, P, P, P]),
    "fa_plan_check_affine": (ctypes.c_int, [P, P, P]),
    "fa_plan_gather_contrib": (ctypes.c_int, [P, P, P, P, P, P]),
    "fa_plan_contrib_bytes": (ctypes.c_int, [P, P, P, P, P, P]),
    "fa_plan_contrib": (ctypes.c_int, [P, P, P, P, I64, P, P]),
    "fa_tabulate_cells": (ctypes.c_int, [P, P, I64, I64, P, P]),
    "fa_assemble_matrix": (ctypes.c_int, [P, P, P, P, P, D, P, I32, P]),
    "fa_gather_work_bytes": (ctypes.c_int, [P, P, P]),
    "fa_gather_prepare": (ctypes.c_int, [P, P, P, P, P]),
    "fa_gather_rows": (ctypes.c_int, [P, P, P, P, P, D, P, P, P]),
    "fa_assemble_vector": (ctypes.c_int, [P, P, P, P, P]),
    "fa_apply_lifting": (ctypes.c_int, [P, P, P, P, P, P, P, D, P]),
    "fa_set_bc": (ctypes.c_int, [P, I64, P, P, P, D, P]),
    "fa_bsr_mult": (ctypes.c_int, [P, P, P, P]),
    "fa_bsr_block_diag": (ctypes.c_int, [P, P, P]),
    "fa_hbm_probe": (ctypes.c_int, [I32, P, P, I64, P]),
}

_lib = None


def load(path: str | None = None):
    """Load libfemasm.so (no fallback: raises FemasmError when it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("FEMASM_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise FemasmError(
            f"{path} is missing: build it with `make -C {CSRC}` (hipcc --offload-arch=gfx950) "
            "or __graft_entry__.build(); femasm has no CPU fallback")
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is None:
            if os.path.abspath(path) == os.path.abspath(LIB_PATH):
                raise FemasmError(f"{path} does not export {name}: rebuild it (make -C {CSRC})")
            continue  # an older measurement build (FEMASM_LIB, A/B runs): entry points it lacks stay unbound
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int, what: str = ""):
    if rc != FA_OK:
        msg = load().fa_last_error().decode(errors="replace")
        raise FemasmError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """Raw device pointer of a torch tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
