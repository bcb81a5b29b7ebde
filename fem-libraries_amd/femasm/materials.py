"""Material coefficients of the reference problem.

E_range: 200 Young's moduli from glibc ``srand(6575)`` / ``rand() % 200``, exactly as the
reference computes them (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:533-545, Python driver
FEniCSx/mechanic2d/asym_elasto_damage_model_symb_sym.py:213-222 through libc as well); a cell with
physical tag t gets E_range[t % 200]; MFEM indexes by attribute (:1076-1098). Lamé parameters
as in FEniCSx/mechanic2d/asym_ufl.py:26-27.
"""
from __future__ import annotations

import ctypes

import numpy as np

_CACHE = {}


def e_range(seed: int = 6575) -> np.ndarray:
    if seed not in _CACHE:
        libc = ctypes.CDLL("libc.so.6")
        libc.srand(seed)
        a = (1.0e8 - 5.0e6) / 199.0
        _CACHE[seed] = np.array([a * (libc.rand() % 200) + 5.0e6 for _ in range(200)])
    return _CACHE[seed]


def lame(E, nu: float):
    mu = E / (2.0 * (1.0 + nu))
    lmbda = E * nu / ((1.0 + nu) * (1.0 - 2.0 * nu))
    return lmbda, mu


def e_from_cell_tags(tags, num_cells: int, seed: int = 6575):
    """E per cell from the cell tags (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:543-545:
    ``E_range[phys % 200]`` over ``cell_tag.values()``): a torch float64 tensor [num_cells] on the
    tags' device. Every cell must carry a tag (the reference indexes the values by cell)."""
    import torch

    if tags.indices.numel() != num_cells or not bool(
            (tags.indices.to(torch.int64) == torch.arange(num_cells, device=tags.indices.device)).all()):
        raise ValueError(f"cell tags cover {tags.indices.numel()} of {num_cells} cells: E needs a tag on every cell")
    er = torch.tensor(e_range(seed), dtype=torch.float64, device=tags.values.device)
    return er[tags.values.to(torch.int64) % 200]
