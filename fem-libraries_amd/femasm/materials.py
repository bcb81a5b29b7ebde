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
