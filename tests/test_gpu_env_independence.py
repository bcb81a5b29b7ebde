"""The C ABI's results do not depend on the process environment: the same assemblies in two child
processes, one with every former tuning switch of the library set to a non-default value, give
bit-identical matrices (deterministic mode, so any difference would be a real one), and the same
error for a neo-Hookean plan that is not positional."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the switches earlier builds read (VERDICT r3 What's weak #8)
FORMER = {"FEMASM_LIN_GATHER": "0", "FEMASM_NEO_M": "0", "FEMASM_GATHER_SCHED": "static",
          "FEMASM_GATHER_GRID_MULT": "3", "FEMASM_CHUNK_ORDER_ALL": "1", "FEMASM_LINU": "0",
          "FEMASM_ORDER_KICKS": "16", "FA_ORDER_STATS": "1", "FA_CHECK": "1", "FEMASM_SLOTS": "0",
          "FEMASM_SLOT_ORDER": "0", "FEMASM_CHUNK_ORDER": "0", "FEMASM_CONTRIB": "1", "FEMASM_MAX_PART_GB": "0.001"}

CHILD = r"""
import hashlib, json, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/fem-libraries_amd")
import numpy as np, torch
from femasm import _lib, fem, mesh
from femasm.materials import e_range
dev = torch.device("cuda", 0)
out = {}
for name, ct, p, n in (("p2tet", -4, 2, (6, 5, 4)), ("p1tri", 3, 1, (20, 17))):
    m = mesh.create_unit_cube(*n, cell_type=ct, device=dev) if len(n) == 3 else \
        mesh.create_unit_square(*n, cell_type=ct, device=dev)
    V = fem.functionspace(m, ("Lagrange", p, (m.gdim,)))
    E = torch.tensor(e_range()[np.arange(m.num_cells) % 200], device=dev)
    a = fem.LinearElasticity(V, E=E, nu=0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V)]
    A = fem.assemble_matrix(a, bcs=bcs, deterministic=True)
    torch.cuda.synchronize()
    out[name] = [len(A.parts), hashlib.sha256(A.data.cpu().numpy().tobytes()).hexdigest()]
m = mesh.create_unit_cube(2, 2, 2, cell_type=-4, device=dev)
V = fem.functionspace(m, ("Lagrange", 2, (3,)))
u = torch.zeros(V.num_dofs, dtype=torch.float64, device=dev)
a = fem.NeoHookean(V, E=1.0, nu=0.3, u=u)
try:
    fem.assemble_matrix(a, plan=dict(order="steps"))
    out["neo_unordered"] = "assembled"
except (ValueError, _lib.FemasmError) as e:  # refused up front (gather_plan) or by the library
    out["neo_unordered"] = type(e).__name__ + ": " + str(e).split(":")[0]
print(json.dumps(out))
"""


def _run(env):
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_results_independent_of_environment():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    base = {k: v for k, v in os.environ.items() if not k.startswith(("FEMASM_", "FA_"))}
    clean = _run(base)
    dirty = _run({**base, **FORMER})
    assert clean == dirty
    assert clean["neo_unordered"] != "assembled"
