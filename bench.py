#!/usr/bin/env python3
"""Benchmark: global stiffness-matrix assembly of 3-D P2 linear elasticity (BASELINE.json metric
"Melements/s assembled + achieved HBM GB/s, 3D P2 elasticity at 1/2/4/8 GPUs").

One step = one fem.assemble_matrix(J, bcs) over the whole mesh — the reference's timed
setJ region (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:849-860: zero + cell loop + scatter
+ bc diagonal), sparsity build excluded as in the reference. Inputs (mesh, dofmap, E, pattern)
are resident in HBM before timing.

Workload: config E's mesh — unit cube, 203^3 cubes x 6 Kuhn tetrahedra = 50,192,562 P2 cells,
202,257,429 dofs — with the linear-elasticity J (d = 0), nu = 0.3, E = E_range[cell % 200]
(libc srand(6575) table), x=0 clamped and x=1 prescribed. N > 1 ranks (one per GPU) shard the
cube into z-slabs (strong scaling: fixed total mesh); by default each rank also assembles the cell
layer above its slab (ghost mode: its owned rows complete with no data-path collective), or, with
--slab-mode exchange, shared slab-interface rows are summed with an RCCL exchange between slab
neighbours (femasm.parallel). At N = 1 with config E the line also carries an "eneo" block: the
neo-Hookean AD tangent (config E's physics) timed on the same mesh in the same process.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

# algorithmic bytes per P2-tet cell under the element-stream model:
# 4*nn (dofmap) + 4*nv (geometry dofmap) + 8*gdim*nv (coords) + 8*n_w (E) + 16*ndof^2
B_E_P2_TET = 4 * 10 + 4 * 4 + 8 * 3 * 4 + 8 * 1 + 16 * 30 * 30  # = 14,560 (bytes_per_cell(CONFIGS["E"]))
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, Chip-level parameters)
FP64_PEAK_TFLOPS = 78.6  # MI355X published FP64 peak (vector = matrix on gfx950; SURVEY.md §8(d) ridge)


def flops_per_cell(cfg) -> int:
    """SURVEY.md §8(d) F_e = n_q (2 ndof^2 n_v + 2 n_v^2 ndof): the B^T D B contraction per cell
    (n_v = 3 / 6 Voigt components in 2-D / 3-D; 9 for the neo-Hookean F formulation). The AD
    tangent's own arithmetic (45 second-derivative passes per point) is not counted."""
    from femasm import fem, mesh

    ct = mesh.CellType[cfg["cell"]]
    gd = mesh.GDIM[ct]
    nd = fem.num_nodes_of(ct, cfg["degree"]) * gd
    nv = 9 if cfg.get("form") == "neo" else (3 if gd == 2 else 6)
    nq = int(fem.element_info(ct, cfg["degree"], cfg.get("qdeg"))[1])
    return nq * (2 * nd * nd * nv + 2 * nv * nv * nd)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


# BASELINE.json configs. The bench line is config E's mesh with linear
# elasticity ("E"); the others are available with --config for DESIGN.md measurements.
CONFIGS = {
    "A": dict(cell="triangle", degree=1, n=71, qdeg=1, label="2-D P1 tri, 71x71x2 (reference mechanic2d J, d=0)"),
    "B": dict(cell="quadrilateral", degree=2, n=1000, qdeg=None, label="2-D Q2 quad, 1000x1000"),
    "C": dict(cell="tetrahedron", degree=1, n=119, qdeg=None, label="3-D P1 tet, 119^3x6"),
    "D": dict(cell="hexahedron", degree=3, n=58, qdeg=None, label="3-D Q3 hex, 58^3 (192x192 local)"),
    "Dq2": dict(cell="hexahedron", degree=2, n=58, qdeg=None, label="3-D Q2 hex, 58^3 (81x81 local)"),
    # config D with interior vertices moved (non-affine trilinear cells): the MFMA element kernel +
    # block-store gather instead of the affine tensor gather
    "Dmfma": dict(cell="hexahedron", degree=3, n=58, qdeg=None, perturb=0.2,
                  label="3-D Q3 hex, 58^3, interior vertices moved 0.2 h (non-affine: MFMA element path)"),
    "E": dict(cell="tetrahedron", degree=2, n=203, qdeg=None, label="3-D P2 tet, 203^3x6 (config E mesh)"),
    "Eneo": dict(cell="tetrahedron", degree=2, n=203, qdeg=2, form="neo",
                 label="3-D P2 tet neo-Hookean (AD tangent), 203^3x6, u = 1e-3 sin(pi x)"),
}


def bytes_per_cell(cfg):
    """SURVEY.md §8(d) element-stream model: 4 nn + 4 nv + 8 gdim nv + 8 n_w + 16 ndof^2."""
    from femasm import fem, mesh

    ct = mesh.CellType[cfg["cell"]]
    gd, nv = mesh.GDIM[ct], mesh.NVERTS[ct]
    nn = fem.num_nodes_of(ct, cfg["degree"])
    nd = nn * gd
    geom = 0 if cfg["degree"] == 1 else 4 * nv  # the geometry dofmap is the dofmap itself at degree 1
    return 4 * nn + geom + 8 * gd * nv + 8 + 16 * nd * nd


def perturb_vertices(m, amp):
    """Move interior vertices by amp * sin(2 pi x) sin(pi y) sin(pi z) (per component, phase-shifted):
    boundary planes stay put (the bcs locate x = 0 and x = 1), trilinear cells become non-affine."""
    x = m.x
    s = torch.sin(torch.pi * x).prod(dim=1, keepdim=True)
    shift = torch.stack([torch.sin(2 * torch.pi * x[:, 0]), torch.cos(2 * torch.pi * x[:, 1]),
                         torch.sin(2 * torch.pi * x[:, 2] + 0.5)], dim=1)
    x += amp * s * shift


def build_problem(n, dev, z_range=None, cfg=None):
    from femasm import fem, mesh

    from femasm.materials import e_range

    cfg = cfg or CONFIGS["E"]
    ct = mesh.CellType[cfg["cell"]]
    if mesh.GDIM[ct] == 2:
        m = mesh.create_rectangle((1.0, 1.0), (n, n), ct, device=dev)
    else:
        m = mesh.create_box((1.0, 1.0, 1.0), (n, n, n), ct, device=dev, z_range=z_range)
    if cfg.get("perturb"):
        perturb_vertices(m, cfg["perturb"] / n)
    gd = m.gdim
    V = fem.functionspace(m, ("Lagrange", cfg["degree"], (gd,)))
    per_layer = n * n * (6 if ct == mesh.CellType.tetrahedron else 1)
    ncell_global0 = (z_range[0] if z_range else 0) * per_layer
    cid = torch.arange(m.num_cells, device=dev, dtype=torch.int64) + ncell_global0
    E = torch.tensor(e_range(), dtype=torch.float64, device=dev)[cid % 200]
    if cfg.get("form") == "neo":
        # SURVEY §8d neo-Hookean state: u = 1e-3 (sin pi x, sin pi y, sin pi z) at the nodes
        u = (1e-3 * torch.sin(torch.pi * V.tabulate_dof_coordinates())).reshape(-1).contiguous()
        a = fem.form(fem.NeoHookean(V, E=E, nu=0.3, u=u, quadrature_degree=cfg["qdeg"]))
    else:
        a = fem.form(fem.LinearElasticity(V, E=E, nu=0.3, quadrature_degree=cfg["qdeg"]))
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01] + [0.0] * (gd - 1), right, V)]
    return m, V, a, bcs


def kernel_hash() -> str:
    """sha256 (16 hex) of the HIP source the library is built from: keys the PMC traffic records."""
    import hashlib

    src = os.path.join(ROOT, "fem-libraries_amd", "csrc", "femasm.hip")
    return hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]


def measured_traffic(config: str, n: int, world: int):
    """HBM bytes per assembly launch from the committed rocprofv3 PMC record of the same workload
    (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE, k_cell_records + k_rec_bcbits + k_gather + k_bc_diag), or None.
    A record of another build of femasm.hip (kernel_hash mismatch) is refused, never reused."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if world != 1 or not os.path.exists(path):
        return None, "no PMC record for this run"
    rec = json.load(open(path)).get(f"{config}:{n}")
    if not rec:
        return None, f"no PMC record for {config}:{n}"
    if rec.get("kernel_hash") != kernel_hash():
        return None, f"PMC record is of femasm.hip {rec.get('kernel_hash')}, this build is {kernel_hash()}"
    return rec, rec["source"]


def compulsory_bytes(V, A, ncells: int, with_bc: bool, state: bool = False) -> dict:
    """Algorithmic bytes of one write-once assembly of A's row window: every matrix
    value written once (8 nnz) plus what any assembler must read -- the BSR pattern (4 B per block +
    8 B per row pointer), the dofmap (4 nn per cell), the geometry dofmap (4 nv per cell at degree
    > 1; it is the dofmap at degree 1), the coordinates (8 gdim per vertex), E (8 B per cell) and
    the bc markers (1 B per dof)."""
    from femasm import mesh

    m = V.mesh
    gd, nv = m.gdim, mesh.NVERTS[m.cell_type]
    r0, r1, data = A.parts[0] if len(A.parts) == 1 else (0, A.num_block_rows, None)
    nblocks = sum(int(p[2].shape[0]) for p in A.parts)
    parts = {
        "values_written": 8 * nblocks * A.bs * A.bs,
        "pattern": 4 * nblocks + 8 * (sum(p[1] - p[0] for p in A.parts) + 1),
        "dofmap": 4 * V.nn * ncells,
        "geometry": (4 * nv * ncells if V.degree > 1 else 0) + 8 * gd * int(m.x.shape[0]),
        "coefficients": 8 * ncells,
        "bc_markers": V.num_dofs if with_bc else 0,
        "state": 8 * V.num_dofs if state else 0,  # the neo-Hookean form's displacement u
    }
    parts["total"] = sum(parts.values())
    return parts


def cpu_core_count():
    """Cores for the all-cores CPU baseline: every core of this process's affinity mask, capped by
    the CPU share the machine gives this process -- a cgroup CPU quota, or the thread budget the GPU
    box exports (OMP_NUM_THREADS = its CPU share per GPU; more processes than the share would only
    time-slice). Returns (cores used, affinity count, share or None)."""
    aff = len(os.sched_getaffinity(0))
    share = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            share = max(1, int(int(q) // int(p)))
    except Exception:
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        share = min(share, int(omp)) if share else int(omp)
    return (min(aff, share) if share else aff), aff, share


def hbm_probe(dev, gib: float = 4.0, reps: int = 5) -> dict:
    """Measured HBM peak beside the 8 TB/s spec: fa_hbm_probe's 16-B-per-lane
    streams over two `gib` GiB buffers -- copy (read + write), write-only (the assembly's store
    stream is ~92 % of its bytes) and read-only -- best of `reps` launches timed with HIP events on
    the launch stream. Runs before the problem is built, so the buffers fit beside it."""
    import ctypes

    from femasm import _lib

    L = _lib.load()
    n = int(gib * (1 << 30)) // 8 // 2 * 2
    a = torch.ones(n, dtype=torch.float64, device=dev)
    b = torch.empty(n, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    out = {}
    for mode, name, nbytes in ((0, "copy", 16 * n), (1, "write", 8 * n), (2, "read", 8 * n)):
        _lib.check(L.fa_hbm_probe(mode, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a.data_ptr()), n, sh),
                   "fa_hbm_probe")  # warm-up
        best = float("inf")
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            _lib.check(L.fa_hbm_probe(mode, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a.data_ptr()), n, sh),
                       "fa_hbm_probe")
            e1.record(stream)
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e-3)
        out[f"{name}_GBps"] = round(nbytes / best / 1e9, 1)
    del a, b
    torch.cuda.empty_cache()
    out["what"] = (f"fa_hbm_probe (16 B per lane, nt loads/stores) over {gib:g} GiB buffers, best of {reps}: "
                   f"copy counts read + write bytes")
    return out


def _cpu_sample(sample_n: int):
    """The CPU baseline's P2-tet partition (numpy arrays for the oracle)."""
    from femasm import fem, mesh
    from femasm.materials import e_range
    from oracle import oracle as O

    m = mesh.create_unit_cube(sample_n, sample_n, sample_n, mesh.CellType.tetrahedron)
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    cells = V.dofmap.numpy()
    E = e_range()[np.arange(m.num_cells) % 200]
    lam, mu = O.lame(E, 0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0.0, 0.0], right, V)]
    marker, _ = fem._combine_bcs(V, bcs)
    indptr, indices = O.sparsity(cells, V.num_nodes)
    return dict(cells=cells, geom=m.cells.numpy(), x=m.x.numpy(), lam=lam, mu=mu, indptr=indptr, indices=indices,
                bc=marker.numpy())


def _cpu_rank(args):
    """One core of the multi-core CPU baseline: the oracle assembling its own partition `reps`
    times (like one MPI rank of the reference assembling its local cells); median seconds."""
    d, reps = args
    from oracle import oracle as O

    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        O.assemble_elasticity(-4, 2, d["cells"], d["geom"], d["x"], d["lam"], d["mu"], d["indptr"], d["indices"],
                              bc=d["bc"], diag=1.0)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def cpu_baseline(sample_n: int, reps: int):
    """Oracle (C restatement of dolfinx assemble_cells + set_diagonal, 1 thread) on a bounded
    P2-tet sample of the same workload; returns Melements/s."""
    from femasm import fem, mesh
    from femasm.materials import e_range
    from oracle import oracle as O

    m = mesh.create_unit_cube(sample_n, sample_n, sample_n, mesh.CellType.tetrahedron)
    V = fem.functionspace(m, ("Lagrange", 2, (3,)))
    cells = V.dofmap.numpy()
    geom = m.cells.numpy()
    x = m.x.numpy()
    E = e_range()[np.arange(m.num_cells) % 200]
    lam, mu = O.lame(E, 0.3)
    left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
    right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
    bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0.0, 0.0], right, V)]
    marker, _ = fem._combine_bcs(V, bcs)
    bc = marker.numpy()
    indptr, indices = O.sparsity(cells, V.num_nodes)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        O.assemble_elasticity(-4, 2, cells, geom, x, lam, mu, indptr, indices, bc=bc, diag=1.0)  # zeroed inside
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return m.num_cells / t / 1e6, m.num_cells, t


def time_steps(step, steps: int, warmup: int, dev, dist=None):
    """W untimed steps, then K steps bracketed by a barrier + synchronize on both sides; returns the
    wall seconds of the K steps and the mean launch time (HIP events on the launch stream, ms)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(steps):
        evs[k][0].record(stream)
        step()
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    return time.perf_counter() - t_start, float(np.mean([s.elapsed_time(e) for s, e in evs]))


def slab_leg(parallel, n: int, rank: int, world: int, dev, args, mode: str, dist) -> dict:
    """N > 1: build this rank's slab in one mode ("exchange": interface rows first, then a one-way RCCL
    send of the upper rank's interface blocks to the owner overlapping the interior rows -- the
    reference's PETSc stash, FEniCSx/mechanic2d/asym_elasto_damage_model.cc:853-854; "ghost": the layer
    above the slab assembled redundantly, no exchange), time K steps (barrier + synchronize on both
    sides, max over ranks), free it. Both modes leave every rank's owned rows complete."""
    t0 = time.time()
    prob = parallel.SlabProblem(n, rank, world, dev, form="neo" if args.config == "Eneo" else "linear", mode=mode)
    prob.plan()
    torch.cuda.synchronize()
    setup = time.time() - t0

    def step():
        prob.assemble(overlap=not args.no_overlap)
    elapsed, launch_ms = time_steps(step, args.steps, args.warmup, dev, dist)
    t = torch.tensor([elapsed, launch_ms, setup], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, launch_ms, setup = float(t[0]), float(t[1]), float(t[2])
    tot = torch.tensor([prob.num_cells, prob.num_cells_assembled, prob.exchange_bytes, prob.exchange_bytes],
                       dtype=torch.int64, device=dev)
    mx = tot[3:].clone()
    dist.all_reduce(tot)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    ms = elapsed / args.steps * 1e3
    comp = compulsory_bytes(prob.V, prob.A, prob.num_cells, True, state=args.config == "Eneo")
    out = {"ms_per_step": round(ms, 4), "launch_ms": round(launch_ms, 4),
           "value": round(int(tot[0]) / (ms * 1e-3) / 1e6, 3), "unit": "Melements/s", "cells": int(tot[0]),
           "cells_assembled": int(tot[1]), "exchange_MB_total": round(int(tot[2]) / 1e6, 1),
           "exchange_MB_max": round(int(mx[0]) / 1e6, 1), "setup_s": round(setup, 2),
           "what": prob.kernel_name, "_ncells_local": prob.num_cells, "_comp": comp}
    del prob, step
    torch.cuda.empty_cache()
    dist.barrier()
    return out


def eneo_block(dev, steps: int, warmup: int, search: bool = False) -> dict:
    """Config E as BASELINE.json states its physics: the neo-Hookean AD tangent on the same 50.2 M-cell
    P2 mesh, timed in this process after the linear problem is freed (secondary block of the default
    line: the driver's clock covers it). FP64-VALU-bound: its roof is the executed FP64 flops (PMC
    record of this build, profiles/traffic.json) over the 78.6 TF/s FP64 peak; no MFMA is issued.
    search: the headline's --plan-search, so both blocks of one line use the same kind of plan."""
    from femasm import fem

    cfg = CONFIGS["Eneo"]
    n = cfg["n"]
    t0 = time.time()
    m, V, a, bcs = build_problem(n, dev, cfg=cfg)
    torch.cuda.synchronize()
    t1 = time.time()
    fem.sparsity_pattern(V)
    torch.cuda.synchronize()
    t1a = time.time()
    A = fem.create_matrix(a)  # the value array: the runtime's allocation of ~139 GB (just freed by config E)
    torch.cuda.synchronize()
    t2 = time.time()
    popt = {"search": True} if search else None
    fem.gather_plan(V, A, 0, a.kind, **(popt or {}))
    torch.cuda.synchronize()
    setup = time.time() - t0
    setup_parts = {"problem_s": round(t1 - t0, 2), "pattern_s": round(t1a - t1, 2), "matrix_alloc_s": round(t2 - t1a, 2),
                   "plan_s": round(time.time() - t2, 2)}
    elapsed, launch_ms = time_steps(lambda: fem.assemble_matrix(a, bcs=bcs, A=A, plan=popt), steps, warmup, dev)
    ms = elapsed / steps * 1e3
    comp = compulsory_bytes(V, A, m.num_cells, True, state=True)
    trec, tsrc = measured_traffic("Eneo", n, 1)
    flops = None if trec is None else trec.get("fp64_flops")
    tf = None if flops is None else flops / (launch_ms * 1e-3) / 1e12
    out = {
        "workload": f"config E physics: {cfg['label']}, {m.num_cells} cells, E=E_range[cell%200], nu=0.3, "
                    f"x=0 clamped / x=1 prescribed, BSR(3) global matrix",
        "ms_per_step": round(ms, 4), "value": round(m.num_cells / (ms * 1e-3) / 1e6, 3), "unit": "Melements/s",
        "steps": steps, "warmup": warmup, "launch_ms": round(launch_ms, 4), "setup_s": round(setup, 2),
        "setup": setup_parts, "plan": "alternating-path search (--plan-search)" if search else "default",
        "bound": "fp64_valu",
        "fp64_executed": None if flops is None else {
            "flops_per_launch": flops, "TFLOPs": round(tf, 3), "peak_TFLOPs": FP64_PEAK_TFLOPS,
            "frac": round(tf / FP64_PEAK_TFLOPS, 4)},
        "hbm": {"algorithmic_bytes": comp["total"],
                "achieved_GBps": round(comp["total"] / (launch_ms * 1e-3) / 1e9, 1),
                "frac": round(comp["total"] / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)},
        "traffic": None if trec is None else round(trec["bytes"] / 1e9, 3),
        "traffic_source": tsrc,
    }
    del A, a, V, m, bcs
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="E", choices=sorted(CONFIGS))
    ap.add_argument("--side", "--n", dest="n", type=int, default=None,
                    help="cells per side (default: the config's); use --side under torchrun")
    ap.add_argument("--method", default="gather", choices=["gather", "scatter"])
    ap.add_argument("--deterministic", action="store_true",
                    help="bit-reproducible gather (FA_DETERMINISTIC: exact fixed-point sums)")
    ap.add_argument("--cpu-sample-n", type=int, default=24)
    ap.add_argument("--cpu-reps", type=int, default=7)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-overlap", action="store_true", help="N > 1: exchange after all rows (no overlap)")
    ap.add_argument("--slab-mode", default="both", choices=["both", "exchange", "ghost"],
                    help="N > 1: 'both' (default) times the RCCL interface exchange (the reference's PETSc-stash "
                         "semantics, north-star path) AND the communication-free redundant ghost layer (SURVEY §8(e) "
                         "alternative) one after the other in this run, each a complete assembly of every rank's "
                         "owned rows; the headline value is the faster leg and the line carries both ('legs'). "
                         "'exchange' / 'ghost' time one mode only")
    ap.add_argument("--no-hbm-probe", action="store_true", help="skip the measured-HBM-peak stream probe")
    ap.add_argument("--plan-search", action="store_true",
                    help="plan the LDS order with the alternating-path search (FA_PLAN_ORDER_SEARCH: ~10x plan time)")
    ap.add_argument("--no-eneo", action="store_true",
                    help="config E at N = 1: skip the secondary neo-Hookean (config E physics) block")
    ap.add_argument("--cpu-all-affinity", type=int, default=1,
                    help="1: also time the CPU baseline with one process per affinity core (beyond the CPU share)")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="processes of the all-cores CPU baseline (0 = every affinity core, capped by the cgroup "
                         "CPU quota; 1 = single core only)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    # Multi-core CPU baseline workers: the fork server starts before this process touches the GPU
    # (workers must not inherit an initialised HIP runtime); the workers themselves are forked from
    # it only after the GPU timing -- a pool of 256 idle workers alive during the timed steps slowed
    # config E from 44.8 to 50.0 ms per step (profiles/r3/cpu_pool_effect.txt)
    cpu_ctx, cpu_pool, cpu_cores, npool = None, None, 1, 1
    cores_avail, cores_aff, cores_quota = cpu_core_count()
    if int(os.environ.get("RANK", "0")) == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_cores != 1:
        try:
            import multiprocessing as mp
            from multiprocessing import forkserver

            cpu_cores = max(1, min(args.cpu_cores or cores_avail, cores_aff))
            # one pool of every affinity core: the CPU-share run uses cpu_cores of its workers, the
            # all-affinity run all of them (BASELINE.md §2 asks for the all-cores figure)
            npool = cores_aff if (args.cpu_all_affinity and not args.cpu_cores) else cpu_cores
            if npool > 1:
                cpu_ctx = mp.get_context("forkserver")
                forkserver.ensure_running()
        except Exception as e:  # the baseline is a reported figure: never fail the bench line for it
            log(f"[bench] multi-core CPU baseline disabled: {e}")
            cpu_ctx, cpu_cores = None, 1
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; FEMASM_DIST_BACKEND=gloo rehearses N > 1 with ranks sharing the visible GPUs
    backend = os.environ.get("FEMASM_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % max(ndev, 1) if backend == "gloo" else local_rank)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            # RCCL over xGMI; a bounded timeout so that a stuck exchange ends in an error, not a hang.
            # Blocking waits without the watchdog's abort: a timed-out or failed transfer of the exchange
            # leg then raises in this process (caught below: the ghost leg's line stands) instead of the
            # watchdog tearing the process down before rank 0 prints (a caller's setting is kept)
            os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
            import datetime

            dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=180))
        else:
            dist.init_process_group(backend)

    from femasm import fem

    cfg = CONFIGS[args.config]
    n = args.n or cfg["n"]
    b_e = bytes_per_cell(cfg)
    hbm_meas = None
    if rank == 0 and not args.no_hbm_probe:
        try:
            hbm_meas = hbm_probe(dev)
        except Exception as e:  # a reported figure: never fail the bench line for it
            log(f"[bench] HBM probe failed: {e}")
    # the library's code object and each setup kernel load at their first launch in a process (~2 s of
    # one-time runtime work on a fresh box, round 6): a 4^3 assembly of the same form first, timed on its
    # own ("library_warmup_s"), so setup_s is the per-mesh cost the reference's create_matrix stands for.
    # Setup only (pattern, matrix, plan): no assembly kernel runs here, so a profiler's per-kernel average
    # over the assembly kernels (rocprofv3 --stats, the PMC records) holds the timed workload's launches
    # only; the assembly kernels load in the untimed warmup steps
    t_w = time.time()
    wcfg = dict(cfg, n=4)
    _wm, _wV, _wa, _wb = build_problem(4, dev, cfg=wcfg)
    _wA = fem.create_matrix(_wa)
    for part in range(len(_wA.parts)):
        fem.gather_plan(_wV, _wA, part, _wa.kind, deterministic=args.deterministic)
    torch.cuda.synchronize()
    del _wm, _wV, _wa, _wb, _wA
    warmup_s = time.time() - t_w
    t0 = time.time()
    t_pattern = t_plan = t_alloc = 0.0
    legs, best = None, None
    if world > 1:
        from femasm import parallel

        if args.config not in ("E", "Eneo"):
            raise SystemExit("N > 1 shards config E's mesh (P2 tets; linear elasticity or neo-Hookean) only")
        legs = {}
        # the communication-free leg first: its line stands even if the exchange leg fails
        modes = ["ghost", "exchange"] if args.slab_mode == "both" else [args.slab_mode]
        for mode in modes:
            try:
                legs[mode] = slab_leg(parallel, n, rank, world, dev, args, mode, dist)
                log(f"[bench] slab mode {mode}: {legs[mode]['ms_per_step']:.3f} ms per step (max over ranks)")
            except Exception as e:  # recorded in the line; the other leg is the headline
                if len(modes) == 1:
                    raise
                legs[mode] = {"error": f"{type(e).__name__}: {e}"[:400]}
                log(f"[bench] slab mode {mode} failed: {e}")
                torch.cuda.empty_cache()
        ok = [k for k in legs if "error" not in legs[k]]
        if not ok:
            raise SystemExit("every slab leg failed")
        best = min(ok, key=lambda k: legs[k]["ms_per_step"])
        L = legs[best]
        ncells_local, comp_leg = L.pop("_ncells_local"), L.pop("_comp")
        for other in legs.values():  # (failed legs hold only their error)
            other.pop("_ncells_local", None)
            other.pop("_comp", None)
        elapsed, launch_ms, ncells_total = L["ms_per_step"] * args.steps * 1e-3, L["launch_ms"], L["cells"]
        exchange_mb = L["exchange_MB_max"]
    else:
        m, V, a, bcs = build_problem(n, dev, cfg=cfg)
        torch.cuda.synchronize()
        t1 = time.time()
        fem.sparsity_pattern(V)  # adjacency + sparsity pattern (dolfinx create_matrix, first half)
        torch.cuda.synchronize()
        t1a = time.time()
        A = fem.create_matrix(a)  # the value array (the HIP runtime's allocation of ~139 GB for config E)
        torch.cuda.synchronize()
        t2 = time.time()
        t_alloc = t2 - t1a
        for part in range(len(A.parts)):
            fem.gather_plan(V, A, part, a.kind, deterministic=args.deterministic,  # chunks, slot map, LDS order
                            **({"search": True} if args.plan_search else {}))
        torch.cuda.synchronize()
        t_pattern, t_plan = t1a - t1, time.time() - t2
        ncells_local = m.num_cells
        V_loc, A_loc, with_bc = V, A, True

        def step():
            fem.assemble_matrix(a, bcs=bcs, A=A, method=args.method, deterministic=args.deterministic,
                                plan={"search": True} if args.plan_search else None)

        torch.cuda.synchronize()
    setup_s = time.time() - t0 if legs is None else legs[best]["setup_s"]
    log(f"[bench] setup {setup_s:.1f}s (pattern {t_pattern:.1f}s, plan {t_plan:.1f}s): {ncells_local} cells "
        f"on rank {rank}")

    if legs is None:
        # per-launch kernel durations: HIP events on the launch stream (torch's current stream)
        elapsed, launch_ms = time_steps(step, args.steps, args.warmup, dev, dist)
        ncells_total = ncells_local

    ms_per_step = elapsed / args.steps * 1e3
    melem_s = ncells_total / (ms_per_step * 1e-3) / 1e6
    # roofline.achieved: the algorithmic (write-once, compulsory) bytes of this rank's assembly over
    # the live event time of one launch on the launch stream
    comp = comp_leg if legs is not None else \
        compulsory_bytes(V_loc, A_loc, ncells_local, with_bc, state=cfg.get("form") == "neo")
    achieved = comp["total"] / (launch_ms * 1e-3) / 1e9
    # traffic: PMC-measured HBM bytes per launch of this build (profiles/traffic.json, keyed on the
    # femasm.hip hash), with its own fraction of peak; the SURVEY §8(d) element-stream model B_e is
    # reported as the bandwidth the reference-shaped algorithm would need at this rate (not bytes moved)
    trec, tsrc = measured_traffic(args.config, n, world)
    traffic = None if trec is None else round(trec["bytes"] / 1e9, 3)
    traffic_gbps = None if trec is None else trec["bytes"] / (launch_ms * 1e-3) / 1e9
    fracs = {"frac": achieved / HBM_PEAK_GBPS}
    f_e = flops_per_cell(cfg)
    tflops = f_e * ncells_local / (launch_ms * 1e-3) / 1e12
    # neo-Hookean: FP64-compute-bound (executed flops / algorithmic bytes ~15 flop/B, above the 9.8
    # flop/B ridge). achieved = the executed FP64 flops of the launch counted by the PMC
    # (SQ_INSTS_VALU_FLOPS_FP64, profiles/traffic.json of this build); F_e stays a model
    compute_bound = cfg.get("form") == "neo"
    exec_flops = None if trec is None else trec.get("fp64_flops")
    tflops_exec = None if exec_flops is None else exec_flops / (launch_ms * 1e-3) / 1e12
    if tflops_exec is not None:
        fracs["flop_frac"] = tflops_exec / FP64_PEAK_TFLOPS
    if traffic_gbps is not None:
        fracs["traffic_frac"] = traffic_gbps / HBM_PEAK_GBPS
    # every fraction reported is measured (algorithmic bytes or PMC counters over the live launch
    # time): a value above 1 means a wrong byte count or time -- recorded in the line, never asserted
    invalid = [f"{k} = {v:.3f} > 1" for k, v in fracs.items() if v > 1.0]
    for w in invalid:
        log(f"[bench] roofline check failed: {w} (a byte count or a time is wrong)")
    # a fraction above 1 is not published: its field is null (the line keeps the reason in "invalid")
    fracs = {k: (None if v > 1.0 else v) for k, v in fracs.items()}
    rnd = lambda v, d=4: None if v is None else round(v, d)  # noqa: E731
    # the FP64 roof applies only with a PMC flop count of this very build; otherwise the line
    # reports the HBM roof (F_e is a model of a contraction this kernel does not run)
    compute_bound = compute_bound and tflops_exec is not None

    eneo = None
    if world == 1 and args.config == "E" and not args.no_eneo and args.method == "gather" and not args.deterministic \
            and (args.n or cfg["n"]) == CONFIGS["Eneo"]["n"]:
        del step, V_loc, A_loc, A, a, V, m, bcs  # the linear problem's ~150 GB
        torch.cuda.empty_cache()
        try:
            eneo = eneo_block(dev, args.steps, args.warmup, search=args.plan_search)
        except Exception as e:  # a secondary block: recorded, never fails the headline line
            eneo = {"error": f"{type(e).__name__}: {e}"}
            log(f"[bench] E-neo block failed: {e}")

    cpu = None
    if cpu_ctx is not None:
        try:
            cpu_pool = cpu_ctx.Pool(npool)
        except Exception as e:
            log(f"[bench] multi-core CPU baseline disabled: {e}")
            cpu_pool, cpu_cores = None, 1
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        v, nc, t = cpu_baseline(args.cpu_sample_n, args.cpu_reps)
        cpu = {"value": round(v, 4), "unit": "Melements/s", "cores": 1, "kind": "port", "value_1core": round(v, 4),
               "sample": f"oracle/fa_oracle.c ora_assemble_elasticity (dolfinx assemble_cells + set_diagonal "
                         f"restated), P2 tet, {args.cpu_sample_n}^3x6 = {nc} cells, zero+assemble+bc diag, "
                         f"median of {args.cpu_reps} runs ({t:.2f} s each), 1 thread"}
        if cpu_pool is not None:
            try:
                d = _cpu_sample(args.cpu_sample_n)
                tmax = max(cpu_pool.map(_cpu_rank, [(d, args.cpu_reps)] * cpu_cores, chunksize=1))
                vm = cpu_cores * nc / tmax / 1e6
                cpu.update(value=round(vm, 4), cores=cpu_cores, cores_affinity=cores_aff, cpu_share=cores_quota,
                           sample=cpu["sample"] + f"; headline value: {cpu_cores} processes at once (the CPU share "
                                  f"of this GPU), each assembling its own {args.cpu_sample_n}^3x6 partition (as MPI "
                                  f"ranks own theirs), {cpu_cores} x {nc} cells / slowest median ({tmax:.2f} s)")
                if args.cpu_all_affinity and cores_aff > cpu_cores and not args.cpu_cores:
                    # every core of the affinity mask, one process each, fewer repetitions (beyond
                    # the share the processes time-slice the CPUs the machine gives this job)
                    reps_a = max(1, min(args.cpu_reps, 3))
                    ta = max(cpu_pool.map(_cpu_rank, [(d, reps_a)] * cores_aff, chunksize=1))
                    cpu["all_affinity"] = {
                        "value": round(cores_aff * nc / ta / 1e6, 4), "unit": "Melements/s", "cores": cores_aff,
                        "what": f"{cores_aff} processes at once (every core of the affinity mask), same sample, "
                                f"median of {reps_a} runs each, {cores_aff} x {nc} cells / slowest ({ta:.2f} s); "
                                f"the CPU share is {cores_quota}"}
            except Exception as e:
                log(f"[bench] multi-core CPU baseline failed: {e}")
            finally:
                cpu_pool.close()

    if rank == 0:
        jform = "neo-Hookean J (device AD tangent)" if cfg.get("form") == "neo" else "linear-elasticity J"
        workload = (f"config {args.config}: {cfg['label']} — {jform}, {ncells_total} cells, "
                    f"E=E_range[cell%200], nu=0.3, x=0 clamped / x=1 prescribed, BSR(gdim) global matrix")
        if args.config == "E":
            workload = (f"config E mesh, linear elasticity J: unit cube {n}^3 x 6 Kuhn tets, P2 "
                        f"({ncells_total} cells, {(2 * n + 1) ** 3 * 3} dofs), E=E_range[cell%200], "
                        f"nu=0.3, x=0 clamped / x=1 prescribed, BSR(3) global matrix")
        out = {
            "metric": "Melements/s assembled + achieved HBM GB/s, 3D P2 elasticity at 1/2/4/8 GPUs",
            "value": round(melem_s, 3),
            "unit": "Melements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "hbm_GBps_algorithmic": round(achieved * world, 1),
            "setup_s": round(setup_s, 2),
            "setup": {"pattern_s": round(t_pattern, 2), "plan_s": round(t_plan, 2),
                      "matrix_alloc_s": round(t_alloc, 2), "problem_s": round(setup_s - t_pattern - t_plan - t_alloc, 2),
                      "library_warmup_s": round(warmup_s, 2), "solve_assembly_s": round(7 * ms_per_step * 1e-3, 3),
                      "solve_assembly_what": "7 x ms_per_step: the assemblies of one reference Newton solve "
                                             "(doc.tex:2051), against one setup_s",
                      "what": "setup_s = problem_s (mesh + function space + bcs) + pattern_s (adjacency + sparsity) "
                              "+ matrix_alloc_s (the value array's device allocation) + plan_s (gather plan), once "
                              "per mesh (the reference's create_matrix is likewise outside its timed region)"},
            "config": {"workload": workload, "method": args.method + ("-deterministic" if args.deterministic else ""),
                       "parallelism": ((f"z-slabs x{world}: interface planes first, then per boundary a one-way "
                                        f"{'RCCL' if backend == 'nccl' else backend} send of the upper rank's "
                                        f"plane blocks to the owner ({exchange_mb} MB max sent per rank) "
                                        f"{'after' if args.no_overlap else 'overlapping'} the interior rows")
                                       if best == "exchange" else
                                       f"z-slabs x{world}, no exchange: each rank also assembles the cell layer "
                                       f"above its slab (redundant ghost layer) so its owned rows are complete")
                       + (f"; the faster of the legs {sorted(legs)} (both in 'legs')" if len(legs) > 1 else "")
                       if world > 1 else "single GPU"},
            "legs": legs,
            # per GPU (rank 0 / slowest rank): achieved = algorithmic bytes of the assembly / launch time
            "roofline": {"bound": "fp64_valu" if compute_bound else "hbm",
                         "achieved": round(tflops_exec, 3) if compute_bound else round(achieved, 1),
                         "achieved_source": "PMC SQ_INSTS_VALU_FLOPS_FP64 of this build (executed FP64 flops, FP64 "
                                            "VALU; no MFMA in this kernel) / launch time" if compute_bound
                         else "algorithmic bytes / launch time" + (
                             "" if cfg.get("form") != "neo" or tflops_exec is not None else
                             " (FP64-bound form, but no PMC flop record of this build: HBM roof reported)"),
                         "peak": FP64_PEAK_TFLOPS if compute_bound else HBM_PEAK_GBPS,
                         "unit": "TFLOP/s" if compute_bound else "GB/s",
                         "frac": rnd(fracs["flop_frac"] if compute_bound else fracs["frac"]), "traffic": traffic,
                         "invalid": invalid or None,
                         "peak_measured": hbm_meas,
                         "hbm": {"achieved_GBps": round(achieved, 1), "frac": rnd(fracs["frac"])},
                         "model_fp64": {"flops_per_cell": f_e, "equivalent_TFLOPs": round(tflops, 3),
                                        "what": "SURVEY §8(d) F_e at this rate: the B^T D B quadrature contraction's "
                                                "flops, a model -- the gathers form blocks from reference tensors "
                                                "(linear) or from F, cof F and invariant coefficients (neo-Hookean)"},
                         "fp64_executed": None if exec_flops is None else {
                             "flops_per_launch": exec_flops, "TFLOPs": round(tflops_exec, 3),
                             "frac": rnd(fracs.get("flop_frac")), "peak_TFLOPs": FP64_PEAK_TFLOPS},
                         "traffic_GBps": None if traffic_gbps is None else round(traffic_gbps, 1),
                         "traffic_frac": None if traffic_gbps is None else rnd(fracs["traffic_frac"]),
                         "traffic_source": tsrc,
                         "mfma_busy": None if trec is None else trec.get("mfma_busy"),
                         "kernel": "the assembly launch: per-cell records and their bc bits (or the MFMA element kernel of non-affine "
                                   "hexahedra) + the row gather + the bc diagonal",
                         "launch_ms": round(launch_ms, 4),
                         "algorithmic_bytes": comp["total"],
                         "algorithmic_bytes_per_cell": round(comp["total"] / ncells_local, 1),
                         "algorithmic_breakdown": {k: v for k, v in comp.items() if k != "total"},
                         "model_element_stream": {
                             "bytes_per_cell": b_e,
                             "equivalent_GBps": round(b_e * ncells_local / (launch_ms * 1e-3) / 1e9, 1),
                             "what": "SURVEY §8(d) B_e: bytes a reference-shaped element scatter moves "
                                     "(read + write of every element-matrix value); not moved by the gather"}},
            "cpu_baseline": cpu,
            "eneo": eneo,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
