"""Multi-GPU assembly: z-slab sharding of a structured box with an RCCL boundary exchange.

The reference runs one MPI rank per core on a (Par)METIS partition and sums the contributions
to rows owned by another rank inside PETSc's ``MatAssemblyBegin/End`` stash
(FEniCSx/mechanic2d/asym_elasto_damage_model.cc:853-859; MFEM: hypre PtAP). Here one process per
GPU owns a slab of cube layers [k0, k1) of an n_x x n_y x n_z box:

* its cells are the cells of its own layers (assembled with the gather kernel);
* its sparsity pattern comes from its layers plus one ghost layer on each side, so the rows of
  the two interface planes (z = k0 and z = k1) carry the full global pattern on both neighbours;
* rows are the lattice planes p*k0 .. p*k1 of the degree-p lattice (a fa_bsr row window); with
  lattice numbering each interface plane is one contiguous slab of BSR values;
* the only exchange is, per slab boundary, ONE one-way transfer from the upper rank to the plane's
  owner (the lower rank, doc.tex:464) of the interface rows' blocks in or above the plane -- the
  only ones the upper rank contributes to (``interface_suffix``) -- which the owner adds into its
  rows (PETSc's stash does the same at MatAssemblyEnd: off-process entries travel to their owner
  only). It runs as an RCCL send/recv on a 2-rank process group (xGMI is point-to-point, a global
  collective over all interfaces would be link-bound -- SURVEY.md §5). Every interior rank sends
  down one link while it receives from above on another. The interface rows are assembled first
  and the transfers run on RCCL's streams while the interior rows assemble (``SlabProblem.assemble``).
  exchange="suffix" keeps the earlier 2-rank all-reduce of the same blocks (both copies complete,
  twice the link bytes), exchange="rows" all-reduces whole interface rows.
* the owner's copy is complete after the add; the upper rank's copy of that plane holds only its
  own partial sums (it owns none of those rows). Dirichlet diagonals on interface rows (inserted
  by both ranks) are reset to `diagonal`.

The partition / numbering logic (``SlabPartition``) and the exchange (``exchange_interfaces``) are
device-agnostic (torch tensors on any device, any torch.distributed backend: tested with gloo on
CPU, run with nccl = RCCL on MI355X).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass

import numpy as np
import torch


def slab_layers(nz: int, world: int, rank: int) -> tuple[int, int]:
    """Balanced split of nz cube layers over `world` ranks: rank gets [k0, k1)."""
    base, extra = divmod(nz, world)
    k0 = rank * base + min(rank, extra)
    return k0, k0 + base + (1 if rank < extra else 0)


@dataclass
class SlabPartition:
    n: tuple  # cubes per direction (nx, ny, nz)
    degree: int
    rank: int
    world: int

    def __post_init__(self):
        nx, ny, nz = self.n
        p = self.degree
        if nz < self.world:
            raise ValueError(f"{nz} layers cannot be split over {self.world} ranks")
        self.k0, self.k1 = slab_layers(nz, self.world, self.rank)
        self.kp0, self.kp1 = max(self.k0 - 1, 0), min(self.k1 + 1, nz)  # pattern layers (with ghosts)
        self.plane = (p * nx + 1) * (p * ny + 1)  # nodes per lattice plane
        self.node_offset = p * self.kp0 * self.plane  # local node = global node - node_offset
        self.num_local_nodes = self.plane * (p * (self.kp1 - self.kp0) + 1)
        # row window: lattice planes p*k0 .. p*k1 (inclusive), in local numbering
        self.row_begin = p * (self.k0 - self.kp0) * self.plane
        self.row_end = (p * (self.k1 - self.kp0) + 1) * self.plane
        self.lower = None if self.rank == 0 else (self.row_begin, self.row_begin + self.plane)
        self.upper = None if self.rank == self.world - 1 else (self.row_end - self.plane, self.row_end)

    @property
    def assembly_layers(self) -> tuple[int, int]:
        """Cell layers whose cells complete every owned row without an exchange (ghost mode): the
        slab's layers plus the layer above (its upper interface plane is owned here)."""
        return self.k0, min(self.k1 + 1, self.n[2])

    @property
    def owned_rows(self) -> tuple[int, int]:
        """Rows this rank owns (interface planes belong to the lower rank)."""
        return (self.row_begin + (self.plane if self.rank > 0 else 0), self.row_end)

    def to_local(self, global_nodes: torch.Tensor) -> torch.Tensor:
        return (global_nodes.to(torch.int64) - self.node_offset).to(torch.int32)


def make_pair_groups(world: int):
    """One 2-rank group per slab boundary (created collectively, same order on every rank)."""
    import torch.distributed as dist

    return [dist.new_group([q, q + 1]) for q in range(world - 1)]


def interface_slices(part: SlabPartition, indptr: torch.Tensor):
    """Value-block ranges (relative to the window base) of the lower/upper interface planes."""
    ip = indptr
    base = int(ip[part.row_begin])
    out = {}
    for name, rr in (("lower", part.lower), ("upper", part.upper)):
        if rr is not None:
            out[name] = (int(ip[rr[0]]) - base, int(ip[rr[1]]) - base)
    return out


def interface_suffix(part: SlabPartition, indptr: torch.Tensor, indices: torch.Tensor) -> dict:
    """Per interface plane: the window-relative block indices of its rows' blocks whose column lies
    in the plane or above it. Lattice numbering is plane-major, so that is "column >= the plane's
    first node". The rank above a plane contributes to those blocks only (its cells lie above), so
    summing them gives the plane's owner -- the rank below (doc.tex:464) -- complete rows, while
    about a third of each interface row (columns below the plane, the owner's alone) never
    crosses the link. Both ranks select the same blocks in the same order (identical patterns)."""
    base = int(indptr[part.row_begin])
    out = {}
    for name, rr in (("lower", part.lower), ("upper", part.upper)):
        if rr is None:
            continue
        b0, b1 = int(indptr[rr[0]]), int(indptr[rr[1]])
        sel = torch.nonzero(indices[b0:b1] >= rr[0]).flatten()
        out[name] = (sel + (b0 - base)).to(torch.int64)
    return out


def bc_diagonal_fixups(part: SlabPartition, indptr: torch.Tensor, indices: torch.Tensor, marker: torch.Tensor | None,
                       bs: int) -> torch.Tensor | None:
    """Flat value indices (window-relative) of Dirichlet diagonal entries on interface rows."""
    if marker is None:
        return None
    # vectorised over the planes' blocks (no per-row host round trips): the diagonal block of each
    # row is the one whose column equals the row; rows ascending, then components
    idx = []
    base = int(indptr[part.row_begin])
    for rr in (part.lower, part.upper):
        if rr is None or rr[1] <= rr[0]:
            continue
        b0, b1 = int(indptr[rr[0]]), int(indptr[rr[1]])
        counts = indptr[rr[0] + 1:rr[1] + 1] - indptr[rr[0]:rr[1]]
        rowid = torch.repeat_interleave(torch.arange(rr[0], rr[1], device=indptr.device), counts)
        dpos = torch.nonzero(indices[b0:b1].to(torch.int64) == rowid).flatten()
        if dpos.numel() != rr[1] - rr[0]:
            raise ValueError("interface rows without a diagonal block in the pattern")
        m = marker.reshape(-1, bs)[rowid[dpos]] != 0  # [nrows, bs]
        k, i = torch.nonzero(m, as_tuple=True)
        idx.append((dpos[k] + (b0 - base)) * (bs * bs) + i * (bs + 1))
    if not idx:
        return None
    out = torch.cat(idx).to(torch.int64)
    return out if out.numel() else None


def _host_staged_ready(t: torch.Tensor, group) -> None:
    """gloo (the CPU rehearsal backend) copies a device tensor to the host on its own thread, without
    waiting for the work queued on the current stream: the tensor must be complete before the call.
    RCCL orders its transfers after the current stream itself, so nothing waits there."""
    import torch.distributed as dist

    if t.is_cuda and dist.get_backend(group) == "gloo":
        torch.cuda.current_stream(t.device).synchronize()


def exchange_interfaces(part: SlabPartition, values: torch.Tensor, slices: dict, groups, fixups=None,
                        diagonal: float = 1.0, async_op: bool = False, suffix: dict | None = None,
                        oneway: bool = False):
    """Combine the interface-plane rows with the slab neighbours, then reset the Dirichlet diagonals
    of interface rows. `values` = the window's [nblocks_window, bs, bs].

    oneway (needs `suffix`): the rank above each plane sends its blocks in or above the plane
    (``interface_suffix``) to the plane's owner, the rank below, which adds them into its rows: the
    owner's rows are complete, the sender's copy keeps its own partial sums. Each rank sends down
    and receives from above on two different links at once.
    Otherwise a 2-rank all-reduce per boundary: of those suffix blocks (`suffix`; the owner's rows
    complete, the non-owner's copy holds the summed suffix) or of whole interface rows (`suffix`
    None; both copies equal).
    async_op: only issue the transfers (RCCL runs them on its own streams, after the work already
    queued on the current stream) and return a handle for ``finish_exchange``; the caller can queue
    the interior rows meanwhile."""
    import torch.distributed as dist

    flat = values.reshape(values.shape[0], -1)
    steps = []
    if part.lower is not None:
        steps.append((part.rank - 1, "lower"))  # boundary q = rank-1
    if part.upper is not None:
        steps.append((part.rank, "upper"))  # boundary q = rank
    pending = []
    if oneway:
        if suffix is None:
            raise ValueError("the one-way exchange sends the interface suffix: pass suffix=interface_suffix(...)")
        # send the lower plane's suffix down, receive the upper plane's from above (different peers
        # and links: issued together, no ordering constraint between them)
        for q, name in steps:
            idx = suffix[name]
            if name == "lower":
                buf = flat.index_select(0, idx)
                _host_staged_ready(buf, groups[q])
                w = dist.isend(buf, dst=part.rank - 1, group=groups[q])
                pending.append((w, None, buf, "send"))
            else:
                buf = torch.empty((idx.numel(), flat.shape[1]), dtype=flat.dtype, device=flat.device)
                w = dist.irecv(buf, src=part.rank + 1, group=groups[q])
                pending.append((w, idx, buf, "add"))
    else:
        # phase order: even boundaries first, then odd -- consistent on both sides of every boundary
        for q, name in sorted(steps, key=lambda s: (s[0] % 2, s[0])):
            if suffix is not None:
                idx = suffix[name]
                buf = flat.index_select(0, idx)
            else:
                b0, b1 = slices[name]
                idx, buf = None, flat[b0:b1]
            _host_staged_ready(buf, groups[q])
            w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=groups[q], async_op=True)
            pending.append((w, idx, buf, "copy"))
    handle = (pending, flat, values, fixups, diagonal)
    if async_op:
        return handle
    finish_exchange(handle)
    return None


def finish_exchange(handle):
    """Wait for the transfers of ``exchange_interfaces(async_op=True)`` (the current stream waits on
    RCCL's), add / scatter the received blocks and reset the Dirichlet diagonals of the interface rows."""
    pending, flat, values, fixups, diagonal = handle
    for w, idx, buf, how in pending:
        if w is not None:
            w.wait()
        if idx is None:
            continue
        if how == "add":
            flat.index_add_(0, idx, buf)
        else:
            flat.index_copy_(0, idx, buf)
    if fixups is not None:
        values.view(-1)[fixups] = diagonal


def interface_dof_ranges(part: SlabPartition, bs: int) -> dict:
    """Dof ranges (local numbering) of the lower / upper interface planes: contiguous, since the
    lattice numbering is plane-major and dofs are blocked (dof = node * bs + comp)."""
    out = {}
    for name, rr in (("lower", part.lower), ("upper", part.upper)):
        if rr is not None:
            out[name] = (rr[0] * bs, rr[1] * bs)
    return out


def exchange_vector_interfaces(part: SlabPartition, b: torch.Tensor, bs: int, groups, async_op: bool = False):
    """The ghost update of a slab-assembled vector: VecGhostUpdateBegin/End(ADD_VALUES,
    SCATTER_REVERSE) of the reference's setF (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:830-831).
    Each interface plane's dofs are summed over the two ranks sharing it (one 2-rank all-reduce per
    boundary, the matrix exchange's groups and phase order), after which both copies -- the owner's
    (lower rank, doc.tex:464) and the neighbour's ghost copy -- hold the complete entries."""
    import torch.distributed as dist

    steps = []
    if part.lower is not None:
        steps.append((part.rank - 1, "lower"))
    if part.upper is not None:
        steps.append((part.rank, "upper"))
    rng = interface_dof_ranges(part, bs)
    works = []
    for q, name in sorted(steps, key=lambda s: (s[0] % 2, s[0])):
        d0, d1 = rng[name]
        _host_staged_ready(b, groups[q])
        works.append(dist.all_reduce(b[d0:d1], op=dist.ReduceOp.SUM, group=groups[q], async_op=async_op))
    if async_op:
        return works
    return None


def slab_state(V, kind: str):
    """The config-E state: u = 1e-3 (sin pi x, sin pi y, sin pi z) at V's nodes."""
    if kind != "neo":
        return None
    return (1e-3 * torch.sin(torch.pi * V.tabulate_dof_coordinates())).reshape(-1).contiguous()


class SlabProblem:
    """One rank's share of the config-E assembly on its GPU (bench.py at N > 1): 3-D P2 on the unit
    cube, E = E_range[global cell % 200], nu = 0.3, x = 0 clamped, x = 1 prescribed; form
    "linear" (elasticity, the reference J at d = 0) or "neo" (neo-Hookean, device AD tangent at
    u = 1e-3 sin(pi x)). ``assemble()`` = local gather assembly + interface exchange;
    ``assemble_residual()`` = the reference's setF sequence on the slab with the ghost update.

    mode "exchange" (default, the RCCL path) or "ghost": the communication-free alternative of
    SURVEY §8(e) (dolfinx GhostMode.shared_facet, doc.tex:448-453) -- the rank also assembles the
    cell layer above its slab, so the rows it owns (its upper interface plane included) are complete
    without any exchange, at the price of one redundant layer of cells; its matrix window is its
    owned rows only. ``assemble_residual`` is exchange-mode only."""

    def __init__(self, n: int, rank: int, world: int, device, degree: int = 2, nu: float = 0.3, groups=None,
                 cell_type=None, exchange: str = "oneway", form: str = "linear", qdeg: int | None = None,
                 mode: str = "exchange"):
        from . import fem, mesh
        from .la import MatrixCSR
        from .materials import e_range

        ct = mesh.CellType.tetrahedron if cell_type is None else cell_type
        part = SlabPartition((n, n, n), degree, rank, world)
        self.part = part
        L = (1.0, 1.0, 1.0)
        m_pat = mesh.create_box(L, (n, n, n), ct, device=device, z_range=(part.kp0, part.kp1))
        if mode not in ("exchange", "ghost"):
            raise ValueError(f"unknown slab mode {mode}")
        self.mode = mode
        # ghost mode: cells of the layer above the slab too (complete rows on the upper plane)
        zr = part.assembly_layers if mode == "ghost" else (part.k0, part.k1)
        m_asm = mesh.create_box(L, (n, n, n), ct, device=device, z_range=zr)
        nloc = part.num_local_nodes
        dof_pat = part.to_local(fem._structured_dofmap(m_pat, degree)[0])
        dof_asm = part.to_local(fem._structured_dofmap(m_asm, degree)[0])
        V_pat = fem.FunctionSpace.from_dofmap(m_pat, degree, 3, dof_pat, nloc)
        V = fem.FunctionSpace.from_dofmap(m_asm, degree, 3, dof_asm, nloc)
        xs = fem._structured_node_coordinates(m_asm, degree)
        V._x = xs[part.node_offset:part.node_offset + nloc].contiguous()
        del xs
        a_pat = fem.LinearElasticity(V_pat, E=1.0, nu=nu)
        pat = fem.create_matrix(a_pat)
        win = part.owned_rows if mode == "ghost" else (part.row_begin, part.row_end)
        self.A = MatrixCSR(pat.indptr, pat.indices, 3, window=win)
        V_pat._adjacency = None  # the pattern's adjacency is not needed after create_matrix
        cells_per_layer = n * n * (6 if ct == mesh.CellType.tetrahedron else 1)
        cid = torch.arange(m_asm.num_cells, device=device, dtype=torch.int64) + part.k0 * cells_per_layer
        E = torch.tensor(e_range(), dtype=torch.float64, device=device)[cid % 200]
        self.form_kind = form
        self.u = slab_state(V, form)
        if form == "neo":
            self.a = fem.NeoHookean(V, E=E, nu=nu, u=self.u, quadrature_degree=2 if qdeg is None else qdeg)
        elif form == "linear":
            self.a = fem.LinearElasticity(V, E=E, nu=nu, quadrature_degree=qdeg)
        else:
            raise ValueError(f"unknown form {form}")
        left = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.zeros_like(x[0])))
        right = fem.locate_dofs_geometrical(V, lambda x: torch.isclose(x[0], torch.ones_like(x[0])))
        self.bcs = [fem.dirichletbc(0.0, left, V), fem.dirichletbc([0.01, 0.0, 0.0], right, V)]
        marker, _ = fem._combine_bcs(V, self.bcs)
        self.V = V
        self.num_cells = n * n * (part.k1 - part.k0) * (6 if ct == mesh.CellType.tetrahedron else 1)
        self.num_cells_assembled = m_asm.num_cells
        if mode == "ghost":
            self.split, self.n_iface, self.slices, self.suffix, self.fixups = None, 0, {}, None, None
            self.exchange_bytes = 0
            self.groups = groups
            self.kernel_name = ("k_cell_records + k_gather over the owned rows, cells of the slab and the "
                                "layer above (no exchange)")
            return
        # rows in three kinds of range: the interface planes (assembled first, then exchanged
        # while the interior rows assemble) and the interior
        iface = [rr for rr in (part.lower, part.upper) if rr is not None]
        inner = (part.row_begin + (part.plane if part.lower else 0), part.row_end - (part.plane if part.upper else 0))
        self.split = fem.SplitGather(self.a, self.bcs, self.A, iface + [inner])
        self.n_iface = len(iface)
        if exchange not in ("oneway", "suffix", "rows"):
            raise ValueError(f"unknown exchange {exchange}")
        self.exchange = exchange
        self.slices = interface_slices(part, self.A.indptr)
        self.suffix = interface_suffix(part, self.A.indptr, self.A.indices) if exchange != "rows" else None
        bs2 = 9
        if exchange == "oneway":  # sent per assembly: the lower plane's suffix (to the rank below)
            nblk = int(self.suffix["lower"].numel()) if "lower" in self.suffix else 0
            nrecv = int(self.suffix["upper"].numel()) if "upper" in self.suffix else 0
        elif self.suffix is not None:  # all-reduced: sent (and received) on each boundary
            nblk = sum(int(v.numel()) for v in self.suffix.values())
            nrecv = nblk
        else:
            nblk = sum(b1 - b0 for b0, b1 in self.slices.values())
            nrecv = nblk
        self.exchange_bytes = 8 * bs2 * nblk  # bytes this rank sends per assembly
        self.exchange_recv_bytes = 8 * bs2 * nrecv  # bytes it receives
        self.fixups = bc_diagonal_fixups(part, self.A.indptr, self.A.indices, marker, 3)
        self.groups = groups if groups is not None else make_pair_groups(world)
        self.kernel_name = ("k_cell_records + k_gather (interface planes, then interior rows) + per slab "
                            "boundary " + ("a one-way send of the upper rank's plane blocks to the owner"
                                           if exchange == "oneway" else "a 2-rank all_reduce(SUM)")
                            + ", overlapping the interior rows")

    def plan(self):
        """Build the gather plans now (ghost mode plans lazily at the first assembly; the exchange
        mode's SplitGather planned its row ranges at construction)."""
        if self.mode == "ghost":
            from . import fem

            fem.gather_plan(self.V, self.A, 0, self.a.kind)

    def assemble(self, overlap: bool = True, check: bool = False):
        """Records of all cells; the interface-plane rows; their 2-rank all-reduces issued on
        RCCL's stream; the interior rows on the compute stream meanwhile; wait; bc diagonals.
        (ghost mode: one gather over the owned rows, nothing exchanged.) check (ghost mode):
        FA_CHECK_ERRORS -- the slab's pattern is a superset of its assembled cells' pairs."""
        if self.mode == "ghost":
            from . import fem

            fem.assemble_matrix(self.a, bcs=self.bcs, A=self.A, check=check)
            return
        sg = self.split
        sg.prepare()
        for i in range(self.n_iface):
            sg.rows(i)
        ow = self.exchange == "oneway"
        if overlap:
            h = exchange_interfaces(self.part, self.A.parts[0][2], self.slices, self.groups, self.fixups,
                                    async_op=True, suffix=self.suffix, oneway=ow)
            sg.rows(self.n_iface)
            finish_exchange(h)
        else:
            sg.rows(self.n_iface)
            exchange_interfaces(self.part, self.A.parts[0][2], self.slices, self.groups, self.fixups,
                                suffix=self.suffix, oneway=ow)

    def assemble_residual(self, f: torch.Tensor | None = None, b: torch.Tensor | None = None) -> torch.Tensor:
        """The reference's setF on this slab (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:817-845):
        b = 0; assemble_vector(b, F) over the rank's cells; apply_lifting(b, {J}, {bcs}, {u}, -1);
        ghost update ADD / REVERSE (exchange_vector_interfaces); set_bc(b, bcs, u, -1). Returns the
        local dof vector [num_local_nodes * 3]: owned rows complete, interface copies consistent."""
        from . import fem

        if self.mode != "exchange":
            raise NotImplementedError("assemble_residual: exchange mode")
        V, a = self.V, self.a
        if b is None:
            b = torch.zeros(V.num_dofs, dtype=torch.float64, device=V.mesh.device)
        else:
            b.zero_()
        F = copy.copy(a)  # the residual form: J's coefficients and state, plus the body force f
        F.f = f
        fem.assemble_vector(F, b)
        x0 = None if F.u is None else [F.u]
        fem.apply_lifting(b, [F], [self.bcs], x0=x0, alpha=-1.0)
        exchange_vector_interfaces(self.part, b, V.bs, self.groups)
        fem.set_bc(b, self.bcs, x0=F.u, alpha=-1.0)
        return b
