"""The GPU slab path end to end on one card: 2-3 ranks share cuda:0, each runs the HIP gather
kernel on its slab (femasm.parallel.SlabProblem: interface planes first, their suffix all-reduce
overlapping the interior rows) with gloo standing in for RCCL (which needs one GPU per rank; the
8-GPU RCCL run is the driver's). Every owned row must equal a single-process full-mesh GPU
assembly; a non-owned interface copy must hold the exchanged blocks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(kind):
    import bench

    return bench.CONFIGS[{"neo": "Eneo", "p1": "C"}.get(kind, "E")]


def _slab(n, rank, world, dev, kind, **kw):
    from femasm import parallel

    if kind == "p1":  # P1 tetrahedra: the slab's own node numbering (from_dofmap), not the mesh's vertices
        return parallel.SlabProblem(n, rank, world, dev, degree=1, **kw)
    return parallel.SlabProblem(n, rank, world, dev, form=kind, **kw)


def _worker(rank, world, port, n, kind="linear"):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from femasm import fem, parallel
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rowparity

    dev = torch.device("cuda", 0)
    prob = _slab(n, rank, world, dev, kind)
    prob.assemble()
    torch.cuda.synchronize()
    m, V, a, bcs = bench.build_problem(n, dev, cfg=_cfg(kind))
    A = fem.assemble_matrix(a, bcs=bcs)
    part = prob.part
    ip_l = prob.A.indptr.cpu().numpy()
    ix_l = prob.A.indices.cpu().numpy()
    vl = prob.A.parts[0][2].cpu().numpy()
    ip_g = A.indptr.cpu().numpy()
    ix_g = A.indices.cpu().numpy()
    vg = A.data.cpu().numpy()
    w0 = ip_l[part.row_begin]
    got, ref, ptr = [], [], [0]
    for r in range(part.row_begin, part.row_end):
        g = r + part.node_offset
        lc = ix_l[ip_l[r]:ip_l[r + 1]]
        assert np.array_equal(lc + part.node_offset, ix_g[ip_g[g]:ip_g[g + 1]])
        lv, gv = vl[ip_l[r] - w0:ip_l[r + 1] - w0], vg[ip_g[g]:ip_g[g + 1]]
        if part.lower is not None and r < part.lower[1]:  # non-owned copy
            if prob.exchange == "oneway":
                continue  # the rank's own partial sums, sent to the owner
            keep = lc >= part.lower[0]  # suffix all-reduce: the exchanged blocks only
            lv, gv = lv[keep], gv[keep]
        got.append(lv)
        ref.append(gv)
        ptr.append(ptr[-1] + len(lv))
    # per scalar row, each row held to its own scale (tests/rowparity.py)
    rowparity.assert_rows_close(np.concatenate(got), np.concatenate(ref), np.array(ptr), what=f"rank {rank}:")
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,kind", [(2, 6, "linear"), (3, 7, "linear"), (2, 6, "neo"), (3, 7, "p1")])
def test_slab_problem_gpu_gloo(world, n, kind):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mp.spawn(_worker, args=(world, _port(), n, kind), nprocs=world, join=True)


def _residual_worker(rank, world, port, n, kind):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import copy

    import bench
    from femasm import fem, parallel

    dev = torch.device("cuda", 0)
    prob = parallel.SlabProblem(n, rank, world, dev, form=kind)
    fl = torch.tensor([0.5, -1.0, 2.0], dtype=torch.float64, device=dev).repeat(prob.V.num_nodes)
    b = prob.assemble_residual(f=fl)
    torch.cuda.synchronize()
    # single process, whole mesh: the same setF sequence without a ghost update
    m, V, a, bcs = bench.build_problem(n, dev, cfg=bench.CONFIGS["Eneo" if kind == "neo" else "E"])
    F = copy.copy(a)
    F.f = torch.tensor([0.5, -1.0, 2.0], dtype=torch.float64, device=dev).repeat(V.num_nodes)
    gb = fem.assemble_vector(F)
    fem.apply_lifting(gb, [F], [bcs], x0=None if F.u is None else [F.u], alpha=-1.0)
    fem.set_bc(gb, bcs, x0=F.u, alpha=-1.0)
    part = prob.part
    r0, r1 = part.owned_rows
    off = part.node_offset
    own, ref = b[r0 * 3:r1 * 3].cpu(), gb[(r0 + off) * 3:(r1 + off) * 3].cpu()
    scale = float(gb.abs().max())
    err = float((own - ref).abs().max())
    assert err <= 1e-12 * scale, f"rank {rank}: residual rel err {err / scale:.2e}"
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,kind", [(2, 6, "linear"), (3, 7, "neo")])
def test_slab_residual_gpu_gloo(world, n, kind):
    """Sharded residual (assemble_vector + apply_lifting + ghost update + set_bc) on slabs sharing
    one GPU equals the single-process residual on every owned dof."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mp.spawn(_residual_worker, args=(world, _port(), n, kind), nprocs=world, join=True)


@pytest.mark.parametrize("world,n,kind", [(2, 6, "linear"), (3, 7, "neo"), (3, 7, "p1")])
def test_slab_ghost_mode_gpu(world, n, kind):
    """SlabProblem(mode="ghost"): no exchange; each rank's owned rows (HIP gather over its slab plus
    the layer above) equal the single-process full-mesh GPU assembly. The ranks need no
    communication, so they run one after the other in this process. The assembly runs with
    FA_CHECK_ERRORS: the slab pattern (built over the ghost layers too) is a superset of the pairs
    of the cells it assembles, which the check must accept. P1 ("p1"): the slab's node numbering
    differs from its mesh's vertex numbering, and ranks > 0 have more nodes than vertices."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "fem-libraries_amd"))
    import bench
    from femasm import fem, parallel
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rowparity

    dev = torch.device("cuda", 0)
    m, V, a, bcs = bench.build_problem(n, dev, cfg=_cfg(kind))
    A = fem.assemble_matrix(a, bcs=bcs)
    ip_g, ix_g, vg = A.indptr.cpu().numpy(), A.indices.cpu().numpy(), A.data.cpu().numpy()
    for rank in range(world):
        prob = _slab(n, rank, world, dev, kind, mode="ghost")
        prob.assemble(check=True)
        torch.cuda.synchronize()
        part = prob.part
        r0, r1 = part.owned_rows
        assert prob.A.parts[0][:2] == (r0, r1) and prob.exchange_bytes == 0
        ip_l, ix_l = prob.A.indptr.cpu().numpy(), prob.A.indices.cpu().numpy()
        vl = prob.A.parts[0][2].cpu().numpy()
        w0 = ip_l[r0]
        g0, g1 = r0 + part.node_offset, r1 + part.node_offset
        for r in range(r0, r1):
            g = r + part.node_offset
            assert np.array_equal(ix_l[ip_l[r]:ip_l[r + 1]] + part.node_offset, ix_g[ip_g[g]:ip_g[g + 1]])
        # owned rows are one contiguous value range on both sides: per-row parity over it
        rowparity.assert_rows_close(vl[ip_l[r0] - w0:ip_l[r1] - w0], vg[ip_g[g0]:ip_g[g1]], ip_l[r0:r1 + 1] - ip_l[r0],
                                    what=f"rank {rank}:")
