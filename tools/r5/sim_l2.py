"""Offline model of the gather's per-cell record re-fetches from beyond the L2 under several chunk
visiting orders (round 5). Structured P2-tet mesh, the linear plan's chunking (<= 455 blocks, <= 128
entries), one LRU of 128-B lines per XCD with a capacity scaled to E's plane size, record accesses in
each XCD's chunk sequence. Prints record line fetches per cell relative to the compulsory one."""
import sys
from collections import OrderedDict

import numpy as np
import torch

sys.path.insert(0, "/root/repo/fem-libraries_amd")
from femasm import fem, mesh as fmesh  # noqa: E402

# E's x extent (203 cubes: the lines and chunks of config E), fewer cube lines / layers in y, z
nx, ny, nz = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "203,24,8").split(","))
rec_b = int(sys.argv[2]) if len(sys.argv) > 2 else 80
MAXB = int(sys.argv[4]) if len(sys.argv) > 4 else 455  # 640: the neo plan
m = fmesh.create_box((1.0, 1.0, 1.0), (nx, ny, nz))
V = fem.functionspace(m, ("Lagrange", 2, (3,)))
cells = V.dofmap.numpy().astype(np.int64)
nc, nn = cells.shape
nnodes = V.num_nodes
# adjacency: entries sorted by node
ent_node = cells.reshape(-1)
order = np.argsort(ent_node, kind="stable")
ent_cell = order // nn
adj_cnt = np.bincount(ent_node, minlength=nnodes)
adj_ptr = np.concatenate([[0], np.cumsum(adj_cnt)])
# row lengths (distinct neighbours)
a = np.repeat(cells, nn, axis=1).reshape(-1)
b = np.tile(cells, (1, nn)).reshape(-1)
key = np.unique(a * nnodes + b)
row_len = np.bincount(key // nnodes, minlength=nnodes)
ip = np.concatenate([[0], np.cumsum(row_len)])
# chunking (plan_gather)
rs = [0]
start = 0
for r in range(nnodes):
    cb = ip[r + 1] - ip[start]
    ca = adj_ptr[r + 1] - adj_ptr[start]
    if r > start and (cb > MAXB or ca > 128 or r + 1 - start > 128):
        rs.append(r)
        start = r
rs.append(nnodes)
rs = np.array(rs)
nch = len(rs) - 1
side = 2 * nx + 1
sidey = 2 * ny + 1
print(f"box={nx}x{ny}x{nz} cells={nc} nodes={nnodes} chunks={nch} rows/chunk={nnodes/nch:.1f}")
# the L2 of one XCD: 4 MB of 128-B lines (the lines along x are E's)
cap_lines = int(sys.argv[3]) if len(sys.argv) > 3 else 4 * 2**20 // 128
print(f"scaled L2 capacity: {cap_lines} lines ({cap_lines*128/1024:.0f} KB)")
# chunk points: first entry's cell centroid -> lattice pos of the chunk's first row
r0 = rs[:-1]
I = r0 % side
J = (r0 // side) % sidey
K = r0 // (side * sidey)


def spread(v):
    v = v.astype(np.uint64) & np.uint64(0x1fffff)
    out = np.zeros_like(v)
    for bit in range(21):
        out |= ((v >> np.uint64(bit)) & np.uint64(1)) << np.uint64(3 * bit)
    return out


def morton(I, J, K):
    return spread(I) | (spread(J) << np.uint64(1)) | (spread(K) << np.uint64(2))


def seq_current():
    # blocks of 16 chunks dealt round-robin to 8 XCDs
    per = {x: [] for x in range(8)}
    for c in range(nch):
        per[(c // 16) % 8].append(c)
    return per


def seq_contig(perm):
    per = {}
    q = (nch + 7) // 8
    for x in range(8):
        per[x] = list(perm[x * q:(x + 1) * q])
    return per


def tiled(T):
    # (J,K) tiles of T x T lines, within a tile I-major then lines; tiles in row-major (K, J)
    tkey = (K // T) * ((sidey + T - 1) // T) + (J // T)
    return np.lexsort((I, J, K % T, tkey))


orders = {
    "current (16-blocks round robin)": seq_current(),
    "rows contiguous per XCD": seq_contig(np.arange(nch)),
    "morton per XCD": seq_contig(np.argsort(morton(I // 4, J, K), kind="stable")),
    "morton(I/16) per XCD": seq_contig(np.argsort(morton(I // 16, J, K), kind="stable")),
    "JK tiles 4": seq_contig(tiled(4)),
    "JK tiles 8": seq_contig(tiled(8)),
}
lines_per_rec = rec_b / 128.0
for name, per in orders.items():
    miss = 0
    acc = 0
    for x in range(8):
        lru = OrderedDict()
        for c in per[x]:
            for e in range(adj_ptr[rs[c]], adj_ptr[rs[c + 1]]):
                cell = int(ent_cell[e])
                lo = cell * rec_b // 128
                hi = (cell * rec_b + rec_b - 1) // 128
                for ln in range(lo, hi + 1):
                    acc += 1
                    if ln in lru:
                        lru.move_to_end(ln)
                    else:
                        miss += 1
                        lru[ln] = 1
                        if len(lru) > cap_lines:
                            lru.popitem(last=False)
    comp = nc * rec_b / 128
    print(f"{name:34s} line fetches / compulsory = {miss / comp:.2f}  (accesses/compulsory {acc / comp:.2f})")
