"""Diagnostic: does a large prior allocation slow the gather assembly (page-fragment / TLB effect)?
usage: alloc_probe.py N DUMMY_GB [ORDER]  (ORDER=before|after: dummy allocated before/after the problem)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402  (sets sys.path for femasm)
import torch  # noqa: E402
from femasm import fem  # noqa: E402

n, gb = int(sys.argv[1]), float(sys.argv[2])
order = sys.argv[3] if len(sys.argv) > 3 else "before"
dev = torch.device("cuda", 0)
dummy = torch.empty(int(gb * 1e9), dtype=torch.uint8, device=dev) if (gb > 0 and order == "before") else None
m, V, a, bcs = bench.build_problem(n, dev)
A = fem.create_matrix(a)
fem.gather_plan(V, A)
if gb > 0 and order == "after":
    dummy = torch.empty(int(gb * 1e9), dtype=torch.uint8, device=dev)
for _ in range(2):
    fem.assemble_matrix(a, bcs=bcs, A=A)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    fem.assemble_matrix(a, bcs=bcs, A=A)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 3
print(f"n={n} dummy={gb}GB ({order}): {dt*1e3:.1f} ms, {m.num_cells/dt/1e6:.1f} Melem/s, values {A.data.numel()*8/1e9:.1f} GB", flush=True)
