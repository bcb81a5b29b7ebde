"""Diagnostic: gather-assembly time vs mesh size, and raw fill bandwidth of large tensors."""
import subprocess, sys, time, torch
dev = torch.device("cuda", 0)
for gb in (4, 40, 140):
    t = torch.empty(int(gb * 1e9 / 8), dtype=torch.float64, device=dev)
    t.fill_(1.0); torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(3): t.fill_(2.0)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - s) / 3
    print(f"fill {gb} GB: {gb / dt:.0f} GB/s", flush=True)
    del t
    torch.cuda.empty_cache()
