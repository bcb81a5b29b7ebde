import sys, os, ctypes, torch
sys.path.insert(0, "fem-libraries_amd")
from femasm import _lib
L = _lib.load()
dev = torch.device("cuda", 0)
for gib in (4.0, 16.0):
    n = int(gib * (1 << 30)) // 8 // 2 * 2
    a = torch.ones(n, dtype=torch.float64, device=dev); b = torch.empty(n, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev); sh = st.cuda_stream
    for mode, name, nb in ((0,"copy nt",16*n),(5,"copy plain",16*n),(1,"write nt",8*n),(3,"write plain",8*n),(6,"write nt 4x grid",8*n),(7,"write plain 4x grid",8*n),(2,"read nt",8*n),
                         (10,"span4 nt",8*n),(11,"span4 plain",8*n),(12,"span16 nt",8*n),(13,"span16 plain",8*n),
                         (14,"lane64 nt",8*n),(15,"lane64 plain",8*n),(16,"span1 nt",8*n),(17,"span1 plain",8*n),
                         (18,"span4 plain half grid",8*n),(19,"span4 plain 2x grid",8*n),
                         (20,"oneshot 4KB/WG plain",8*n),(21,"oneshot 16KB/WG plain",8*n),(22,"oneshot 16KB/WG nt",8*n),
                         (23,"oneshot 8KB/WG lane32",8*n),(24,"oneshot 32KB/WG plain",8*n)):
        L.fa_hbm_probe(mode, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a.data_ptr()), n, sh)
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st); rc = L.fa_hbm_probe(mode, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a.data_ptr()), n, sh); e1.record(st); e1.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e-3)
        print(f"{gib:5.1f} GiB {name:22s} {nb/best/1e9:8.1f} GB/s rc={rc}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record(st); b.fill_(0.0); e1.record(st); e1.synchronize(); best = min(best, e0.elapsed_time(e1)*1e-3)
    print(f"{gib:5.1f} GiB torch fill_              {8*n/best/1e9:8.1f} GB/s")
    best = 1e9
    for _ in range(5):
        e0.record(st); b.fill_(1.5); e1.record(st); e1.synchronize(); best = min(best, e0.elapsed_time(e1)*1e-3)
    print(f"{gib:5.1f} GiB torch fill_(1.5)         {8*n/best/1e9:8.1f} GB/s")
    best = 1e9
    for _ in range(5):
        e0.record(st); b.copy_(a); e1.record(st); e1.synchronize(); best = min(best, e0.elapsed_time(e1)*1e-3)
    print(f"{gib:5.1f} GiB torch copy_              {16*n/best/1e9:8.1f} GB/s")
    del a, b; torch.cuda.empty_cache()
