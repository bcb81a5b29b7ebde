"""How long does the device allocation of config E's value array (139 GB) take on this box? torch.empty
(caching allocator -> hipMalloc), after empty_cache, and a raw hipMalloc / hipFree of the same size,
repeated. One JSON line."""
import ctypes
import json
import time

import torch

dev = torch.device("cuda", 0)
torch.ones(1, device=dev)
torch.cuda.synchronize()
out = {}
nbytes = 139 * 10**9
for k in range(3):
    t = time.time()
    x = torch.empty(nbytes // 8, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    out[f"torch_empty_{k}"] = round(time.time() - t, 3)
    t = time.time()
    x[:1 << 20].fill_(1.0)
    torch.cuda.synchronize()
    out[f"first_touch_{k}"] = round(time.time() - t, 3)
    del x
    torch.cuda.empty_cache()
hip = ctypes.CDLL("libamdhip64.so")
for k in range(2):
    p = ctypes.c_void_p()
    t = time.time()
    rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes))
    hip.hipDeviceSynchronize()
    out[f"hipMalloc_{k}"] = (rc, round(time.time() - t, 3))
    t = time.time()
    hip.hipFree(p)
    hip.hipDeviceSynchronize()
    out[f"hipFree_{k}"] = round(time.time() - t, 3)
for gb in (1, 8, 32):
    t = time.time()
    x = torch.empty(gb * 10**9 // 8, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    out[f"torch_empty_{gb}GB"] = round(time.time() - t, 4)
    del x
    torch.cuda.empty_cache()
print(json.dumps(out))
