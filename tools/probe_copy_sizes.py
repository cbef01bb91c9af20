"""tbdk_hbm_copy (16 B/lane stream copy) rate vs buffer size: what a single
launch moving as many bytes as a pyramid build can reach (HIP events, best of
20 after warm-up; read + write bytes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from opencv_amd import klt

ctx = klt.Context.get(0)
st = torch.cuda.current_stream()
for mb in (1, 2, 4, 8, 11, 16, 32, 64, 256, 2048):
    n = mb << 20
    src = torch.ones(n, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    best = 1e9
    for i in range(25):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        klt.hbm_copy(dst, src, ctx=ctx, stream=st)
        e1.record(st)
        e1.synchronize()
        if i >= 5:
            best = min(best, e0.elapsed_time(e1))
    print(f"{mb:5d} MiB copy: {best * 1000:8.1f} us  {2 * n / (best / 1000) / 1e9:8.1f} GB/s", flush=True)
    del src, dst
