"""lk_multi (FLY, levels-only 1080p pyramids, 3 levels, win 21) at tiny point
counts, to expose one wave's latency chain; run under rocprofv3 --kernel-trace
for kernel durations (HIP events add a ~6 us floor).  Also prints the mean
iterations of the points."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from opencv_amd import klt

ctx = klt.Context.get(0)
W, H, NOBJ = 1920, 1080, 128
frames, gt = klt.synth_render(20261015, W, H, NOBJ, 0, 2, ctx=ctx)
rng = np.random.default_rng(0)
pts = []
for o in range(NOBJ):
    v, x, y, w, h = gt[0, o].tolist()
    if v:
        pts.append(np.stack([rng.uniform(x, x + w, 256), rng.uniform(y, y + h, 256)], 1))
base = np.concatenate(pts).astype(np.float32)
P0 = klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[0])
P1 = klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[1])
lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)
for n in [int(v) for v in (sys.argv[1:] or ["3", "3072", "18000"])]:
    d = torch.from_numpy(base[:n].copy()).cuda()
    for _ in range(20):
        r = lk.calc(P0, P1, d, want_iters=True)
    torch.cuda.synchronize()
    print(f"n {n}: mean iters {r.iters.float().mean().item():.2f} max {r.iters.max().item()}", flush=True)
