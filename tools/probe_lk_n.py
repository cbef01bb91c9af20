"""Standalone lk_multi (FLY instance: levels-only pyramids, as in the TBD loop)
launch time vs point count, 1080p synthetic pair, 128 boxes x 256 points
(replicated / cut to n), 3 levels, win 21; HIP events over 30 launches.
TBDK_LIB selects the build (A/B runs)."""
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
lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, int(os.environ.get("LK_ITERS", "30")))  # criteria maxCount
out = []
for n in [int(v) for v in (sys.argv[1:] or ["6000", "12000", "18000", "32000", "131000"])]:
    d = torch.from_numpy(np.resize(base, (n, 2)).astype(np.float32)).cuda()
    for _ in range(3):
        lk.calc(P0, P1, d)
    torch.cuda.synchronize()
    ctx.timing_select(["lk_sparse"])
    ctx.timing_enable(True)
    for _ in range(30):
        lk.calc(P0, P1, d)
    torch.cuda.synchronize()
    c, ms = ctx.timing_query("lk_sparse")
    ctx.timing_enable(False)
    out.append(f"n {n}: {ms / c * 1000:.1f} us")
print(os.path.basename(os.environ.get("TBDK_LIB", "libtbdk.so")), "maxCount", lk.iters, "; ".join(out), flush=True)
