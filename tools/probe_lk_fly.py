"""A/B of lk_multi's level setup: Scharr derivatives read from the pyramid's
planes (default) vs derived in the kernel from the u8 window (ctx option
lk_scharr_fly).  Checks the outputs are identical, then times both on the
1080p 128-box point set replicated to several sizes (HIP events, 20 reps)."""
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
        pts.append(np.stack([rng.uniform(x - 8, x + w + 8, 256), rng.uniform(y - 8, y + h + 8, 256)], 1))
base = np.concatenate(pts).astype(np.float32)
# a few points at and beyond the frame edges (the derivative planes' zero frame)
edge = np.array([[0, 0], [1919.5, 1079.5], [3, 540], [1915, 20], [-5, 100], [960, 1085], [10.25, 1070.75]], np.float32)
base = np.concatenate([edge, base])
P0 = klt.Pyramid(ctx, W, H, 2).build(frames[0])
P1 = klt.Pyramid(ctx, W, H, 2).build(frames[1])
lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)


def timed(p, reps=20):
    d = torch.from_numpy(p).cuda()
    for _ in range(3):
        r = lk.calc(P0, P1, d, want_iters=True)
    torch.cuda.synchronize()
    ctx.timing_enable(True)
    for _ in range(reps):
        r = lk.calc(P0, P1, d, want_iters=True)
    torch.cuda.synchronize()
    c, ms = ctx.timing_query("lk_sparse")
    ctx.timing_enable(False)
    return ms / c * 1000, r


res = {}
for fly in (0, 1):
    ctx.set_option("lk_scharr_fly", fly)
    res[fly] = {}
    for mult in (0.125, 0.6, 1, 4):
        n = int(len(base) * mult)
        p = np.resize(base, (n, 2)).astype(np.float32)
        t, r = timed(p)
        res[fly][n] = (t, r.next_pts.cpu().numpy(), r.status.cpu().numpy(), r.err.cpu().numpy())
ctx.set_option("lk_scharr_fly", 0)
for n in res[0]:
    a, b = res[0][n], res[1][n]
    same = np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])
    print(f"n {n:7d}: planes {a[0]:7.1f} us  fly {b[0]:7.1f} us  ({b[0] / a[0]:.3f})  identical={same}")
