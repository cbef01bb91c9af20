"""Per-wave latency of the multi-point LK kernel: one wave per SIMD (3072
points), several level / iteration limits; eps = 0 so every point runs
max_count Newton steps per level (unless it leaves the image)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
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
P0 = klt.Pyramid(ctx, W, H, 2).build(frames[0])
P1 = klt.Pyramid(ctx, W, H, 2).build(frames[1])
for n in (3072, 12288):
    d = torch.from_numpy(base[rng.permutation(len(base))[:n]].copy()).cuda()
    for ml, mc in ((0, 1), (0, 2), (0, 5), (0, 10), (1, 1), (2, 1), (2, 5)):
        lk = klt.SparsePyrLKOpticalFlow((21, 21), ml, mc, epsilon=0.0)
        for _ in range(3):
            r = lk.calc(P0, P1, d, want_iters=True)
        torch.cuda.synchronize()
        ctx.timing_enable(True)
        for _ in range(20):
            r = lk.calc(P0, P1, d, want_iters=True)
        torch.cuda.synchronize()
        c, ms = ctx.timing_query("lk_sparse")
        it = r.iters.cpu().numpy()
        extra = f", J reloads per wave {(it // 1000).mean():.2f}" if it.max() >= 1000 else ""
        print(f"n {n} levels {ml + 1} max_count {mc}: {ms / c * 1000:6.1f} us, mean iters {(it % 1000).mean():.2f}{extra}")
