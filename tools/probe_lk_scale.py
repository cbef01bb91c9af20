"""LK kernel time vs point count and point order (tail effects): 1080p synthetic
pair, 128 boxes x 256 points replicated, 3-level LK, win 21."""
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
    return ms / c * 1000, r


t, r = timed(base)
it = r.iters.cpu().numpy()
if it.max() >= 1000:  # a TBDK_LK_PROBE_RELOADS=2 build: reloads per wave in the thousands
    rl = it // 1000
    it = it % 1000
    print(f"J reloads per wave (per point's wave): mean {rl.mean():.2f} max {rl.max()}")
print(f"iters per point: mean {it.mean():.2f} p50 {np.percentile(it, 50):.0f} p90 {np.percentile(it, 90):.0f} "
      f"p99 {np.percentile(it, 99):.0f} max {it.max()}")
g = it[: len(it) // 3 * 3].reshape(-1, 3)
print(f"per 3-point group: mean of max {g.max(1).mean():.2f} (useful {it.mean() / g.max(1).mean():.2f})")
for mult in ((0.125, 0.5, 1, 4) if len(sys.argv) < 2 else (0.5, 1)):
    n = int(len(base) * mult)
    p = np.resize(base, (n, 2)).astype(np.float32)
    tt, _ = timed(p)
    print(f"n {n:7d}: {tt:7.1f} us  ({tt / n * 1e3:.2f} ns/point)")
order = np.argsort(-it, kind="stable")
tt, r2 = timed(base[order])
print(f"sorted by iterations (desc): {tt:.1f} us vs {t:.1f} us")
g2 = it[order][: len(it) // 3 * 3].reshape(-1, 3)
print(f"sorted per 3-point group: mean of max {g2.max(1).mean():.2f}")
