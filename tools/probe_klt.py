"""Quick kernel probe: 1080p synthetic pair, 128 boxes x 256 points, 3-level LK."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from opencv_amd import klt

ctx = klt.Context.get(0)
W, H, NOBJ = 1920, 1080, 128
frames, gt = klt.synth_render(20261015, W, H, NOBJ, 0, 2, ctx=ctx)
pts = []
rng = np.random.default_rng(0)
for o in range(NOBJ):
    v, x, y, w, h = gt[0, o].tolist()
    if not v: continue
    pts.append(np.stack([rng.uniform(x, x + w, 256), rng.uniform(y, y + h, 256)], 1))
pts = torch.from_numpy(np.concatenate(pts).astype(np.float32)).cuda()
n = pts.shape[0]
P0 = klt.Pyramid(ctx, W, H, 2).build(frames[0])
P1 = klt.Pyramid(ctx, W, H, 2).build(frames[1])
lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)
for _ in range(3):
    r = lk.calc(P0, P1, pts, want_iters=True)
torch.cuda.synchronize()
ctx.timing_enable(True)
t = time.time()
for _ in range(20):
    P1.build(frames[1])
    r = lk.calc(P0, P1, pts, want_iters=True)
torch.cuda.synchronize()
wall = (time.time() - t) / 20
for k in ["pyr_build", "lk_sparse"]:
    c, ms = ctx.timing_query(k)
    print(f"{k}: {c} launches, avg {ms / c * 1000:.1f} us")
st = r.status.cpu().numpy(); it = r.iters.cpu().numpy()
print(f"points {n}, tracked {st.mean():.3f}, mean iters {it.mean():.2f}, wall/iter {wall*1e3:.3f} ms")
# the fp16 pixel path on the same frames and points
Q0 = klt.Pyramid(ctx, W, H, 2, dtype=torch.float16).build(frames[0])
Q1 = klt.Pyramid(ctx, W, H, 2, dtype=torch.float16).build(frames[1])
ctx.timing_enable(True)
for _ in range(20):
    r16 = lk.calc(Q0, Q1, pts, want_iters=True)
torch.cuda.synchronize()
c, ms = ctx.timing_query("lk_sparse")
print(f"fp16 lk_sparse: avg {ms / c * 1000:.1f} us; mean iters {r16.iters.float().mean().item():.2f}")
# the other kernels for comparison (impl 1 strip, 2 generic LDS, 3 multi-point)
for impl in (1, 2, 3):
    lk2 = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30, impl=impl)
    ctx.timing_enable(True)
    for _ in range(20):
        r2 = lk2.calc(P0, P1, pts, want_iters=True)
    torch.cuda.synchronize()
    c, ms = ctx.timing_query("lk_sparse")
    same = torch.equal(r2.next_pts, r.next_pts) and torch.equal(r2.status, r.status) and torch.equal(r2.iters, r.iters)
    print(f"impl {impl} lk_sparse: avg {ms / c * 1000:.1f} us; same result: {same}")
