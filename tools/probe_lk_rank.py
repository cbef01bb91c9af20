"""Newton steps of a PyrLK point against its corner's rank in its GFTT set
(corners come strongest first).  1080p synthetic pair, GFTT corners (256 per
box) of frame 1's boxes tracked 1 -> 2; per rank decile: mean iterations, and
per wave (three consecutive corners, as the loop's launches take them) the
mean and 99th percentile of the wave's max.  Question: do the long waves sit at
a predictable place in a set (a launch order that starts them first)?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from opencv_amd import klt  # noqa: E402


def main():
    ctx = klt.Context.get(0)
    W, H, NOBJ = 1920, 1080, 128
    frames, gt = klt.synth_render(20261015, W, H, NOBJ, 0, 3, ctx=ctx)
    rois = []
    for v, x, y, w, h in gt[1].numpy().tolist():
        x0, y0 = max(0, x), max(0, y)
        x1, y1 = min(W, x + w), min(H, y + h)
        if v and x1 - x0 >= 8 and y1 - y0 >= 8:
            rois.append((x0, y0, x1 - x0, y1 - y0))
    c, n = klt.GoodFeaturesToTrackDetector(256, 0.01, 3.0).detect_rois(frames[1], rois)
    c, n = c.cpu().numpy(), n.cpu().numpy()
    pts = np.concatenate([c[i, :n[i]] for i in range(len(rois))]).astype(np.float32)
    rank = np.concatenate([np.arange(n[i]) / max(1, n[i]) for i in range(len(rois))])
    P = [klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[i]) for i in (1, 2)]
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)
    r = lk.calc(P[0], P[1], torch.from_numpy(pts).cuda(), want_iters=True)
    torch.cuda.synchronize()
    it = r.iters.cpu().numpy().astype(np.int64)
    print(f"{len(pts)} points, mean iterations {it.mean():.2f}")
    dec = np.minimum((rank * 10).astype(int), 9)
    for d in range(10):
        m = dec == d
        print(f"rank decile {d}: {m.sum():6d} points, mean iters {it[m].mean():.2f}, p99 {np.percentile(it[m], 99):.0f}")
    # waves of three consecutive corners inside each set
    wmax, wrank = [], []
    off = 0
    for i in range(len(rois)):
        for j in range(0, n[i], 3):
            wmax.append(it[off + j:off + min(n[i], j + 3)].max())
            wrank.append(j / max(1, n[i]))
        off += n[i]
    wmax, wrank = np.array(wmax), np.array(wrank)
    wd = np.minimum((wrank * 10).astype(int), 9)
    for d in range(10):
        m = wd == d
        print(f"wave decile {d}: {m.sum():5d} waves, mean max {wmax[m].mean():.2f}, p99 {np.percentile(wmax[m], 99):.0f}")
    print("corr(rank, iters) =", np.corrcoef(rank, it)[0, 1].round(3))


if __name__ == "__main__":
    main()
