"""How much of a PyrLK wave's Newton work runs with a single point of its three
still active (TBDK_LIB = a build with -DTBDK_LK_PROBE_ITERS_LV: the iteration
output holds the steps per level, 8 bits each).  1080p synthetic pair, GFTT
corners (256 per box) of frame 1's boxes tracked 1 -> 2, three consecutive
points per wave as the loop's launches take them.  Per level a wave runs
max(steps) Newton steps; (max - second max) of them have one point active.
Prints the wave-steps, the one-point share, and a cost model of a wave
(setup S steps per level, a one-point step at cost c of a full one, a switch
cost of r steps) for the whole launch and its longest waves."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from opencv_amd import klt


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
    P = [klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[i]) for i in (1, 2)]
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)
    r = lk.calc(P[0], P[1], torch.from_numpy(pts).cuda(), want_iters=True)
    torch.cuda.synchronize()
    it = r.iters.cpu().numpy().astype(np.int64)
    lv = np.stack([(it >> (8 * L)) & 0xFF for L in (2, 1, 0)], axis=1)  # levels 2, 1, 0
    npts = len(pts) - len(pts) % 3
    w = lv[:npts].reshape(-1, 3, 3)  # wave, point, level
    srt = np.sort(w, axis=1)
    m1, m2 = srt[:, 2, :], srt[:, 1, :]
    steps = m1.sum()
    solo = (m1 - m2).sum()
    print(f"{len(pts)} points, {len(w)} waves; mean steps per point per level {lv.mean(axis=0).round(2)}; "
          f"wave-steps {steps}, of which one point active {solo} ({solo / steps:.3f}); useful "
          f"{lv[:npts].sum() / (3 * steps):.3f}", flush=True)
    per_wave = m1.sum(axis=1)
    top = np.argsort(-per_wave)[:max(1, len(w) // 100)]
    for S, cst, sw in ((4.0, 0.55, 1.0), (4.0, 0.65, 1.5), (4.0, 0.5, 0.5)):
        base = S * 3 + m1.sum(axis=1)
        # a level switches to one-point steps only when it has some (m1 > m2) and the switch pays
        gain = np.where(m1 - m2 > 0, (m1 - m2) * (1 - cst) - sw, 0.0)
        gain = np.maximum(gain, 0.0) if False else gain
        new = base - np.clip(gain, 0, None).sum(axis=1)
        print(f"setup {S} steps, one-point step {cst}, switch {sw}: total work {new.sum() / base.sum():.3f}, "
              f"longest 1% of waves {new[top].mean() / base[top].mean():.3f} (base {base[top].mean():.1f} steps), "
              f"max {new.max():.1f} vs {base.max():.1f}", flush=True)
    hist = np.bincount((m1 - m2).ravel(), minlength=31)
    print("per wave-level one-point steps histogram:", hist.tolist())


if __name__ == "__main__":
    main()
