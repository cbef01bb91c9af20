"""Does the order of a PyrLK launch's points move its time, and can the order
be predicted?  1080p synthetic sequence, GFTT corners (256 per box) of frame
0's boxes, tracked 0 -> 1 -> 2.  The 1 -> 2 launch (the points of the first
`nbox` boxes, ~1.4 rounds of the 4096 wave slots at 68 boxes, as the TBD
loop's refreshed-set launch) is timed with HIP events in several point orders:

  natural     the points as the boxes list them
  oracle      by their own 1 -> 2 iteration count, descending (longest first)
  predicted   by the same point's 0 -> 1 iteration count, descending
  boxmean     by the box's mean 0 -> 1 iteration count, descending (the only
              history a freshly detected corner set has)
  shuffled    random

and the correlation of a point's iterations across consecutive frame pairs is
printed.  TBDK_LIB selects the build."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from opencv_amd import klt


def main():
    nbox = int(sys.argv[1]) if len(sys.argv) > 1 else 68
    ctx = klt.Context.get(0)
    W, H, NOBJ = 1920, 1080, 128
    frames, gt = klt.synth_render(20261015, W, H, NOBJ, 0, 3, ctx=ctx)
    rois, boxid = [], []
    for v, x, y, w, h in gt[0].numpy().tolist():
        x0, y0 = max(0, x), max(0, y)
        x1, y1 = min(W, x + w), min(H, y + h)
        if v and x1 - x0 >= 8 and y1 - y0 >= 8:
            rois.append((x0, y0, x1 - x0, y1 - y0))
    det = klt.GoodFeaturesToTrackDetector(256, 0.01, 3.0)
    c, n = det.detect_rois(frames[0], rois)
    c, n = c.cpu().numpy(), n.cpu().numpy()
    pts = np.concatenate([c[i, :n[i]] for i in range(len(rois))]).astype(np.float32)
    box = np.concatenate([np.full(n[i], i) for i in range(len(rois))])
    rank = np.concatenate([np.arange(n[i]) for i in range(len(rois))])  # GFTT order: strongest corner first
    bx = np.array(rois, dtype=np.float64)
    bdist = np.minimum.reduce([pts[:, 0] - bx[box, 0], pts[:, 1] - bx[box, 1], bx[box, 0] + bx[box, 2] - 1 - pts[:, 0],
                               bx[box, 1] + bx[box, 3] - 1 - pts[:, 1]])  # to the box's border, px
    P = [klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[i]) for i in range(3)]
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)
    r01 = lk.calc(P[0], P[1], torch.from_numpy(pts).cuda(), want_iters=True)
    torch.cuda.synchronize()
    ok = r01.status.cpu().numpy() == 1
    it0 = r01.iters.cpu().numpy()
    print(f"fresh corners 0->1: corr(iterations, rank in box) {np.corrcoef(it0, rank)[0, 1]:.3f}, "
          f"corr(iterations, distance to box border) {np.corrcoef(it0, bdist)[0, 1]:.3f}, "
          f"corr(iterations, border distance < 11) {np.corrcoef(it0, bdist < 11)[0, 1]:.3f}; iterations by border "
          f"distance <11 / >=11: {it0[bdist < 11].mean():.2f} / {it0[bdist >= 11].mean():.2f}", flush=True)
    nb0 = int(sys.argv[1]) if len(sys.argv) > 1 else 68
    s0 = box < nb0
    q0, it0s, rk0, bd0 = pts[s0], it0[s0], rank[s0], bdist[s0]
    o0 = {"natural": np.arange(len(q0)), "oracle": np.argsort(-it0s, kind="stable"),
          "border_first": np.lexsort((np.arange(len(q0)), bd0 >= 11)),
          "weak_first_in_box": np.lexsort((-rk0, box[s0]))}
    r0 = {k: [] for k in o0}
    for rnd in range(5):
        for name, o in o0.items():
            d = torch.from_numpy(q0[o]).cuda()
            for _ in range(3):
                lk.calc(P[0], P[1], d)
            torch.cuda.synchronize()
            ctx.timing_select(["lk_sparse"])
            ctx.timing_enable(True)
            for _ in range(20):
                lk.calc(P[0], P[1], d)
            torch.cuda.synchronize()
            cnt, ms = ctx.timing_query("lk_sparse")
            ctx.timing_enable(False)
            r0[name].append(ms / cnt * 1000)
    print(f"fresh corners 0->1, {len(q0)} points: " + "; ".join(f"{k} {np.median(v):.1f} us" for k, v in r0.items()),
          flush=True)
    p1 = r01.next_pts.cpu().numpy()[ok]
    it01 = r01.iters.cpu().numpy()[ok]
    b1 = box[ok]
    r12 = lk.calc(P[1], P[2], torch.from_numpy(p1).cuda(), want_iters=True)
    torch.cuda.synchronize()
    it12 = r12.iters.cpu().numpy()
    ok2 = r12.status.cpu().numpy() == 1
    bm = np.zeros(len(rois))
    for i in range(len(rois)):
        if (b1 == i).any():
            bm[i] = it01[b1 == i].mean()
    print(f"{len(p1)} points tracked 0->1; iterations 0->1 mean {it01.mean():.2f}, 1->2 mean {it12.mean():.2f}; "
          f"corr(point 0->1, point 1->2) {np.corrcoef(it01[ok2], it12[ok2])[0, 1]:.3f}; "
          f"corr(box mean 0->1, point 1->2) {np.corrcoef(bm[b1][ok2], it12[ok2])[0, 1]:.3f}", flush=True)
    sel = b1 < nbox
    q, tq, pq, bq = p1[sel], it12[sel], it01[sel], bm[b1[sel]]
    rng = np.random.default_rng(3)
    orders = {"natural": np.arange(len(q)), "oracle": np.argsort(-tq, kind="stable"),
              "predicted": np.argsort(-pq, kind="stable"), "boxmean": np.argsort(-bq, kind="stable"),
              "shuffled": rng.permutation(len(q))}
    res = {k: [] for k in orders}
    for rnd in range(5):  # interleaved rounds
        for name, o in orders.items():
            d = torch.from_numpy(q[o]).cuda()
            for _ in range(3):
                lk.calc(P[1], P[2], d)
            torch.cuda.synchronize()
            ctx.timing_select(["lk_sparse"])
            ctx.timing_enable(True)
            for _ in range(20):
                lk.calc(P[1], P[2], d)
            torch.cuda.synchronize()
            cnt, ms = ctx.timing_query("lk_sparse")
            ctx.timing_enable(False)
            res[name].append(ms / cnt * 1000)
    lib = os.path.basename(os.environ.get("TBDK_LIB", "libtbdk.so"))
    print(f"{lib}: {len(q)} points ({nbox} boxes), per launch (median of 5 x 20): " +
          "; ".join(f"{k} {np.median(v):.1f} us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
