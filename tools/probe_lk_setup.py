"""Level-setup phases of lk_multi by launch size (trace build, TBDK_LIB =
opencv_amd/lib/libtbdk_trace.so): the same 1080p pair and GFTT corners, launches
of 3 points (one wave), one wave per SIMD, and the full set, each run twice
(the second run warm).  Per level: the window rows' arrival, the window terms
and the G sums (the first level split by the trace stamps [14] / [15]), the
Newton phase per step; tells a cold-start or first-level cost from contention."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C

import numpy as np
import torch

import probe_lk_trace as T
from opencv_amd import klt


def main():
    lib = C.CDLL(os.environ["TBDK_LIB"])
    buf = torch.zeros(16 * T.CAP, dtype=torch.int64, device="cuda")
    ctx = klt.Context.get(0)
    W, H = 1920, 1080
    frames, gt = klt.synth_render(20261015, W, H, 128, 0, 2, ctx=ctx)
    rois = []
    for v, x, y, w, h in gt[0].numpy().tolist():
        x0, y0, x1, y1 = max(0, x), max(0, y), min(W, x + w), min(H, y + h)
        if v and x1 - x0 >= 8 and y1 - y0 >= 8:
            rois.append((x0, y0, x1 - x0, y1 - y0))
    c, n = klt.GoodFeaturesToTrackDetector(256, 0.01, 3.0).detect_rois(frames[0], rois)
    c, n = c.cpu().numpy(), n.cpu().numpy()
    pts = np.concatenate([c[i, :n[i]] for i in range(len(rois))]).astype(np.float32)
    P0 = klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[0])
    P1 = klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[1])
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)
    for npts in (3, 3 * 1024, 3 * 4096, len(pts)):
        d = torch.from_numpy(pts[:npts]).cuda()
        for rep in range(2):
            T.arm(lib, buf)
            lk.calc(P0, P1, d)
            torch.cuda.synchronize()
            rec = T.records(lib, buf)
            ph = rec[:, 6:14].copy().view(np.uint32).astype(np.float64) * T.TICK_US
            steps = (rec[:, 5] & 0xFFFF).astype(np.float64)
            m = lambda a, b: np.mean(ph[:, b] - ph[:, a])
            span = (rec[:, 1].max() - rec[:, 0].min()) * T.TICK_US
            print(f"n {npts:6d} rep {rep} waves {len(rec):5d} span {span:6.1f}: pt {np.mean(ph[:, 13]):.2f} | "
                  f"L2 rows {m(8, 14):.2f} terms {m(14, 15):.2f} G {m(15, 9):.2f} newton {m(10, 11):.2f} | "
                  f"L1 setup {m(4, 5):.2f} newton {m(6, 7):.2f} | L0 setup {m(0, 1):.2f} newton {m(2, 3):.2f} | "
                  f"steps/wave {steps.mean():.1f}", flush=True)


if __name__ == "__main__":
    main()
