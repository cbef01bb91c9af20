"""Standalone GFTT timing probe: detect_rois over the bench frame's boxes, N
times, for rocprofv3 --kernel-trace --stats (kernels alone on the device)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from opencv_amd import klt  # noqa: E402

n_iter = int(sys.argv[1]) if len(sys.argv) > 1 else 50
nroi = int(sys.argv[2]) if len(sys.argv) > 2 else 128
ctx = klt.Context.get(0)
frames, gt = klt.synth_render(20261015, 1920, 1080, 128, 0, 1, ctx=ctx)
rois = []
for g in gt[0].numpy():
    if not g[0]:
        continue
    x, y, w, h = (int(v) for v in g[1:])
    x0, y0, x1, y1 = max(x, 0), max(y, 0), min(x + w, 1920), min(y + h, 1080)
    if x1 - x0 >= 3 and y1 - y0 >= 3:
        rois.append((x0, y0, x1 - x0, y1 - y0))
rois = rois[:nroi]
det = klt.GoodFeaturesToTrackDetector(256, 0.01, 3.0)
for _ in range(n_iter):
    c, n = det.detect_rois(frames[0], rois)
    torch.cuda.synchronize()
print("rois", len(rois), "px", sum(r[2] * r[3] for r in rois), "max h", max(r[3] for r in rois),
      "counts", n.cpu().numpy()[:10])
