import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from opencv_amd import klt
ctx = klt.Context.get(0)
frames, gt = klt.synth_render(20261015, 1920, 1080, 128, 0, 1, ctx=ctx)
rois = [tuple(int(v) for v in g[1:]) for g in gt[0].numpy() if g[0]]
det = klt.GoodFeaturesToTrackDetector(256, 0.01, 3.0)
for _ in range(3):
    c, n = det.detect_rois(frames[0], rois)
torch.cuda.synchronize()
print("counts", n.cpu().numpy()[:20])
