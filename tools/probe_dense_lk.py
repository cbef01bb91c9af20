"""Dense PyrLK (tbdk_lk_dense, cv::cuda::DensePyrLKOpticalFlow defaults: win 13, 3 levels,
30 iterations) on synthetic frame pairs: pairs/s and pixels/s at two sizes, one JSON line
per size, with the case-image setup (ctx option lk_dense_case 1) and the per-point one (0)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from opencv_amd import klt  # noqa: E402

ctx = klt.Context.get(0)
for mode, (w, h), pairs in ((m, sz, n) for m in (1, 0) for sz, n in (((640, 480), 20), ((1920, 1080), 5))):
    ctx.set_option("lk_dense_case", mode)  # 1: case images (default), 0: per-point setup
    fr, _ = klt.synth_render(20261015, w, h, 24, 0, pairs + 1, device=0, ctx=ctx)
    lk = klt.DensePyrLKOpticalFlow.create()
    flow = lk.calc(fr[0], fr[1])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(pairs):
        flow = lk.calc(fr[i], fr[i + 1], flow)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"lk_dense_case": mode, "size": [w, h], "pairs_per_s": round(pairs / el, 2), "ms_per_pair": round(1000 * el / pairs, 3),
                      "mpix_per_s": round(pairs * w * h / el / 1e6, 1)}), flush=True)
