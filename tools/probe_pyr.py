"""tbdk_pyr_build timing by ctx option pyr_fuse (2: levels 0-2 in one tiled
launch, 1: the two-role launch + one per level, 0: one launch per level),
levels-only and with derivative planes (+ the Scharr launch), 1080p / KITTI /
4K, HIP events over 200 builds each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from opencv_amd import klt

ctx = klt.Context.get(0)
for (W, H, ml) in ((1920, 1080, 2), (1242, 375, 2), (3840, 2160, 2), (1920, 1080, 3)):
    fr, _ = klt.synth_render(7, W, H, 64, 0, 2, ctx=ctx)
    out = []
    for derivs, fuse, rows in ((False, 2, 4), (False, 1, 4), (False, 0, 4), (True, 2, 4), (True, 1, 4), (False, 1, 1),
                               (False, 1, 2)):
        ctx.set_option("pyr_fuse", fuse)
        ctx.set_option("pyr_rows", rows)
        P = klt.Pyramid(ctx, W, H, ml, (21, 21), derivs=derivs)
        for _ in range(20):
            P.build(fr[0])
        torch.cuda.synchronize()
        ctx.timing_select(["pyr_build"])
        ctx.timing_enable(True)
        for i in range(200):
            P.build(fr[i & 1])
        torch.cuda.synchronize()
        c, ms = ctx.timing_query("pyr_build")
        ctx.timing_enable(False)
        ctx.timing_select(None)
        out.append(ms / c * 1000)
    ctx.set_option("pyr_fuse", 1)
    ctx.set_option("pyr_rows", 4)
    print(f"{W}x{H} maxLevel {ml}: levels only: tiled {out[0]:6.1f} us, two-role {out[1]:6.1f} us (4 rows/thread; "
          f"1: {out[5]:6.1f}, 2: {out[6]:6.1f}), per level {out[2]:6.1f} us; with Scharr planes: tiled "
          f"{out[3]:6.1f} us, two-role {out[4]:6.1f} us", flush=True)
