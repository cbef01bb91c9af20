"""Floating-point pyramid build timing by ctx option pyr_fuse (>= 1: the
role-split build of klt_pyr_fp.hip, 0: one launch per plane): fp16 levels from
u8 / fp16 frames and fp32 levels from u8 / fp32 frames, 1080p and 4K, HIP events
over 100 builds each; with each build's minimal HBM bytes (frame read once,
every padded level and derivative plane written once, levels 1.. read once)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from opencv_amd import klt

ctx = klt.Context.get(0)
# optional filter, e.g. 3840x2160:float16:uint8 (one configuration, for kernel traces)
only = sys.argv[1] if len(sys.argv) > 1 else None


def min_bytes(P, src_es):
    b = P.width * P.height * src_es
    for i in range(P.nlevels):
        lv, dv = P.pyr.lv[i], P.pyr.dv[i]
        b += lv.pitch * (lv.height + 2 * lv.pad) + dv.width * dv.height * (8 if P.dtype == torch.float32 else 4)
        if i:
            b += lv.width * lv.height * (4 if P.dtype == torch.float32 else 2)
    return b


for (W, H, ml) in ((1920, 1080, 2), (3840, 2160, 2)):
    fr, _ = klt.synth_render(7, W, H, 64, 0, 2, ctx=ctx)
    for store, src in ((torch.float16, torch.uint8), (torch.float16, torch.float16), (torch.float32, torch.uint8),
                       (torch.float32, torch.float32)):
        if only and only != f"{W}x{H}:{str(store)[6:]}:{str(src)[6:]}":
            continue
        frames = [f.to(src) for f in fr]
        P = klt.Pyramid(ctx, W, H, ml, (21, 21), store)
        res = {(1, 1): [], (1, 0): [], (0, 1): []}
        for rnd in range(6):  # variants interleaved; round 0 warms up
            for fuse, xcd in res:
                ctx.set_option("pyr_fuse", fuse)
                ctx.set_option("pyr_xcd", xcd)
                n = 20 if rnd == 0 else 100
                ctx.timing_select(["pyr_build"])
                ctx.timing_enable(True)
                for i in range(n):
                    P.build(frames[i & 1])
                torch.cuda.synchronize()
                c, ms = ctx.timing_query("pyr_build")
                ctx.timing_enable(False)
                ctx.timing_select(None)
                if rnd:
                    res[fuse, xcd].append(ms / c * 1000)
        ctx.set_option("pyr_fuse", 1)
        ctx.set_option("pyr_xcd", 1)
        mb = min_bytes(P, frames[0].element_size())
        med = {k: statistics.median(v) for k, v in res.items()}
        print(f"{W}x{H} {str(store)[6:]} levels from {str(src)[6:]} ({mb / 1e6:.1f} MB): role-split "
              f"{med[1, 1]:.1f} us ({mb / med[1, 1] / 1e3:.0f} GB/s), without XCD bands {med[1, 0]:.1f}, "
              f"per plane {med[0, 1]:.1f} us", flush=True)
