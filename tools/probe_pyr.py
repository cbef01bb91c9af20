"""tbdk_pyr_build timing by ctx options pyr_fuse (2: levels 0-2 in one tiled
launch, 1: the two-role launch + one per level, 0: one launch per level) and
pyr_rows (rows per thread of the two-role launch) and pyr_xcd (row bands per
XCD), levels-only and with
derivative planes, 1080p / KITTI / 4K.  HIP events over 100 builds per
variant, the variants interleaved over 5 rounds; per variant the median and
min of the rounds' means."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from opencv_amd import klt

ctx = klt.Context.get(0)
only = sys.argv[1:]  # optional variant names (a library without pyr_rows / pyr_xcd: "two-role r4" etc. still run)


def opt(name, v):
    try:
        ctx.set_option(name, v)
    except Exception:  # option unknown to this library build
        pass


VARIANTS = [("tiled", False, 2, 4, 1), ("two-role r4", False, 1, 4, 1), ("two-role r4 noxcd", False, 1, 4, 0),
            ("two-role r2", False, 1, 2, 1), ("two-role r1", False, 1, 1, 1), ("two-role r1 noxcd", False, 1, 1, 0),
            ("per level", False, 0, 4, 1), ("planes two-role r4", True, 1, 4, 1)]


def timed(P, frames, n=100):
    ctx.timing_select(["pyr_build"])
    ctx.timing_enable(True)
    for i in range(n):
        P.build(frames[i & 1])
    torch.cuda.synchronize()
    c, ms = ctx.timing_query("pyr_build")
    ctx.timing_enable(False)
    ctx.timing_select(None)
    return ms / c * 1000


for (W, H, ml) in ((1920, 1080, 2), (1242, 375, 2), (3840, 2160, 2)):
    fr, _ = klt.synth_render(7, W, H, 64, 0, 2, ctx=ctx)
    pyrs = {v[0]: klt.Pyramid(ctx, W, H, ml, (21, 21), derivs=v[1]) for v in VARIANTS if not only or v[0] in only}
    res = {v[0]: [] for v in VARIANTS}
    for rnd in range(6):
        for name, derivs, fuse, rows, xcd in VARIANTS:
            if only and name not in only:
                continue
            opt("pyr_fuse", fuse)
            opt("pyr_rows", rows)
            opt("pyr_xcd", xcd)
            t = timed(pyrs[name], fr, 20 if rnd == 0 else 100)
            if rnd:
                res[name].append(t)
    opt("pyr_fuse", 1)
    opt("pyr_rows", 1)
    opt("pyr_xcd", 1)
    print(f"{W}x{H} maxLevel {ml}: " + ", ".join(f"{k} {statistics.median(v):.1f} (min {min(v):.1f})"
                                                 for k, v in res.items() if v) + " us", flush=True)
