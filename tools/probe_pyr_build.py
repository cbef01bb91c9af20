#!/usr/bin/env python3
"""Event-timed u8 levels-only pyramid builds (padded and borrowed level 0) at
4K and 1080p for the library in TBDK_LIB (A/B of pyramid kernel variants):
prints one JSON line of mean microseconds per build."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from opencv_amd import klt  # noqa: E402


def timed(ctx, fn, n):
    for i in range(10):
        fn(i)
    torch.cuda.synchronize()
    ctx.timing_select(["pyr_build"])
    ctx.timing_enable(True)
    for i in range(n):
        fn(i)
    torch.cuda.synchronize()
    c, ms = ctx.timing_query("pyr_build")
    ctx.timing_enable(False)
    ctx.timing_select(None)
    return round(ms / c * 1000.0, 2)


def main(n=200):
    ctx = klt.Context()
    out = {}
    for W, H in ((3840, 2160), (1920, 1080)):
        fr, _ = klt.synth_render(7, W, H, 64, 0, 2, ctx=ctx)
        P = klt.Pyramid(ctx, W, H, 2, (21, 21), derivs=False)
        out[f"{W}x{H}_padded"] = timed(ctx, lambda i: P.build(fr[i & 1]), n)
        out[f"{W}x{H}_borrowed"] = timed(ctx, lambda i: P.build_borrowed(fr[i & 1]), n)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
