"""Dense Farneback probe (BASELINE configs[4]: 4K frame pairs): per-kernel HIP-event
times and the HBM roofline of the iteration kernel.  Usage:
    python tools/bench_farneback.py [--width 3840 --height 2160 --pairs 20 --flags 0]
Prints one JSON line."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from opencv_amd import _lib, farneback as F  # noqa: E402
from opencv_amd.klt import Context  # noqa: E402

HBM_PEAK_GBS = 8000.0
# fb_iter algorithmic bytes per output pixel: flow in 8 + R0 20 + R1 20 + flow out 8
FB_ITER_BYTES_PER_PX = 56


def render(ctx, w, h, nobj, nframes, seed=20261015):
    pitch = (w + 255) // 256 * 256
    buf = torch.empty((nframes, h, pitch), dtype=torch.uint8, device="cuda")
    _lib.check(ctx.lib.tbdk_synth_render(ctx.handle, seed, w, h, nobj, 0, nframes, C.c_void_p(buf.data_ptr()),
                                         pitch, None, C.c_void_p(torch.cuda.current_stream().cuda_stream)),
               "tbdk_synth_render")
    return buf[:, :, :w]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--objects", type=int, default=512)
    ap.add_argument("--pairs", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--prep-ahead", type=int, default=1, help="ctx option fb_prep_ahead")
    a = ap.parse_args()
    ctx = Context.get(0)
    ctx.set_option("fb_prep_ahead", a.prep_ahead)
    frames = render(ctx, a.width, a.height, a.objects, a.pairs + 1)
    fb = F.FarnebackOpticalFlow.create(flags=a.flags, ctx=ctx)
    flow = torch.empty((a.height, a.width, 2), dtype=torch.float32, device="cuda")
    for i in range(a.warmup):
        fb.calc(frames[i], frames[i + 1], flow)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.pairs):
        fb.calc(frames[i], frames[i + 1], flow)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ctx.timing_enable(True)
    for i in range(a.pairs):
        fb.calc(frames[i], frames[i + 1], flow)
    torch.cuda.synchronize()
    kern = {}
    for name in ("fb_pyr", "fb_polyexp", "fb_flow_init", "fb_iter"):
        n, ms = ctx.timing_query(name)
        kern[name] = {"launches": n, "total_ms": ms, "avg_us": 1000 * ms / max(n, 1)}
    ctx.timing_enable(False)
    levels = fb.levels(a.width, a.height)
    px_iters = sum(w * h for (w, h) in levels) * fb.getNumIters()
    it_bytes = FB_ITER_BYTES_PER_PX * px_iters * a.pairs
    it_s = kern["fb_iter"]["total_ms"] / 1000
    gbs = it_bytes / it_s / 1e9
    out = {
        "metric": "Farneback frame pairs/sec", "value": a.pairs / wall, "unit": "pairs/s",
        "config": {"width": a.width, "height": a.height, "objects": a.objects, "flags": a.flags,
                   "levels": [list(l) for l in levels], "num_iters": fb.getNumIters(), "win_size": fb.getWinSize()},
        "ms_per_pair": 1000 * wall / a.pairs,
        "kernels_ms_per_pair": {k: v["total_ms"] / a.pairs for k, v in kern.items()},
        "kernels": kern,
        "roofline_fb_iter": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": gbs / HBM_PEAK_GBS, "bytes_per_px": FB_ITER_BYTES_PER_PX},
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
