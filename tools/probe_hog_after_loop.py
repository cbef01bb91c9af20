"""HOG frames/s (bench.py's measurement, level lanes on) on a fresh context, with a
TBD loop object alive on the same context, and after that object is deleted."""
import argparse
import gc
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from opencv_amd import klt, tbd  # noqa: E402

args = argparse.Namespace(hog_width=1920, hog_height=1080, hog_frames=30, seed=20261015, objects=128)
if os.environ.get("SET_DEVICE"):
    torch.cuda.set_device(0)
ctx = klt.Context.get(0)


def hog(tag):
    r = bench.hog_secondary(ctx, args, 0, cpu=False)
    print(json.dumps({"case": tag, "fps": r["value"],
                      "kernels": {k: round(v["ms_per_frame"], 4) for k, v in r["kernels"].items()}}), flush=True)


if not os.environ.get("SKIP_FRESH"):
    hog("fresh")
frames, gt = klt.synth_render(args.seed, 1920, 1080, 128, 0, 6, device=0, ctx=ctx)
dets = [tbd.detections_from_gt(gt.numpy()[f]) for f in range(6)]
loop = tbd.TbdLoop(tbd.default_config(1920, 1080, win=21, max_level=2, redetect_every=5), ctx=ctx)
hog("loop created")
s = torch.cuda.current_stream()
for f in range(6):
    loop.step(frames[f], f, dets[f], s)
torch.cuda.synchronize()
hog("loop stepped")
loops = [tbd.TbdLoop(tbd.default_config(1920, 1080, win=21, max_level=2, redetect_every=5), ctx=ctx)
         for _ in range(int(os.environ.get("EXTRA_LOOPS", "2")))]
hog("extra loops created")
del loop, loops
gc.collect()
hog("loops deleted")
