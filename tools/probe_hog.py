"""A/B of the HOG block kernels: bench.py's HOG measurement (1080p BGRA, 15 levels)
with ctx option hog_block_tiled 1, 0 and 2, one JSON line each."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from opencv_amd import klt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=30)
a = ap.parse_args()
args = argparse.Namespace(hog_width=1920, hog_height=1080, hog_frames=a.frames, seed=20261015, objects=128)
ctx = klt.Context(0)
for tiled in (1, 0, 2, 1):
    ctx.set_option("hog_block_tiled", tiled)
    r = bench.hog_secondary(ctx, args, 0, cpu=False)
    print(json.dumps({"tiled": tiled, "fps": r["value"], "ms": r["ms_per_frame"],
                      "found": r["config"]["detections_first_frames"],
                      "kernels": {k: round(v["ms_per_frame"], 4) for k, v in r["kernels"].items()}}), flush=True)
