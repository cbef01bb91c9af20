"""A/B of the HOG block kernels: bench.py's HOG measurement (1080p BGRA, 15 levels)
under ctx options hog_block_tiled / hog_level_streams / hog_window_tiled, one JSON
line each."""
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
for tiled, lanes, wt in ((1, 3, 1), (1, 3, 0), (1, 1, 1), (1, 1, 0), (1, 3, 1)):
    ctx.set_option("hog_block_tiled", tiled)
    ctx.set_option("hog_level_streams", lanes)
    ctx.set_option("hog_window_tiled", wt)
    r = bench.hog_secondary(ctx, args, 0, cpu=False)
    print(json.dumps({"tiled": tiled, "lanes": lanes, "win_tiled": wt, "fps": r["value"], "ms": r["ms_per_frame"],
                      "found": r["config"]["detections_first_frames"],
                      "kernels": {k: round(v["ms_per_frame"], 4) for k, v in r["kernels"].items()}}), flush=True)
