"""Per-frame work and host times of the bench's loop (bench.py defaults): one
run of frames [5, 285) after 5 warm-up frames; prints frames [5, 25) (the
driver's timed region) one by one and the means over [5, 25), [25, 125) and
[125, 285): PyrLK points and iterations, GFTT refreshes, tracks, and the
host's launch / wait / tracker / step times per frame."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import bench
from opencv_amd import klt, tbd

F = ["ntracks", "lk_points", "klt_points", "lk_iters", "redetected", "early_gftt", "host_launch_us", "host_wait_us",
     "host_tracker_us", "host_step_us"]


def main():
    args = types.SimpleNamespace(sequence_frames=500, warmup=5, steps=20, width=1920, height=1080, objects=128,
                                 seed=20261015, win=21, max_level=2, redetect=5, bounds="reference")
    dev = torch.cuda.current_device()
    ctx = klt.Context.get(dev)
    ctx.set_option("tbd_early_gftt", 2)
    ctx.set_option("tbd_spec_lookahead", 1)
    ctx.set_option("tbd_zero_copy", 1)
    for kv in os.environ.get("PROBE_CTX", "").split():
        name, _, val = kv.partition("=")
        ctx.set_option(name, int(val))
    m = bench.TbdMeasure(args, ctx, dev)
    m.prepare(args.seed)
    for rep in range(2):
        loop = m.new_loop(5)
        fl = [m.frames[f] for f in range(5, 285)]
        ms = loop.run(fl, 5, None, m.stream, packed=tbd.TbdLoop.pack_detections(m.dets[5:285]))
        torch.cuda.synchronize()
        a = np.array([[float(getattr(x, k)) for k in F] for x in ms])
        if rep == 1:
            print("frame " + " ".join(f"{k[:12]:>12s}" for k in F))
            for i in range(20):
                print(f"{5 + i:5d} " + " ".join(f"{v:12.1f}" for v in a[i]))
        for lo, hi in ((5, 25), (25, 125), (125, 285)):
            s = a[lo - 5:hi - 5].mean(axis=0)
            print(f"rep {rep} mean [{lo},{hi}) " + " ".join(f"{k}={v:.1f}" for k, v in zip(F, s)), flush=True)


if __name__ == "__main__":
    main()
