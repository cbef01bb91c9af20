"""The driver's bench shape (--steps 20 --warmup 5): where does a 20-frame
timed region's time go?  Renders configs[2]'s sequence, warms a fresh loop up
with W per-frame steps, then times tbdk_tbd_run over frames [W, W + K) between
two device syncs (as run_contract), and prints the wall time beside the sum of
the per-frame host step times (the rest is the final drain), the first and
last frames' host times and the per-frame waits.  Regions at frame 5 and at
frame 200 (steady state), a fresh loop each, several repeats."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from opencv_amd import klt, tbd


def main():
    W, H, NOBJ = 1920, 1080, 128
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ctx = klt.Context.get(0)
    frames, gt = klt.synth_render(20261015, W, H, NOBJ, 0, 240, ctx=ctx)
    gtn = gt.numpy()
    dets = [tbd.detections_from_gt(gtn[f]) for f in range(240)]
    cfg = tbd.default_config(W, H, win=21, max_level=2, redetect_every=5)
    s = torch.cuda.current_stream()
    for start in (5, 200, 5, 200, 5, 200):
        loop = tbd.TbdLoop(cfg, ctx=ctx)
        for f in range(start):
            loop.step(frames[f], f, dets[f], s)
        fl = [frames[f] for f in range(start, start + K)]
        packed = tbd.TbdLoop.pack_detections(dets[start:start + K])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ms = loop.run(fl, start, None, s, packed=packed)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        st = np.array([m.host_step_us for m in ms])
        wt = np.array([m.host_wait_us for m in ms])
        print(f"frames [{start}, {start + K}): wall {(t2 - t0) * 1e3:.3f} ms = {(t2 - t0) * 1e6 / K:.1f} us/frame "
              f"({K / (t2 - t0):.0f} fps); run() returned after {(t1 - t0) * 1e3:.3f} ms, drain "
              f"{(t2 - t1) * 1e6:.0f} us; host steps sum {st.sum() / 1e3:.3f} ms, first {st[0]:.0f} / second "
              f"{st[1]:.0f} / median {np.median(st):.0f} us; waits median {np.median(wt):.0f}, first {wt[0]:.0f}",
              flush=True)
        del loop


if __name__ == "__main__":
    main()
