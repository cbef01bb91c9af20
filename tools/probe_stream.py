"""Which stream should the caller hand the TBD loop?  One fresh process per
call: render configs[2]'s sequence, then run loops on
  null   : torch's default stream (the HIP null stream; bench.py's choice)
  before : a torch side stream (non-blocking) created before the first loop
  after  : a torch side stream created after the first loop was created
W = 20 warm-up steps, frames [W, W + K) through tbdk_tbd_run between two device
syncs, K = 480 and K = 20 (the driver's shape, W = 5), three fresh loops
each.  Prints frames/s."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from opencv_amd import klt, tbd


def region(loop, frames, dets, s, W, K):
    for f in range(W):
        loop.step(frames[f], f, dets[f], s)
    fl = [frames[f] for f in range(W, W + K)]
    packed = tbd.TbdLoop.pack_detections(dets[W:W + K])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop.run(fl, W, None, s, packed=packed)
    torch.cuda.synchronize()
    return K / (time.perf_counter() - t0)


def main():
    mode = sys.argv[1]
    ctx = klt.Context.get(0)
    n = 500
    frames, gt = klt.synth_render(20261015, 1920, 1080, 128, 0, n, ctx=ctx)
    gtn = gt.numpy()
    dets = [tbd.detections_from_gt(gtn[f]) for f in range(n)]
    cfg = tbd.default_config(1920, 1080, win=21, max_level=2, redetect_every=5)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    if mode == "before":
        s = torch.cuda.Stream()
    out = []
    for W, K in ((20, 480), (5, 20), (20, 480), (5, 20)):
        loop = tbd.TbdLoop(cfg, ctx=ctx)
        if mode == "after" and s is torch.cuda.current_stream():
            s = torch.cuda.Stream()
        out.append(region(loop, frames, dets, s, W, K))
        del loop
    print(f"{mode:6s} " + " ".join(f"{v:7.0f}" for v in out), flush=True)


if __name__ == "__main__":
    main()
