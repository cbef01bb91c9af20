"""Why is the first TBD loop of a process slower than later ones?  One fresh
process per call: render configs[2]'s sequence, then (mode)
  cold  : nothing
  gpu   : keep the GPU busy for ~60 ms first (a chain of large copies)
  host  : keep the host thread busy for ~60 ms first (a Python spin)
  loop  : run a throw-away loop over frames [0, 5) first
  sleep : sleep 60 ms first
then a fresh loop: 5 warm-up steps and frames [5, 25) through tbdk_tbd_run
between two device syncs (the driver's bench shape), three such loops in a
row.  Prints the regions' frames/s."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from opencv_amd import klt, tbd


def region(ctx, cfg, frames, dets, s, W=5, K=20):
    loop = tbd.TbdLoop(cfg, ctx=ctx)
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
    frames, gt = klt.synth_render(20261015, 1920, 1080, 128, 0, 30, ctx=ctx)
    gtn = gt.numpy()
    dets = [tbd.detections_from_gt(gtn[f]) for f in range(30)]
    cfg = tbd.default_config(1920, 1080, win=21, max_level=2, redetect_every=5)
    s = torch.cuda.current_stream()
    torch.cuda.synchronize()
    if mode == "gpu":
        a = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.06:
            for _ in range(8):
                b.copy_(a)
            torch.cuda.synchronize()
        del a, b
    elif mode == "host":
        t0 = time.perf_counter()
        x = 0
        while time.perf_counter() - t0 < 0.06:
            x += 1
    elif mode == "loop":
        loop = tbd.TbdLoop(cfg, ctx=ctx)
        for f in range(5):
            loop.step(frames[f], f, dets[f], s)
        torch.cuda.synchronize()
        del loop
    elif mode == "sleep":
        time.sleep(0.06)
    r = [region(ctx, cfg, frames, dets, s) for _ in range(3)]
    print(f"{mode:6s} " + " ".join(f"{v:7.0f}" for v in r), flush=True)


if __name__ == "__main__":
    main()
