"""Host time of the TBD loop's step by phase (probe build with
-DTBDK_STEP_PROFILE: TBDK_LIB=opencv_amd/lib/libtbdk_sprof.so).  configs[2]'s
1080p x 128-object sequence, 20 warm-up steps, then frames [20, 500) through
tbdk_tbd_run as bench.py's timed region; prints the mean us per frame of each
segment between the step's marks (tbd_loop.hip STEP_MARK)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from opencv_amd import klt, tbd  # noqa: E402

NAMES = ["step start -> early GFTT launched", "-> slot lists, unchanged-set PyrLK", "-> refreshed-set PyrLK launched",
         "-> fit + next pyramid launched (wait starts)", "wait for the fit", "-> fit results, predictions",
         "-> speculative / early-row PyrLK launched", "tracker step", "-> deletions, refreshed ROIs",
         "-> post-tracker GFTT launched", "-> look-ahead PyrLK launched, end"]


def main():
    W, H, N = 1920, 1080, 128
    ctx = klt.Context.get(0)
    frames, gt = klt.synth_render(20261015, W, H, N, 0, 500, ctx=ctx)
    gtn = gt.numpy()
    dets = [tbd.detections_from_gt(gtn[f]) for f in range(500)]
    cfg = tbd.default_config(W, H)
    s = torch.cuda.current_stream()
    out = (C.c_double * 18)()
    for rep in range(3):
        loop = tbd.TbdLoop(cfg, ctx=ctx)
        for f in range(20):
            loop.step(frames[f], f, dets[f], s)
        ctx.lib.tbdk_probe_step_profile(out, 18)  # drop the warm-up
        packed = tbd.TbdLoop.pack_detections(dets[20:500])
        torch.cuda.synchronize()
        loop.run([frames[f] for f in range(20, 500)], 20, None, s, packed=packed)
        torch.cuda.synchronize()
        assert ctx.lib.tbdk_probe_step_profile(out, 18) == 0
        tot = sum(out[1:12])
        print(f"run {rep}: {int(out[0])} steps, {tot:.1f} us per step")
        for i, n in enumerate(NAMES, 1):
            print(f"   {n:48s} {out[i]:7.1f}")
        print(f"   speculative block ({int(out[12])} runs): list {out[13]:.1f}, wait edge {out[14]:.1f}, "
              f"lk_internal {out[15]:.1f}, la_done record {out[16]:.1f}, membership {out[17]:.1f} us")
        del loop


if __name__ == "__main__":
    main()
