"""Where the driver's short timed region loses to the long one: tbdk_tbd_run over
K frames after a warm-up of 5 frames, as bench.py's defaults configure the
loop.  PROBE_WARM=step|run picks how the warm-up frames go through the loop
(tbdk_tbd_step per frame, bench.py's warm-up until round 6, or one
tbdk_tbd_run); the process's first measurement is the driver's situation
(nothing run through tbdk_tbd_run before).  Then per fresh loop: the first
run() of 20 frames, the next 20 on the same loop, runs of 80 and 160, and a
loop warmed over 25 frames running [25, 45) (content vs first-call effects);
host return time (no sync) beside the synced time; the Python wrapper's own
cost; idle gaps before the region."""
import os
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench
from opencv_amd import klt, tbd


def main():
    args = types.SimpleNamespace(sequence_frames=500, warmup=5, steps=20, width=1920, height=1080, objects=128,
                                 seed=20261015, win=21, max_level=2, redetect=5, bounds="reference")
    dev = torch.cuda.current_device()
    ctx = klt.Context.get(dev)
    ctx.set_option("tbd_early_gftt", 2)
    ctx.set_option("tbd_spec_lookahead", 1)
    ctx.set_option("tbd_zero_copy", 1)
    ctx.set_option("tbd_pyr_derivs", 0)
    for kv in os.environ.get("PROBE_CTX", "").split():
        name, _, val = kv.partition("=")
        ctx.set_option(name, int(val))
    warm = os.environ.get("PROBE_WARM", "step")
    m = bench.TbdMeasure(args, ctx, dev)
    m.prepare(args.seed)
    packs = {}

    def pack(f0, k):
        if (f0, k) not in packs:
            packs[(f0, k)] = tbd.TbdLoop.pack_detections(m.dets[f0:f0 + k])
        return packs[(f0, k)]

    def fresh(w):
        if warm == "step":
            return m.new_loop(w)
        loop = tbd.TbdLoop(m.cfg, ctx=ctx)
        loop.run([m.frames[f] for f in range(w)], 0, None, m.stream, packed=pack(0, w))
        return loop

    def timed(loop, f0, k):
        fl = [m.frames[f] for f in range(f0, f0 + k)]
        p = pack(f0, k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.run(fl, f0, None, m.stream, packed=p)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return f"[{f0},{f0 + k}) {k / (t2 - t0):6.0f} fps host {1e3 * (t1 - t0):.3f}/{1e3 * (t2 - t0):.3f} ms"

    pack(5, 20)
    pack(0, 5)
    loop = fresh(5)
    print(f"warm={warm} first in process: " + timed(loop, 5, 20), flush=True)
    for rep in range(4):
        loop = fresh(5)
        out = [timed(loop, 5, 20), timed(loop, 25, 20), timed(loop, 45, 80), timed(loop, 125, 160)]
        pack(0, 25)
        loop = fresh(25)
        out.append("w25 " + timed(loop, 25, 20))
        print(f"rep {rep}: " + " | ".join(out), flush=True)
    fl = [m.frames[f] for f in range(5, 25)]
    t0 = time.perf_counter()
    for _ in range(100):
        for f in fl:
            tbd.TbdLoop._check_frame(f)
        [f.data_ptr() for f in fl]
    print(f"wrapper checks + pointers for 20 frames: {1e6 * (time.perf_counter() - t0) / 100:.1f} us", flush=True)
    for idle in (0.0, 0.01, 0.05, 0.5):
        loop = fresh(5)
        torch.cuda.synchronize()
        time.sleep(idle)
        print(f"idle {idle:.2f}s then " + timed(loop, 5, 20), flush=True)


if __name__ == "__main__":
    main()
