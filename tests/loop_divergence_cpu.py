"""CPU-only: the TBD loop in the GPU's exact-sum PyrLK order against the same
loop in the reference's SSE2 order, over a whole configs[2]-shaped sequence
(tests/_loop_compare.py says what is measured).  The GPU is bit-exact with the
exact-order oracle (tests/test_gpu_tbd_e2e.py), so these figures are the
GPU-vs-reference-order divergence.

  python tests/loop_divergence_cpu.py [--frames 500] [--threads 8] [--seed 20261015] [--out f.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import tbd_loop_oracle as L  # noqa: E402
import _loop_compare as LC  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    W, H, N, F = a.width, a.height, a.objects, a.frames
    t0 = time.time()
    frames, gt = L.O.synth(a.seed, W, H, N, 0, F)
    ex = L.KltTbdLoop(W, H, accum=L.O.ACCUM_EXACT, shadow_accum=L.O.ACCUM_SSE2, nthreads=a.threads)
    ss = L.KltTbdLoop(W, H, accum=L.O.ACCUM_SSE2, nthreads=a.threads)
    cs, ls = LC.CallStats(), LC.LoopStats()
    for f in range(F):
        d = L.detections(gt[f], f)
        ma = ex.step(frames[f], f, d)
        cs.add(ex.shadow)
        mb = ss.step(frames[f], f, d)
        ls.add(f, ma, mb, ex.track_rows(), ss.track_rows())
        if f % 50 == 49:
            print(f"frame {f + 1}/{F} {time.time() - t0:.0f}s", cs.summary()["status_disagree"],
                  ls.summary()["first_pred_diff_frame"], flush=True)
    out = dict(config=dict(width=W, height=H, objects=N, frames=F, seed=a.seed), per_call=cs.summary(),
               per_loop=ls.summary(), seconds=round(time.time() - t0, 1))
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
