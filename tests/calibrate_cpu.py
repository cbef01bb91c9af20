"""BASELINE.md §3 calibration: the oracle restatement of the reference's CPU
PyrLK timed on the input shape BASELINE.md §2 measured the real reference on
(1080p synthetic blurred-noise frame, global (2.5, -1.75) px shift, win 21,
maxLevel 3, 128 boxes x 256 points), 1 and 8 threads, in the SSE2 accumulation
order, so the bench's cpu_baseline (a "port") can be read against the
reference itself: ratio = restatement time / reference time on that input.

  TBDK_ORACLE_LIB=<-O3 -march=native build> python tests/calibrate_cpu.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import _oracle as O  # noqa: E402

REF = {  # BASELINE.md §2, the real reference (OpenCV 3.4.7, WITH_IPP=OFF) in the survey container
    "lk_1080p_128x256_1t_ms": 333.6, "lk_1080p_128x256_8t_ms": 54.0,
    "lk_1080p_64x256_1t_ms": 159.9, "lk_1080p_64x256_8t_ms": 26.9,
}


def blurred_noise(w, h, seed=1):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (h, w)).astype(np.float32)
    k = np.array([1, 4, 6, 4, 1], np.float32) / 16
    for _ in range(2):  # separable [1 4 6 4 1]^2 blur, twice
        img = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 1, img)
        img = np.apply_along_axis(lambda c: np.convolve(c, k, "same"), 0, img)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def main():
    W, H = 1920, 1080
    a = blurred_noise(W, H)
    M = np.array([[1.0, 0.0, 2.5], [0.0, 1.0, -1.75]])
    b = O.warp_affine(a, M, (W, H), O.INTER_LINEAR, O.BORDER_REFLECT_101)
    rng = np.random.default_rng(2)
    out = {}
    for nbox in (64, 128):
        boxes = [(rng.uniform(40, W - 240), rng.uniform(40, H - 240), rng.uniform(64, 200), rng.uniform(64, 200))
                 for _ in range(nbox)]
        pts = np.concatenate([np.stack([rng.uniform(x, x + bw, 256), rng.uniform(y, y + bh, 256)], 1)
                              for x, y, bw, bh in boxes]).astype(np.float32)
        P0, P1 = O.Pyramid(a, (21, 21), 3), O.Pyramid(b, (21, 21), 3)
        for th in (1, 8):
            O.lk(P0, P1, pts[:2048], max_level=3, accum=O.ACCUM_SSE2, nthreads=th, want_err=False)
            best = 1e9
            for _ in range(3 if th > 1 else 1):
                t = time.perf_counter()
                nx, st, _, it = O.lk(P0, P1, pts, max_level=3, accum=O.ACCUM_SSE2, nthreads=th, want_err=False)
                best = min(best, time.perf_counter() - t)
            key = f"lk_1080p_{nbox}x256_{th}t_ms"
            out[key] = {"restatement_ms": round(best * 1e3, 1), "reference_ms": REF[key],
                        "ratio": round(best * 1e3 / REF[key], 3), "points": len(pts),
                        "mean_iters": round(float(it.mean()), 2), "tracked": round(float(st.mean()), 4)}
            print(key, out[key], flush=True)
    res = {"input": "1920x1080 blurred noise ([1 4 6 4 1]^2 twice), next = warpAffine translate (2.5, -1.75), "
                    "win 21, maxLevel 3, boxes 64-200 px x 256 uniform points, SSE2 order",
           "oracle_lib": os.environ.get("TBDK_ORACLE_LIB", "oracle/liboracle.so (-O2)"),
           "host": os.uname().machine + f", {os.cpu_count()} CPUs", "results": out,
           "note": "reference_ms from BASELINE.md §2 (the survey container, same 8-CPU VM type, inputs of "
                   "the same shape generated there, not these exact pixels); ratio > 1: the restatement is slower"}
    print(json.dumps(res, indent=1))
    return res


if __name__ == "__main__":
    r = main()
    if len(sys.argv) > 1:
        json.dump(r, open(sys.argv[1], "w"), indent=1)
