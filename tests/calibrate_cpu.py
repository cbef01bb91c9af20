"""BASELINE.md §3 calibration: the oracle restatement of the reference's CPU
PyrLK timed on the input shape BASELINE.md §2 measured the real reference on
(1080p synthetic blurred-noise frame, global (2.5, -1.75) px shift, win 21,
maxLevel 3, 128 boxes x 256 points), 1 and 8 threads, in the SSE2 accumulation
order, so the bench's cpu_baseline (a "port") can be read against the
reference itself: ratio = restatement time / reference time on that input.

The reference's input iterated "2-3 times per level on smooth motion"
(8-12 Newton steps per point over the 4 levels of maxLevel 3).
The blur strength is chosen here so the restatement's mean lands in that range
(the first round's [1 4 6 4 1]^2 x2 input iterated ~19.6 times per point, which
confounds iteration count with per-iteration speed); both inputs are reported,
each with its mean iterations and the ratio per Newton iteration as well as
per call.

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


REF_ITERS = (8.0, 12.0)  # 2-3 per level x 4 levels


def blurred_noise(w, h, seed=1, passes=2):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (h, w)).astype(np.float32)
    k = np.array([1, 4, 6, 4, 1], np.float32) / 16
    for _ in range(passes):  # separable [1 4 6 4 1]^2 blur, `passes` times
        img = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 1, img)
        img = np.apply_along_axis(lambda c: np.convolve(c, k, "same"), 0, img)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def frame_pair(passes):
    W, H = 1920, 1080
    a = blurred_noise(W, H, passes=passes)
    M = np.array([[1.0, 0.0, 2.5], [0.0, 1.0, -1.75]])
    return a, O.warp_affine(a, M, (W, H), O.INTER_LINEAR, O.BORDER_REFLECT_101)


def box_points(nbox, seed=2):
    W, H = 1920, 1080
    rng = np.random.default_rng(seed)
    boxes = [(rng.uniform(40, W - 240), rng.uniform(40, H - 240), rng.uniform(64, 200), rng.uniform(64, 200))
             for _ in range(nbox)]
    return np.concatenate([np.stack([rng.uniform(x, x + bw, 256), rng.uniform(y, y + bh, 256)], 1)
                           for x, y, bw, bh in boxes]).astype(np.float32)


def time_input(a, b):
    out = {}
    P0, P1 = O.Pyramid(a, (21, 21), 3), O.Pyramid(b, (21, 21), 3)
    for nbox in (64, 128):
        pts = box_points(nbox)
        for th in (1, 8):
            O.lk(P0, P1, pts[:2048], max_level=3, accum=O.ACCUM_SSE2, nthreads=th, want_err=False)
            best = 1e9
            for _ in range(3 if th > 1 else 2):
                t = time.perf_counter()
                nx, st, _, it = O.lk(P0, P1, pts, max_level=3, accum=O.ACCUM_SSE2, nthreads=th, want_err=False)
                best = min(best, time.perf_counter() - t)
            key = f"lk_1080p_{nbox}x256_{th}t_ms"
            k = float(it.mean())
            kt = float(it[st == 1].mean())
            ref = REF[key]
            # per Newton iteration: call time / (points x mean iterations), the
            # reference's at both ends of its stated 8-12 iterations per point
            per_it = best * 1e3 / (len(pts) * k)
            ref_per_it = [ref / (len(pts) * ki) for ki in REF_ITERS]
            out[key] = {"restatement_ms": round(best * 1e3, 1), "reference_ms": ref,
                        "ratio": round(best * 1e3 / ref, 3), "points": len(pts),
                        "mean_iters": round(k, 2), "mean_iters_tracked": round(kt, 2),
                        "reference_mean_iters": list(REF_ITERS),
                        "ratio_per_iteration": [round(per_it / r, 3) for r in ref_per_it[::-1]],
                        "tracked": round(float(st.mean()), 4)}
            print(key, out[key], flush=True)
    return out


def main():
    # the blur whose mean iteration count lands in the reference's 8-12
    probe = box_points(16)
    sweep = {}
    for passes in (2, 8, 16, 24, 32):
        a, b = frame_pair(passes)
        _, st, _, it = O.lk(O.Pyramid(a, (21, 21), 3), O.Pyramid(b, (21, 21), 3), probe, max_level=3,
                            accum=O.ACCUM_SSE2, nthreads=8, want_err=False)
        sweep[passes] = {"mean_iters": round(float(it.mean()), 2), "tracked": round(float(st.mean()), 4)}
        print("blur passes", passes, sweep[passes], flush=True)
    # the reference's input tracked its points (32,486 of 32,768
    # points kept by its box generator, all tracked); among blurs that keep >= 99 %
    # tracked, the one with the fewest iterations
    mid = sum(REF_ITERS) / 2
    ok = [p for p in sweep if sweep[p]["tracked"] >= 0.99] or [2]
    matched = min(ok, key=lambda p: abs(sweep[p]["mean_iters"] - mid))
    res = {"inputs": {}, "blur_sweep_mean_iters": sweep,
           "oracle_lib": os.environ.get("TBDK_ORACLE_LIB", "oracle/liboracle.so (-O2)"),
           "host": os.uname().machine + f", {os.cpu_count()} CPUs",
           "note": "matched_iterations: the blur (of those keeping >= 99 % of the points tracked) whose mean "
                   "iteration count is closest to the reference's 2-3 per level; noise blurred further loses "
                   "texture and the minEig gate drops points. "
                   "reference_ms from BASELINE.md §2 (the survey container, same 8-CPU VM type, inputs of "
                   "the same shape generated there, not these exact pixels; its iteration count is stated as "
                   "2-3 per level, 8-12 per point over 4 levels); ratio > 1: the restatement is slower; "
                   "ratio_per_iteration = (restatement ms per point-iteration) / (reference ms per "
                   "point-iteration at 12 and at 8 iterations per point)"}
    for name, passes in (("matched_iterations", matched), ("round4_input", 2)):
        a, b = frame_pair(passes)
        res["inputs"][name] = {
            "input": f"1920x1080 blurred noise ([1 4 6 4 1]^2 x{passes}), next = warpAffine translate (2.5, "
                     "-1.75), win 21, maxLevel 3, boxes 64-200 px x 256 uniform points, SSE2 order",
            "results": time_input(a, b)}
    print(json.dumps(res, indent=1))
    return res


if __name__ == "__main__":
    r = main()
    if len(sys.argv) > 1:
        json.dump(r, open(sys.argv[1], "w"), indent=1)
