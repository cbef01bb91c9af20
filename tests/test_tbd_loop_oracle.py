"""CPU checks of the loop oracle (oracle/tbd_loop_oracle.py) that
tests/test_gpu_tbd_e2e.py compares the native loop against: on a synthetic
sequence with known motion it tracks the objects, its KLT predictions land
near the ground-truth centres, and its slot / refresh bookkeeping follows the
stated rules."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tbd_loop_oracle as L  # noqa: E402


def test_loop_oracle_tracks_synthetic_objects():
    W, H, N, F = 640, 480, 12, 11
    fr, gt = L.O.synth(7, W, H, N, 0, F)
    lp = L.KltTbdLoop(W, H, bounds=(0, W, 0, H), nthreads=4)
    preds = 0
    for f in range(F):
        m = lp.step(fr[f], f, L.detections(gt[f], f))
        assert m["gt"] == int(gt[f][:, 0].sum())
        if f == 0:
            assert m["redetected"] == m["ntracks"] and m["lk_points"] == 0
        elif f % 5 == 0:
            assert m["redetected"] == m["ntracks"]  # re-detection frame: every set refreshed
        else:
            assert m["lk_points"] >= m["klt_points"] > 0
        # predictions near the truth: some object's GT centre in this frame
        g = gt[f][gt[f][:, 0] != 0]
        centres = np.stack([g[:, 1] + g[:, 3] / 2, g[:, 2] + g[:, 4] / 2], 1)
        for cx, cy in lp.preds.values():
            assert np.min(np.hypot(centres[:, 0] - cx, centres[:, 1] - cy)) < 4.0
        preds += len(lp.preds)
        if f >= 2:
            assert m["tp"] >= 0.9 * m["gt"]
    assert preds > (F - 1) * N // 2


def test_loop_oracle_slot_pool_exhaustion():
    """With fewer slots than tracks the extra tracks own no point set (constant-velocity model)."""
    W, H, N, F = 640, 480, 10, 4
    fr, gt = L.O.synth(3, W, H, N, 0, F)
    lp = L.KltTbdLoop(W, H, bounds=(0, W, 0, H), max_tracks=4, nthreads=2)
    for f in range(F):
        m = lp.step(fr[f], f, L.detections(gt[f], f))
        assert len(lp.slot) <= 4
        if f:
            assert m["klt_predicted"] <= 4
    rows = lp.track_rows()
    assert sum(1 for r in rows if r[-1] > 0) <= 4


def test_bench_cpu_baseline_leg_runs_on_cpu():
    """bench.py's CPU baseline (the loop oracle with the C++ host tracker and
    concurrent GFTT calls) runs and matches the pure-Python tracker's frames."""
    import argparse

    sys.path.insert(0, ROOT)
    import bench

    fr, gt = L.O.synth(5, 640, 480, 8, 0, 6)
    args = argparse.Namespace(bounds="frame", win=21, max_level=2, redetect=5)
    fps, n = bench.cpu_baseline(fr, gt, args, 0.05, 2)
    assert fps > 0 and n >= 3
    # the native tracker adapter gives the same loop as the pure-Python tracker
    from concurrent.futures import ThreadPoolExecutor

    a = L.KltTbdLoop(640, 480, bounds=(0, 640, 0, 480), nthreads=2)
    with ThreadPoolExecutor(2) as pool:
        b = L.KltTbdLoop(640, 480, nthreads=2, tracker=bench._NativeTracker((0, 640, 0, 480)), gftt_pool=pool)
        for f in range(6):
            assert a.step(fr[f], f, L.detections(gt[f], f)) == b.step(fr[f], f, L.detections(gt[f], f))
            assert a.track_rows() == b.track_rows()
