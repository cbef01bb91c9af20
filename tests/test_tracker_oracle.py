"""The native tracker of libtbdk (host-only C ABI tbdk_tracker_*) against the
pure-Python restatement of the reference cv::tbd::Tracker (oracle/tbd_oracle.py):
identical tracks (ids, boxes, predicted boxes, ages, visibility, confidence,
overlap) and identical per-frame metrics, bit for bit, on GT-driven sequences
with dropouts, jitter, clutter, low-confidence detections, degenerate boxes,
the reference's 1280x720 filter at 1080p, and KLT-style predicted centres.
No GPU needed."""
import ctypes as C
import math
import os
import sys

import numpy as np
import pytest

from opencv_amd import _lib


sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import tbd_oracle as T  # noqa: E402


class Native:
    """the package's cv::tbd::Tracker mirror (opencv_amd.tbd.Tracker)"""

    def __init__(self, bounds):
        from opencv_amd import tbd

        self.t = tbd.Tracker(bounds=bounds)

    def step(self, dets, frame_id, preds):
        from opencv_amd import tbd

        arr = np.zeros(len(dets), tbd.DET_DTYPE)
        for i, d in enumerate(dets):
            arr[i] = (d.id, d.bbox.x, d.bbox.y, d.bbox.width, d.bbox.height, d.confidence)
        m = self.t.performTrackingStep(arr, frame_id, preds)
        return m, self.t.getTracks()


def same_float(a, b):
    return (math.isnan(a) and math.isnan(b)) or a == b


def compare(frame, ora: T.Tracker, m, tracks):
    ctx = f"frame {frame}"
    assert (m.tp, m.fn, m.fp, m.gt, m.matches) == (ora.true_positives[-1], ora.false_negatives[-1],
                                                   ora.false_positives[-1], ora.ground_truths[-1],
                                                   ora.num_matches[-1]), ctx
    assert same_float(m.bbox_overlap, ora.bbox_overlap[-1]), ctx
    assert len(tracks) == len(ora.tracks) == m.ntracks, ctx
    for got, t in zip(tracks, ora.tracks):
        b, p = t.bboxes[-1], t.predPosition
        assert (got.id, got.x, got.y, got.width, got.height) == (t.id, b.x, b.y, b.width, b.height), ctx
        assert (got.pred_x, got.pred_y, got.pred_w, got.pred_h) == (p.x, p.y, p.width, p.height), ctx
        assert (got.age, got.total_visible) == (t.age, t.totalVisibleCount), ctx
        assert same_float(got.max_confidence, t.maxConfidence), ctx
        assert same_float(got.bbox_overlap, t.bboxOverlap), ctx


def sequence(seed, W, H, nobj, nframes, dropout, jitter, clutter, lowconf, degenerate):
    """GT-like detections of bouncing boxes with detector noise."""
    rng = np.random.default_rng(seed)
    pos = rng.uniform([0, 0], [W - 64, H - 64], (nobj, 2))
    vel = rng.uniform(-6, 6, (nobj, 2))
    size = rng.integers(24, 200, (nobj, 2))
    for f in range(nframes):
        dets = []
        for o in range(nobj):
            pos[o] += vel[o]
            for k, lim in ((0, W), (1, H)):
                if pos[o, k] < -40 or pos[o, k] > lim - 20:
                    vel[o, k] = -vel[o, k]
            if rng.random() < dropout:
                continue
            x, y = (pos[o] + rng.integers(-jitter, jitter + 1, 2)).astype(int)
            w, h = (size[o] + rng.integers(-jitter, jitter + 1, 2)).clip(1).astype(int)
            conf = 1.0 if rng.random() >= lowconf else float(rng.uniform(0.0, 0.4))
            dets.append(T.Detection(o, f, T.Rect(int(x), int(y), int(w), int(h)), conf))
        for _ in range(rng.poisson(clutter)):
            x, y = rng.integers(0, W), rng.integers(0, H)
            w, h = rng.integers(0 if degenerate else 8, 120, 2)
            dets.append(T.Detection(-1, f, T.Rect(int(x), int(y), int(w), int(h)), float(rng.uniform(0, 1))))
        rng.shuffle(dets)
        yield f, dets, rng


CASES = [
    dict(seed=1, W=1280, H=720, nobj=24, nframes=60, dropout=0.1, jitter=3, clutter=1.0, lowconf=0.05,
         degenerate=False, preds=0.0),
    dict(seed=2, W=1920, H=1080, nobj=40, nframes=50, dropout=0.15, jitter=2, clutter=2.0, lowconf=0.1,
         degenerate=False, preds=0.0),
    dict(seed=3, W=1280, H=720, nobj=30, nframes=50, dropout=0.05, jitter=4, clutter=0.5, lowconf=0.0,
         degenerate=True, preds=0.6),
    dict(seed=4, W=640, H=480, nobj=12, nframes=80, dropout=0.3, jitter=6, clutter=3.0, lowconf=0.2,
         degenerate=True, preds=0.3),
]


@pytest.mark.parametrize("case", CASES, ids=[f"seed{c['seed']}" for c in CASES])
@pytest.mark.parametrize("bounds", ["reference", "frame"])
def test_native_tracker_matches_reference_restatement(case, bounds):
    bnd = (0, 1280, 0, 720) if bounds == "reference" else (0, case["W"], 0, case["H"])
    ora = T.Tracker(bounds=bnd)
    nat = Native(bnd)
    for f, dets, rng in sequence(case["seed"], case["W"], case["H"], case["nobj"], case["nframes"],
                                 case["dropout"], case["jitter"], case["clutter"], case["lowconf"],
                                 case["degenerate"]):
        preds = {}
        for t in ora.tracks:  # KLT-style predicted centres for a subset of the live tracks
            if rng.random() < case["preds"]:
                b = t.bboxes[-1]
                preds[t.id] = (b.x + b.width / 2 + float(rng.normal(0, 3)), b.y + b.height / 2 + float(rng.normal(0, 3)))
        ora.step(dets, f, preds)
        m, tracks = nat.step(dets, f, preds)
        compare(f, ora, m, tracks)


def test_tracker_empty_and_argument_errors():
    lib = _lib.load()
    a = _lib.TrackerArgs()
    lib.tbdk_tracker_default_args(C.byref(a))
    assert (a.bounds_xmax, a.bounds_ymax, a.time_window_size) == (1280, 720, 16)
    a.time_window_size = 0
    h = C.c_void_p()
    assert lib.tbdk_tracker_create(C.byref(a), C.byref(h)) == _lib.TBDK_EINVAL
    nat = Native((0, 1280, 0, 720))
    ora = T.Tracker()
    for f in range(5):  # no detections at all, then one, then none
        dets = [T.Detection(0, f, T.Rect(10, 10, 30, 30), 1.0)] if f == 2 else []
        ora.step(dets, f)
        m, tr = nat.step(dets, f, {})
        compare(f, ora, m, tr)
