"""tbd_loop_oracle.py — the KLT tracking-by-detection loop composed from the
oracle's independent restatements.  TEST INFRASTRUCTURE ONLY: tests/ drive it
next to libtbdk's native loop (tbdk_tbd_run / tbdk_tbd_step_ahead) on the same
synthetic sequence and compare every frame; the product never imports it.

The reference's frame loop is samples/gpu/tbd.cpp:624-706: per frame
Tracker::performTrackingStep (modules/trackingbydetection/src/tbd.cpp:210-286),
whose predictNewLocationsOfTracks (:288-304) asks Track::motionModel
(include/opencv2/tbd.hpp:111) for each track's predicted centre.  north_star's
KLT box propagation is that motion model, built from the reference's own
primitives, as videostab's KeypointBasedMotionEstimatorGpu composes them
(modules/videostab/src/global_motion.cpp:804-863: GFTT -> PyrLK -> keep
status 1 -> motion fit):

  per frame f (frame id f):
    1. P_f = buildOpticalFlowPyramid(frame f)          lkpyramid.cpp:697-793
    2. every track owning a point set (tracker order): its corners from frame
       f-1 -> calcOpticalFlowPyrLK(P_{f-1}, P_f)        lkpyramid.cpp:1207-1377
       (win 21, maxLevel 2, COUNT+EPS (30, 0.01), minEig 1e-4, err =
       noArray()); keep the status-1 pairs, they are the set from now on
    3. >= min_fit pairs: getRTMatrix(fullAffine=false)  lkpyramid.cpp:1398-1470
       solved by cv::solve(DECOMP_EIG) (box_fit_oracle); the track's last box
       centre (x + w/2, y + h/2, tbd.cpp:1064-1065) mapped through it is the
       prediction, valid when 0.5 < scale < 2 and finite
    4. Tracker::performTrackingStep(detections, f) with those predictions in
       place of the constant-velocity model (tbd_oracle.Tracker)
    5. tracks the step created, and tracks on a re-detection frame (f % 5 == 0)
       or left with < min_points corners: goodFeaturesToTrack(256, 0.01, 3) in
       the track's box clipped to the frame, as an isolated ROI
       (featureselect.cpp:361-516); a box under 3x3 gets an empty set.
  Point sets live in a pool of max_tracks slots, handed out lowest-first; a
  track created with the pool exhausted keeps the constant-velocity model.

Every piece is an independent restatement: the pyramid, PyrLK and GFTT are the
C oracle (klt_oracle.c, gftt_oracle.c), the fit is numpy's eigen-solve of the
reference's normal equations, the tracker is pure Python.  Nothing here reads
libtbdk's outputs.
"""
from __future__ import annotations

import heapq
import math
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, _HERE)
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "tests"))

import _oracle as O  # noqa: E402  (ctypes binding of oracle/liboracle.so)
import box_fit_oracle as BF  # noqa: E402
import tbd_oracle as T  # noqa: E402


class KltTbdLoop:
    """One stream of the KLT TBD loop; parameters are tbdk_tbd_default_config's."""

    def __init__(self, width, height, win=21, max_level=2, lk_iters=30, lk_epsilon=0.01, min_eig=1e-4,
                 max_corners=256, quality=0.01, min_distance=3.0, redetect_every=5, min_points=32,
                 min_fit_points=4, bounds=(0, 1280, 0, 720), max_tracks=1024, accum=None, nthreads=16,
                 tracker=None, gftt_pool=None, shadow_accum=None, **tracker_args):
        """tracker: an object with tbd_oracle.Tracker's step / tracks / metric lists
        (default: tbd_oracle.Tracker); gftt_pool: an executor running the ROIs'
        goodFeaturesToTrack calls concurrently (default: one after another);
        shadow_accum: also run every frame's PyrLK call on the same inputs in this
        accumulation order (it drives nothing) and keep both calls' outputs and
        gate margins in self.shadow (SURVEY.md §8(c)'s per-call tolerance along
        the loop's own trajectory)."""
        self.W, self.H = width, height
        self.win, self.ml, self.iters, self.eps, self.min_eig = win, max_level, lk_iters, lk_epsilon, min_eig
        self.max_corners, self.quality, self.min_distance = max_corners, quality, min_distance
        self.redetect, self.min_points, self.min_fit = redetect_every, min_points, min_fit_points
        self.accum = O.ACCUM_EXACT if accum is None else accum
        self.nthreads = nthreads
        self.tracker = tracker if tracker is not None else T.Tracker(bounds=bounds, **tracker_args)
        self.gftt_pool = gftt_pool
        self.prev = None
        self.sets = {}     # track id -> float32 (n, 2) corners of the last frame
        self.npts = {}     # track id -> corners left after the last fit
        self.slot = {}     # track id -> slot
        self.free = list(range(max_tracks))
        heapq.heapify(self.free)
        self.preds = {}
        self.metrics = {}
        self.shadow_accum = shadow_accum
        self.shadow = None

    def _klt(self, P):
        """Steps 2-3 for every slotted track, in the tracker's order."""
        ids = [t.id for t in self.tracker.tracks if t.id in self.slot]
        counts = [len(self.sets.get(i, ())) for i in ids]
        pts = np.concatenate([self.sets[i] for i in ids if len(self.sets.get(i, ()))]) if sum(counts) else \
            np.zeros((0, 2), np.float32)
        gate = np.empty(len(pts), np.float32) if self.shadow_accum is not None else None
        nxt, st, _, _ = O.lk(self.prev, P, pts, (self.win, self.win), self.ml, self.iters, self.eps, 0,
                             self.min_eig, self.accum, self.nthreads, want_err=False, gate=gate)
        if self.shadow_accum is not None:
            sgate = np.empty(len(pts), np.float32)
            snxt, sst, _, _ = O.lk(self.prev, P, pts, (self.win, self.win), self.ml, self.iters, self.eps, 0,
                                   self.min_eig, self.shadow_accum, self.nthreads, want_err=False, gate=sgate)
            self.shadow = dict(nxt=nxt, st=st, gate=gate, s_nxt=snxt, s_st=sst, s_gate=sgate)
        preds, off, tracked = {}, 0, 0
        boxes = {t.id: t.bboxes[-1] for t in self.tracker.tracks}
        for i, n in zip(ids, counts):
            ok = st[off:off + n] == 1
            a, b = pts[off:off + n][ok], nxt[off:off + n][ok]
            off += n
            self.sets[i] = b
            self.npts[i] = len(b)
            tracked += len(b)
            if len(b) < self.min_fit:
                continue
            M = BF.get_rt_matrix(a, b)
            bb = boxes[i]
            cx, cy = BF.propagate_box(M, (bb.x, bb.y, bb.width, bb.height))
            scale = math.hypot(M[0, 0], M[1, 0])
            if 0.5 < scale < 2.0 and math.isfinite(cx) and math.isfinite(cy):
                preds[i] = (cx, cy)
        return preds, int(sum(counts)), tracked

    def step(self, frame: np.ndarray, frame_id: int, dets):
        """dets: tbd_oracle.Detection list of this frame."""
        P = O.Pyramid(frame, (self.win, self.win), self.ml)
        preds, lk_points, tracked = {}, 0, 0
        self.shadow = None
        if self.prev is not None and self.tracker.tracks:
            preds, lk_points, tracked = self._klt(P)
        before = {t.id for t in self.tracker.tracks}
        self.tracker.step(dets, frame_id, preds)
        after = {t.id for t in self.tracker.tracks}
        for i in before - after:  # filtered out of bounds or lost: the slot returns to the pool
            s = self.slot.pop(i, None)
            if s is not None:
                heapq.heappush(self.free, s)
            self.sets.pop(i, None)
            self.npts.pop(i, None)
        rois, owners, refreshed = [], [], 0
        for t in self.tracker.tracks:
            if t.id not in self.slot:
                if not self.free:
                    continue  # pool exhausted: constant-velocity model for this track
                self.slot[t.id] = heapq.heappop(self.free)
            elif frame_id % self.redetect != 0 and self.npts.get(t.id, 0) >= self.min_points:
                continue
            b = t.bboxes[-1]
            x0, y0 = max(b.x, 0), max(b.y, 0)
            x1, y1 = min(b.x + b.width, self.W), min(b.y + b.height, self.H)
            self.npts[t.id] = self.max_corners
            refreshed += 1
            if x1 - x0 < 3 or y1 - y0 < 3:
                self.sets[t.id] = np.zeros((0, 2), np.float32)
                continue
            rois.append((x0, y0, x1 - x0, y1 - y0))
            owners.append(t.id)
        if self.gftt_pool is not None:
            found = list(self.gftt_pool.map(lambda r: O.gftt_rois(frame, [r], self.max_corners, self.quality,
                                                                   self.min_distance)[0], rois))
        else:
            found = O.gftt_rois(frame, rois, self.max_corners, self.quality, self.min_distance)
        for i, c in zip(owners, found):
            self.sets[i] = np.ascontiguousarray(c, np.float32)
        self.prev = P
        self.preds = preds
        tk = self.tracker
        self.metrics = dict(tp=tk.true_positives[-1], fn=tk.false_negatives[-1], fp=tk.false_positives[-1],
                            gt=tk.ground_truths[-1], ntracks=len(tk.tracks), lk_points=lk_points,
                            klt_points=tracked, klt_predicted=len(preds), redetected=refreshed)
        return self.metrics

    def track_rows(self):
        """(id, x, y, w, h, pred x, y, w, h, age, visible, corners) per track, tracker order."""
        out = []
        for t in self.tracker.tracks:
            b, p = t.bboxes[-1], t.predPosition
            out.append((t.id, b.x, b.y, b.width, b.height, p.x, p.y, p.width, p.height, t.age,
                        t.totalVisibleCount, len(self.sets.get(t.id, ())) if t.id in self.slot else 0))
        return out


def detections(gt_frame, frame_id: int, keep=None):
    """GT rows {valid, x, y, w, h} -> tbd_oracle.Detection (id = object index,
    confidence 1.0), as parseDetections builds them (samples/gpu/tbd.cpp:1297-1340)."""
    g = np.asarray(gt_frame)
    out = []
    for k in np.nonzero(g[:, 0])[0]:
        if keep is not None and not keep[k]:
            continue
        out.append(T.Detection(int(k), frame_id, T.Rect(int(g[k, 1]), int(g[k, 2]), int(g[k, 3]), int(g[k, 4])), 1.0))
    return out
