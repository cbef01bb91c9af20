"""tbd_oracle.py — pure-Python restatement of the reference tracker
cv::tbd::Tracker (modules/trackingbydetection/src/tbd.cpp, include/opencv2/tbd.hpp).

TEST INFRASTRUCTURE ONLY (tests/ use it as the checker of the native tracker in
libtbdk; the product never imports it).  It follows the reference function by
function with its data structures: ever-growing per-track vectors, a
vector<vector<double>> cost matrix padded to a square, and the same loop order
everywhere, so every floating-point comparison sees the same doubles:

  Track(Detection&)                       tbd.cpp:67-91
  performTrackingStep                     tbd.cpp:210-286
  predictNewLocationsOfTracks             tbd.cpp:288-304
  filterTracksOutOfBounds                 tbd.cpp:306-331 (bounds hard-coded there: 0,1280,0,720)
  calculateCostMatrix                     tbd.cpp:333-351
  classifyAssignments                     tbd.cpp:353-379
  solveAssignmentProblem                  tbd.cpp:381-891
  updateTrackConfidence                   tbd.cpp:913-930
  updateAssignedTracks                    tbd.cpp:935-981
  updateUnassignedTracks                  tbd.cpp:986-1009
  deleteLostTracks                        tbd.cpp:1011-1037
  createNewTracks                         tbd.cpp:1043-1055
  constantVelocityMotionModel             tbd.cpp:1057-1083
  computeBoundingBoxOverlap               tbd.cpp:1085-1106
  equalsZero                              tbd.hpp:180-183

The product's KLT hook (a per-track predicted centre replacing
Track::motionModel, tbd.hpp:111) is modelled by `preds`: {track_id: (cx, cy)}.
C semantics restated: int division truncates toward zero; Rect(Point2d, Size)
rounds with cvRound (half to even; Python's round() on floats is the same);
double division by zero gives inf/nan as IEEE does.
"""
from __future__ import annotations

import copy
import math
from dataclasses import dataclass, field


def c_div(a: int, b: int) -> int:
    """C integer division (truncation toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def ieee_div(a: float, b: float) -> float:
    if b == 0:
        if a == 0 or math.isnan(a):
            return math.nan
        return math.copysign(math.inf, a) * (1 if math.copysign(1, b) > 0 else -1)
    return a / b


def cv_round(v: float) -> int:
    """cvRound(double): nearest, ties to even."""
    return int(round(v))


@dataclass
class Rect:
    x: int
    y: int
    width: int
    height: int

    def area(self) -> int:
        return self.width * self.height


def rect_from_point2d(px: float, py: float, w: int, h: int) -> Rect:
    return Rect(cv_round(px), cv_round(py), w, h)


@dataclass
class Detection:
    id: int
    frame_id: int
    bbox: Rect
    confidence: float


@dataclass
class Track:
    id: int
    bboxes: list = field(default_factory=list)
    scores: list = field(default_factory=list)
    frames: list = field(default_factory=list)
    age: int = 1
    totalVisibleCount: int = 1
    maxConfidence: float = 0.0
    avgConfidence: float = 0.0
    predPosition: Rect | None = None
    bboxOverlap: float = 1.0
    color: tuple = (0, 0, 0)


def traj_get(traj: dict, key: int):
    """std::map<int, Trajectory>::operator[]: default-constructs (id -1) when absent."""
    if key not in traj:
        from tbd_app_oracle import Trajectory  # noqa: PLC0415 (sibling module, avoids a cycle)
        traj[key] = Trajectory(-1)
    return traj[key]


def equals_zero(v: float) -> bool:
    return (v > -0.00000001) if v < 0.0 else (v < 0.00000001)


def compute_bounding_box_overlap(p: Rect, b: Rect) -> float:
    xleft = float(max(p.x, b.x))
    xright = float(min(p.x + p.width, b.x + b.width))
    ytop = float(max(p.y, b.y))
    ybottom = float(min(p.y + p.height, b.y + b.height))
    if xright < xleft or ybottom < ytop:
        return 0.0
    inter = (xright - xleft) * (ybottom - ytop)
    union = float(p.area() + b.area()) - inter
    return ieee_div(inter, union)


def constant_velocity_motion_model(t: Track, frame_id: int):
    if t.age == 1:
        b = t.bboxes[-1]
        return float(b.x + c_div(b.width, 2)), float(b.y + c_div(b.height, 2))
    f1, f2 = t.frames[-1], t.frames[-2]
    b1, b2 = t.bboxes[-1], t.bboxes[-2]
    ratio = ieee_div(float(frame_id - f1), float(f1 - f2))
    dx = ratio * (b1.x - b2.x)
    dy = ratio * (b1.y - b2.y)
    w = (b1.width + b2.width) / 2.0
    h = (b1.height + b2.height) / 2.0
    return b1.x + w / 2 + dx, b1.y + h / 2 + dy


class Tracker:
    def __init__(self, cost_of_non_assignment=10.0, time_window_size=16, track_age_threshold=4,
                 track_visibility_threshold=0.3, track_confidence_threshold=0.2,
                 bounds=(0, 1280, 0, 720)):
        self.cost_of_non_assignment = cost_of_non_assignment
        self.time_window_size = time_window_size
        self.track_age_threshold = track_age_threshold
        self.track_visibility_threshold = track_visibility_threshold
        self.track_confidence_threshold = track_confidence_threshold
        self.bounds = bounds
        self.rng = None            # CRand drawn for track colours (tbd_app_oracle), or None
        self.next_track_id = 0
        self.tracks: list[Track] = []
        self.true_positives, self.false_negatives, self.false_positives = [], [], []
        self.ground_truths, self.num_matches, self.bbox_overlap = [], [], []

    # tbd.cpp:67-91
    def _new_track(self, d: Detection) -> Track:
        t = Track(id=self.next_track_id)
        self.next_track_id += 1
        if self.rng is not None:  # Scalar(rand() % 256, rand() % 256, rand() % 256), tbd.cpp:71-74
            t.color = (self.rng.rand() % 256, self.rng.rand() % 256, self.rng.rand() % 256)
        t.bboxes.append(d.bbox)
        t.scores.append(d.confidence)
        t.frames.append(d.frame_id)
        t.age = 1
        t.totalVisibleCount = 1
        t.maxConfidence = d.confidence
        t.avgConfidence = d.confidence
        t.predPosition = d.bbox
        t.bboxOverlap = 1.0
        return t

    # tbd.cpp:197-208
    def reset(self):
        self.next_track_id = 0
        self.tracks = []
        self.true_positives, self.false_negatives, self.false_positives = [], [], []
        self.ground_truths, self.num_matches, self.bbox_overlap = [], [], []

    # tbd.cpp:187-190 (Track copy constructor per element, tbd.cpp:93-117)
    def set_tracks(self, tracks):
        self.tracks = [copy.deepcopy(t) for t in tracks]

    # tbd.cpp:210-286; traj: {gt id: Trajectory} (tbd_app_oracle), or None
    def step(self, dets: list[Detection], frame_id: int, preds: dict | None = None, traj: dict | None = None):
        self._predict(frame_id, preds or {})
        self._filter_out_of_bounds(*self.bounds)
        assignments, un_tracks, un_dets = self._assign(dets)
        self._update_assigned(dets, assignments)
        self._update_unassigned(un_tracks, frame_id)
        num_assigned = 0
        for i, t in enumerate(self.tracks):
            if assignments[i] < 0:
                continue
            num_assigned += 1
            d = dets[assignments[i]]
            if traj is not None and d.id >= 0:
                traj_get(traj, d.id).add_tracking_info(frame_id, t)
        if traj is not None:
            for j in un_dets:
                if dets[j].id >= 0:
                    traj_get(traj, dets[j].id).add_tracking_info(frame_id, None)
        self._delete_lost()
        for j in un_dets:
            self.tracks.append(self._new_track(dets[j]))
        self.true_positives.append(num_assigned)
        self.false_negatives.append(len(un_dets))
        self.false_positives.append(len(un_tracks))
        self.ground_truths.append(len(dets))
        self.num_matches.append(num_assigned)
        ov = 0.0
        for t in self.tracks:
            ov += t.bboxOverlap
        self.bbox_overlap.append(ov)

    # tbd.cpp:288-304
    def _predict(self, frame_id, preds):
        for t in self.tracks:
            b = t.bboxes[-1]
            if t.id in preds:
                cx, cy = preds[t.id]
            else:
                cx, cy = constant_velocity_motion_model(t, frame_id)
            t.predPosition = rect_from_point2d(cx - c_div(b.width, 2), cy - c_div(b.height, 2), b.width, b.height)

    # tbd.cpp:306-331
    def _filter_out_of_bounds(self, xmin, xmax, ymin, ymax):
        filtered = []
        for i, t in enumerate(self.tracks):
            r = t.predPosition
            if r.x + r.width < xmin or r.x >= xmax or r.y + r.height < ymin or r.y >= ymax:
                filtered.append(i)
        for i in reversed(filtered):
            del self.tracks[i]

    # detectionToTrackAssignment: calculateCostMatrix (:333-351) + solveAssignmentProblem (:381-891)
    def _assign(self, dets):
        cost = []
        for t in self.tracks:
            cost.append([1.0 - compute_bounding_box_overlap(t.predPosition, d.bbox) for d in dets])
        num_tracks, num_dets = len(self.tracks), len(dets)
        huge = 10000000.0
        if num_tracks > num_dets:
            for i in range(num_tracks):
                for _ in range(num_tracks - num_dets):
                    cost[i].append(self.cost_of_non_assignment * 2)
        if num_dets > num_tracks:
            for _ in range(num_dets - num_tracks):
                cost.append([self.cost_of_non_assignment * 2] * num_dets)
        n = len(cost)
        per_row = [n] * n
        if n == 0:
            return self._classify(per_row, num_tracks, num_dets)
        for r in range(n):  # step 1
            m = huge
            for c in range(n):
                m = cost[r][c] if cost[r][c] < m else m
            for c in range(n):
                cost[r][c] -= m
        for c in range(n):  # step 2
            m = huge
            for r in range(n):
                m = cost[r][c] if cost[r][c] < m else m
            for r in range(n):
                cost[r][c] -= m
        while True:
            row_a = [False] * n
            col_a = [False] * n
            num_assigned = 0
            per_row = [n] * n
            made = True
            while made:
                made = False
                for r in range(n):
                    if row_a[r]:
                        continue
                    z = [c for c in range(n) if equals_zero(cost[r][c])]
                    if len(z) == 1 and not col_a[z[0]]:
                        row_a[r] = col_a[z[0]] = True
                        per_row[r] = z[0]
                        made = True
                        num_assigned += 1
                for c in range(n):
                    if col_a[c]:
                        continue
                    z = [r for r in range(n) if equals_zero(cost[r][c])]
                    if len(z) == 1 and not row_a[z[0]]:
                        row_a[z[0]] = col_a[c] = True
                        per_row[z[0]] = c
                        made = True
                        num_assigned += 1
                if not made:
                    for r in range(n):
                        if row_a[r]:
                            continue
                        z = [c for c in range(n) if equals_zero(cost[r][c])]
                        for c in z:
                            if not col_a[c]:
                                row_a[r] = col_a[c] = True
                                per_row[r] = c
                                made = True
                                num_assigned += 1
                                break
            if num_assigned == n:
                break
            # step 3
            row_m = [not row_a[r] for r in range(n)]
            col_m = [False] * n
            while True:
                newly = 0
                for r in range(n):
                    if not row_m[r]:
                        continue
                    for c in range(n):
                        if equals_zero(cost[r][c]) and not col_m[c]:
                            col_m[c] = True
                            newly += 1
                for c in range(n):
                    if not col_m[c]:
                        continue
                    for r2 in range(n):
                        if per_row[r2] == c:
                            row_m[r2] = True
                if newly == 0:
                    break
            row_cov = [not row_m[r] for r in range(n)]
            if all(row_m):
                break
            col_cov = list(col_m)
            # step 4
            mu = huge
            for r in range(n):
                if row_cov[r]:
                    continue
                for c in range(n):
                    if col_cov[c]:
                        continue
                    mu = cost[r][c] if cost[r][c] < mu else mu
            for r in range(n):
                for c in range(n):
                    if not row_cov[r] and not col_cov[c]:
                        cost[r][c] -= mu
                    elif row_cov[r] and col_cov[c]:
                        cost[r][c] += mu
        return self._classify(per_row, num_tracks, num_dets)

    # tbd.cpp:353-379
    @staticmethod
    def _classify(per_row, num_tracks, num_dets):
        assignments, un_tracks = [], []
        det_a = [False] * num_dets
        for i in range(num_tracks):
            if per_row[i] < num_dets:
                assignments.append(per_row[i])
                det_a[per_row[i]] = True
            else:
                assignments.append(-1)
                un_tracks.append(i)
        un_dets = [j for j in range(num_dets) if not det_a[j]]
        return assignments, un_tracks, un_dets

    # tbd.cpp:913-930
    def _update_confidence(self, t: Track):
        num = min(len(t.scores), self.time_window_size)
        mx, s = 0.0, 0.0
        for k in range(len(t.scores) - num, len(t.scores)):
            sc = t.scores[k]
            s += sc
            if sc > mx:
                mx = sc
        t.maxConfidence = mx
        t.avgConfidence = ieee_div(s, float(num))

    # tbd.cpp:935-981
    def _update_assigned(self, dets, assignments):
        for i, t in enumerate(self.tracks):
            if assignments[i] < 0:
                continue
            d = dets[assignments[i]]
            nprior = min(len(t.bboxes), 4)
            wsum = hsum = 0
            for k in range(len(t.bboxes) - nprior, len(t.bboxes)):
                wsum += t.bboxes[k].width
                hsum += t.bboxes[k].height
            w = (wsum + d.bbox.width) // (nprior + 1)   # unsigned arithmetic, positive sizes
            h = (hsum + d.bbox.height) // (nprior + 1)
            cx = float(d.bbox.x)
            cy = float(d.bbox.y)
            cx += c_div(d.bbox.width, 2) - c_div(w, 2)
            cy += c_div(d.bbox.height, 2) - c_div(h, 2)
            t.bboxes.append(rect_from_point2d(cx, cy, w, h))
            t.frames.append(d.frame_id)
            t.bboxOverlap = compute_bounding_box_overlap(d.bbox, t.predPosition)
            t.age += 1
            t.totalVisibleCount += 1
            t.scores.append(d.confidence)
            self._update_confidence(t)

    # tbd.cpp:986-1009
    def _update_unassigned(self, un_tracks, frame_id):
        for i in un_tracks:
            t = self.tracks[i]
            t.age += 1
            t.bboxes.append(t.predPosition)
            t.scores.append(0.0)
            t.frames.append(frame_id)
            t.bboxOverlap = 0.0
            self._update_confidence(t)

    # tbd.cpp:1011-1037
    def _delete_lost(self):
        dead = []
        for i, t in enumerate(self.tracks):
            vis = t.totalVisibleCount / t.age
            if (t.age <= self.track_age_threshold and vis <= self.track_visibility_threshold) or \
                    (t.maxConfidence >= 0.0 and t.maxConfidence <= self.track_confidence_threshold):
                dead.append(i)
        for i in reversed(dead):
            del self.tracks[i]
