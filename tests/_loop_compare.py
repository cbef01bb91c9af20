"""Loop-level comparison of the TBD loop in the GPU's accumulation order with
the reference's SSE2 order (TEST INFRASTRUCTURE ONLY; used by
tests/test_gpu_tbd_e2e.py and tests/loop_divergence_cpu.py).

The GPU's PyrLK sums G and b exactly (integers) and rounds once; the reference
adds float products in SSE2 lane order (video/src/lkpyramid.cpp:278-316,
422-440, 507-534, 619-633).  Both are restated by the oracle (ACCUM_EXACT /
ACCUM_SSE2), and the GPU is bit-exact with ACCUM_EXACT.  Two measurements:

* per call (`CallStats`): every frame's PyrLK call of the exact-order loop is
  re-run in SSE2 order on the SAME inputs (KltTbdLoop(shadow_accum=...)), so
  the comparison follows the loop's whole trajectory: |dnextPts| of the
  points tracked by both, status agreement, and for every status
  disagreement the smallest relative gate margin either order saw
  ("any disagreement must lie within 1e-3 (relative) of the
  minEig/bounds thresholds");
* per loop (`LoopStats`): two independent loops, one per order, each driving
  itself; per frame the metrics (TP/FN/FP/GT, IDSW-relevant track ids) and
  every common track's predPosition (the cvRound-ed Rect of
  tbd.cpp:288-304) compared, with the first frame that differs.
"""
from __future__ import annotations

import numpy as np

METRIC_KEYS = ("tp", "fn", "fp", "gt", "ntracks", "lk_points", "klt_points", "klt_predicted", "redetected")


class CallStats:
    """Accumulates KltTbdLoop.shadow over frames."""

    def __init__(self):
        self.points = 0
        self.both_tracked = 0
        self.within_1e2 = 0
        self.max_dev = 0.0
        self.status_disagree = 0
        self.worst_gate = 0.0         # max over disagreements of min(gate_exact, gate_sse2)
        self.ref_criterion_bad = 0    # the reference's own: int-truncated positions differ (test_optflow.cpp:241-264)
        self.calls = 0

    def add(self, sh):
        if sh is None or len(sh["st"]) == 0:
            return
        self.calls += 1
        st, sst = sh["st"], sh["s_st"]
        n = len(st)
        self.points += n
        both = (st == 1) & (sst == 1)
        d = np.abs(sh["nxt"][both].astype(np.float64) - sh["s_nxt"][both].astype(np.float64)).max(axis=1) \
            if both.any() else np.zeros(0)
        self.both_tracked += int(both.sum())
        self.within_1e2 += int((d <= 1e-2).sum())
        if d.size:
            self.max_dev = max(self.max_dev, float(d.max()))
        ia = sh["nxt"][both].astype(np.int32)
        ib = sh["s_nxt"][both].astype(np.int32)
        self.ref_criterion_bad += int((np.abs(ia - ib) > 1).any(axis=1).sum())
        dis = st != sst
        k = int(dis.sum())
        self.status_disagree += k
        if k:
            g = np.minimum(sh["gate"][dis], sh["s_gate"][dis])
            self.worst_gate = max(self.worst_gate, float(g.max()))

    def summary(self):
        return dict(calls=self.calls, points=self.points, both_tracked=self.both_tracked,
                    frac_within_1e2=self.within_1e2 / max(1, self.both_tracked), max_dev_px=self.max_dev,
                    status_disagree=self.status_disagree,
                    status_agree=1.0 - self.status_disagree / max(1, self.points),
                    worst_disagreement_gate_margin=self.worst_gate,
                    ref_criterion_mismatch=self.ref_criterion_bad / max(1, self.both_tracked))


def track_map(rows):
    """KltTbdLoop.track_rows / tbdk rows -> {id: (box, predPosition)}"""
    return {r[0]: (tuple(r[1:5]), tuple(r[5:9])) for r in rows}


class LoopStats:
    """Per-frame comparison of two independently driven loops."""

    def __init__(self):
        self.frames = 0
        self.metric_equal = 0
        self.tpfnfp_equal = 0
        self.first_metric_diff = None
        self.track_frames = 0
        self.pred_equal = 0
        self.box_equal = 0
        self.first_pred_diff = None
        self.track_set_equal = 0

    def add(self, f, ma, mb, rows_a, rows_b):
        self.frames += 1
        if ma == mb:
            self.metric_equal += 1
        elif self.first_metric_diff is None:
            self.first_metric_diff = f
        if all(ma[k] == mb[k] for k in ("tp", "fn", "fp", "gt")):
            self.tpfnfp_equal += 1
        a, b = track_map(rows_a), track_map(rows_b)
        if a.keys() == b.keys():
            self.track_set_equal += 1
        ids = a.keys() | b.keys()
        self.track_frames += len(ids)
        for i in ids:
            if i in a and i in b:
                self.box_equal += a[i][0] == b[i][0]
                if a[i][1] == b[i][1]:
                    self.pred_equal += 1
                    continue
            if self.first_pred_diff is None:
                self.first_pred_diff = f

    def summary(self):
        return dict(frames=self.frames, frac_frames_metrics_equal=self.metric_equal / max(1, self.frames),
                    frac_frames_tp_fn_fp_equal=self.tpfnfp_equal / max(1, self.frames),
                    first_metric_diff_frame=self.first_metric_diff,
                    frac_frames_same_track_ids=self.track_set_equal / max(1, self.frames),
                    track_frames=self.track_frames,
                    frac_track_frames_pred_equal=self.pred_equal / max(1, self.track_frames),
                    frac_track_frames_box_equal=self.box_equal / max(1, self.track_frames),
                    first_pred_diff_frame=self.first_pred_diff)
