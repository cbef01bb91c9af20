"""End-to-end TBD loop on the GPU: runs, is deterministic, and the KLT path
actually predicts boxes (GT-driven synthetic sequence)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def run_loop(gpu, W=640, H=480, nobj=16, nframes=30, seed=7, **cfg):
    from opencv_amd import klt, tbd

    frames, gt = klt.synth_render(seed, W, H, nobj, 0, nframes, ctx=gpu)
    c = tbd.default_config(W, H, bounds_xmax=W, bounds_ymax=H, **cfg)
    loop = tbd.TbdLoop(c, ctx=gpu)
    ms = []
    for f in range(nframes):
        m = loop.step(frames[f], f, tbd.detections_from_gt(gt[f].numpy()))
        ms.append((m.tp, m.fn, m.fp, m.gt, m.ntracks, m.lk_points, m.klt_points, m.klt_predicted, m.redetected))
    torch.cuda.synchronize()
    return ms, loop.tracks()


def test_tbd_loop_runs_and_is_deterministic(gpu):
    a, ta = run_loop(gpu)
    b, tb = run_loop(gpu)
    assert a == b and ta == tb
    tp = sum(x[0] for x in a)
    assert tp > 0.8 * sum(x[3] for x in a[1:])  # most GT detections are matched
    assert sum(x[7] for x in a) > 0             # KLT predictions were used
    assert all(x[5] >= x[6] for x in a)         # tracked <= entered


def test_tbd_loop_constant_velocity_mode(gpu):
    a, _ = run_loop(gpu, use_klt=0)
    assert all(x[5] == 0 and x[8] == 0 for x in a)  # no KLT work at all
    assert sum(x[0] for x in a) > 0


def test_tbd_loop_reference_bounds_quirk(gpu):
    from opencv_amd import klt, tbd

    # 1080p with the reference's hard-coded 1280x720 filter (tbd.cpp:218): tracks
    # whose prediction starts beyond it are dropped and re-created every frame
    frames, gt = klt.synth_render(3, 1920, 1080, 32, 0, 6, ctx=gpu)
    loop = tbd.TbdLoop(tbd.default_config(1920, 1080), ctx=gpu)
    for f in range(6):
        m = loop.step(frames[f], f, tbd.detections_from_gt(gt[f].numpy()))
    tr = loop.tracks()
    assert len(tr) > 0


def test_tbd_loop_tracker_matches_reference_restatement(gpu, tmp_path):
    """End to end: every frame, the loop's tracker state equals the pure-Python
    cv::tbd::Tracker restatement (oracle/tbd_oracle.py) fed the same detections
    and the KLT predictions the loop computed on the GPU (ids, boxes, predicted
    boxes, ages, visibility, confidence, overlap, TP/FN/FP/GT)."""
    import math
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import tbd_app_oracle as A
    import tbd_oracle as T
    from opencv_amd import klt, tbd

    W, H, N, F = 1280, 720, 24, 40
    frames, gt = klt.synth_render(11, W, H, N, 0, F, ctx=gpu)
    loop = tbd.TbdLoop(tbd.default_config(W, H), ctx=gpu)
    traj, otraj = tbd.Trajectories(), {}
    loop.set_trajectories(traj)
    ora = T.Tracker(bounds=(0, 1280, 0, 720))
    rng = np.random.default_rng(5)
    used_preds = 0
    for f in range(F):
        d = tbd.detections_from_gt(gt[f].numpy())
        d = d[rng.random(len(d)) > 0.1]  # detector dropouts
        m = loop.step(frames[f], f, d)
        preds = loop.predictions()
        used_preds += len(preds)
        od = [T.Detection(int(r["id"]), f, T.Rect(int(r["x"]), int(r["y"]), int(r["width"]), int(r["height"])),
                          float(r["confidence"])) for r in d]
        for x in od:  # parseDetections' trajectory positions
            otraj.setdefault(x.id, A.Trajectory(x.id)).add_position(f, x.bbox)
        ora.step(od, f, preds, traj=otraj)
        assert (m.tp, m.fn, m.fp, m.gt) == (ora.true_positives[-1], ora.false_negatives[-1],
                                            ora.false_positives[-1], ora.ground_truths[-1]), f
        tr = loop.tracks()
        assert len(tr) == len(ora.tracks), f
        for g, t in zip(tr, ora.tracks):
            b, p = t.bboxes[-1], t.predPosition
            assert (g["id"], g["x"], g["y"], g["width"], g["height"]) == (t.id, b.x, b.y, b.width, b.height), f
            assert (g["pred_x"], g["pred_y"], g["pred_w"], g["pred_h"]) == (p.x, p.y, p.width, p.height), f
            assert (g["age"], g["total_visible"]) == (t.age, t.totalVisibleCount), f
            assert g["max_confidence"] == t.maxConfidence
            assert g["bbox_overlap"] == t.bboxOverlap or (math.isnan(g["bbox_overlap"]) and math.isnan(t.bboxOverlap))
    assert used_preds > 0  # the KLT motion model was exercised
    # the sample's tracking output (history|object|frame|scenario lines) of the GPU loop
    out = os.path.join(str(tmp_path), "track.txt")
    m = loop.write_tracking_output(F, out)
    txt, om = A.write_tracking_output(ora, [1] * F, otraj, F)
    assert open(out).read() == txt
    assert m["mt"] == om["mt"] and m["mota"] == om["mota"]


def _mkey(m):
    return (m.tp, m.fn, m.fp, m.gt, m.matches, m.bbox_overlap, m.ntracks, m.lk_points, m.klt_points,
            m.klt_predicted, m.redetected, m.lk_iters)


@pytest.mark.parametrize("W,H,N,F,cfg", [
    (1280, 720, 24, 30, {}),
    (640, 480, 20, 24, {"redetect_every": 3, "min_points": 120}),  # frequent refreshes
    (640, 480, 40, 24, {"max_tracks": 24, "track_age_threshold": 2}),  # slot pool exhausted, slots reused
])
def test_tbd_lookahead_and_run_match_step(gpu, W, H, N, F, cfg):
    """tbdk_tbd_step_ahead and tbdk_tbd_run (the next frame's pyramid and the
    tracker-independent PyrLK enqueued before the tracker step) give the same
    per-frame metrics, predictions and final tracks as tbdk_tbd_step."""
    from opencv_amd import klt, tbd

    frames, gt = klt.synth_render(21, W, H, N, 0, F, ctx=gpu)
    rng = np.random.default_rng(9)
    dets = []
    for f in range(F):
        d = tbd.detections_from_gt(gt[f].numpy())
        dets.append(np.ascontiguousarray(d[rng.random(len(d)) > 0.15]))
    c = tbd.default_config(W, H, bounds_xmax=W, bounds_ymax=H, **cfg)

    plain = tbd.TbdLoop(c, ctx=gpu)
    ahead = tbd.TbdLoop(c, ctx=gpu)
    ma, mb = [], []
    for f in range(F):
        ma.append(_mkey(plain.step(frames[f], f, dets[f])))
        pa = plain.predictions()
        mb.append(_mkey(ahead.step(frames[f], f, dets[f], next_frame=frames[f + 1] if f + 1 < F else None)))
        assert ahead.predictions() == pa, f"frame {f}"
    assert ma == mb
    assert plain.tracks() == ahead.tracks()

    batch = tbd.TbdLoop(c, ctx=gpu)
    ms = batch.run(frames, 0, dets)
    assert [_mkey(m) for m in ms] == ma
    assert batch.tracks() == plain.tracks()
    assert sum(m[9] for m in ma) > 0 and sum(m[10] for m in ma) > 0


def test_tbd_lookahead_discarded_on_other_frame(gpu):
    """A step whose frame is not the one announced as next_frame (or runs on
    another stream) recomputes everything: same results as plain steps."""
    from opencv_amd import klt, tbd

    W, H, N, F = 640, 480, 16, 12
    frames, gt = klt.synth_render(4, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=W, bounds_ymax=H)
    plain = tbd.TbdLoop(c, ctx=gpu)
    odd = tbd.TbdLoop(c, ctx=gpu)
    other = torch.cuda.Stream()
    wrong = frames[0].clone()
    for f in range(F):
        a = _mkey(plain.step(frames[f], f, dets[f]))
        if f % 3 == 0:    # announce a different buffer than the one passed next
            b = _mkey(odd.step(frames[f], f, dets[f], next_frame=wrong))
        elif f % 3 == 1:  # announce the right frame, then step on another stream
            b = _mkey(odd.step(frames[f], f, dets[f], next_frame=frames[f + 1]))
        else:
            b = _mkey(odd.step(frames[f], f, dets[f], stream=other))
        assert a == b, f"frame {f}"
        assert plain.predictions() == odd.predictions()
    torch.cuda.synchronize()
    assert plain.tracks() == odd.tracks()


@pytest.mark.parametrize("api", ["step", "ahead", "run"])
def test_tbd_early_gftt_matches_post_tracker_gftt(gpu, api):
    """The early GFTT (detections beyond the tracker's bounds filter, GFTT'd at
    the start of the step) hands new tracks exactly the corners the
    post-tracker GFTT computes, so do the early GFTTs of the guessed
    re-detection boxes (option value 2) where the tracker confirms the guess,
    and the speculative look-ahead PyrLK (launched
    before the tracker step) and the look-ahead PyrLK of the early rows (option
    tbd_early_la, re-detection frames or every frame) equal the post-tracker
    ones: same per-frame
    metrics, predictions and tracks with the options on and off, under the
    reference's bounds quirk (most new tracks served early, speculated sets
    deleted by the tracker) and with re-detection frames mixed in."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 40, 16
    frames, gt = klt.synth_render(33, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=640, bounds_ymax=360, redetect_every=4)
    res = {}
    try:
        for early, spec, ela, order, prio in ((2, 1, 1, 0, 0), (2, 1, 0, 0, 0), (2, 1, 2, 0, 0), (2, 0, 1, 0, 0),
                                              (1, 1, 1, 0, 0), (1, 1, 2, 0, 0), (1, 0, 1, 0, 0), (0, 1, 1, 0, 0),
                                              (0, 0, 0, 0, 0), (2, 1, 1, 1, 0), (2, 1, 1, 2, 0), (1, 0, 2, 2, 0),
                                              (2, 1, 1, 1, 1), (2, 1, 1, 0, 1)):
            gpu.set_option("tbd_early_gftt", early)
            gpu.set_option("tbd_spec_lookahead", spec)
            gpu.set_option("tbd_early_la", ela)
            gpu.set_option("tbd_early_order", order)  # where the step launches the early GFTT
            gpu.set_option("tbd_early_prio", prio)  # its stream's priority (read by the loop's creation)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms, preds = [], []
            if api == "run":
                ms = loop.run(frames, 0, dets)
            else:
                for f in range(F):
                    nxt = frames[f + 1] if api == "ahead" and f + 1 < F else None
                    ms.append(loop.step(frames[f], f, dets[f], next_frame=nxt))
                    preds.append(loop.predictions())
            res[early, spec, ela, order, prio] = ([_mkey(m) for m in ms], preds, loop.tracks(),
                                            sum(m.early_gftt for m in ms))
    finally:
        gpu.set_option("tbd_early_gftt", 2)
        gpu.set_option("tbd_spec_lookahead", 1)
        gpu.set_option("tbd_early_la", 1)
        gpu.set_option("tbd_early_order", 0)  # the default
        gpu.set_option("tbd_early_prio", 0)
    base = res[0, 0, 0, 0, 0]
    for key, r in res.items():
        assert r[0] == base[0], key
        assert r[1] == base[1], key
        assert r[2] == base[2], key
    assert res[1, 1, 1, 0, 0][3] > 2 * F and base[3] == 0  # the early path was taken (and off means off)
    assert res[2, 1, 1, 0, 0][3] > res[1, 1, 1, 0, 0][3] + F  # re-detection guesses confirmed
    assert res[2, 1, 1, 1, 0][3] == res[2, 1, 1, 2, 0][3] == res[2, 1, 1, 0, 0][3] == res[2, 1, 1, 1, 1][3]


def test_tbd_zero_copy_matches_copies(gpu):
    """Zero-copy staging (kernels reading the pinned tables, the fit writing to
    pinned memory) and staged copies give the same frames."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 32, 12
    frames, gt = klt.synth_render(8, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=640, bounds_ymax=360, redetect_every=3)
    res = []
    try:
        for zc in (1, 0):
            gpu.set_option("tbd_zero_copy", zc)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = loop.run(frames, 0, dets)
            res.append(([_mkey(m) for m in ms], loop.tracks()))
    finally:
        gpu.set_option("tbd_zero_copy", 1)
    assert res[0] == res[1]


def test_tbd_fit_flag_matches_event(gpu):
    """Fit completion published by the fit kernel's system-scope flag (default)
    and by an event behind the fit give the same frames; with the flag, one
    release per fit workgroup (tbd_fit_wgpub 1, the default: every wave's
    stores acknowledged before the barrier) and one per wave (0) agree too,
    with and without the look-ahead pyramid on the look-ahead stream (where
    the speculative PyrLK has no stream edge to the fit), and with
    the fit launched by the host after the look-ahead PyrLK's event (tbd_fit_gate
    1, the default) or behind a stream wait on it (0)."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 32, 12
    frames, gt = klt.synth_render(9, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=640, bounds_ymax=360, redetect_every=3)
    res = []
    try:
        for fl, wg, side, gate in ((1, 1, 2, 1), (0, 1, 2, 1), (1, 0, 2, 1), (1, 1, 0, 1), (1, 0, 0, 1),
                                   (1, 1, 2, 0), (0, 1, 2, 0), (1, 1, 0, 0)):
            gpu.set_option("tbd_fit_flag", fl)
            gpu.set_option("tbd_fit_wgpub", wg)
            gpu.set_option("tbd_la_pyr_side", side)
            gpu.set_option("tbd_fit_gate", gate)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = loop.run(frames, 0, dets)
            res.append(([_mkey(m) for m in ms], loop.tracks()))
    finally:
        gpu.set_option("tbd_fit_flag", 1)
        gpu.set_option("tbd_fit_wgpub", 1)
        gpu.set_option("tbd_la_pyr_side", 2)
        gpu.set_option("tbd_fit_gate", 1)
    for r in res[1:]:
        assert r == res[0]


def test_tbd_deferred_lookahead_matches(gpu):
    """The look-ahead PyrLK of the unchanged sets launched by the next step
    right after its critical PyrLK (ctx option tbd_la_defer), and the
    look-ahead pyramid built on the look-ahead stream (tbd_la_pyr_side), give
    the same frames as the defaults, through tbdk_tbd_run and per-frame steps
    with and without an announced next frame."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 40, 16
    frames, gt = klt.synth_render(12, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=W, bounds_ymax=H, redetect_every=4)
    res = []
    try:
        for d, side, pd in ((0, 0, 1), (1, 0, 1), (0, 1, 1), (1, 1, 1), (0, 2, 1), (1, 2, 1), (0, 2, 0)):
            gpu.set_option("tbd_la_defer", d)
            gpu.set_option("tbd_la_pyr_side", side)
            gpu.set_option("tbd_post_direct", pd)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = loop.run(frames, 0, dets)
            stepped = tbd.TbdLoop(c, ctx=gpu)
            mt = []
            for f in range(F):  # the look-ahead announced on two frames of three
                nxt = frames[f + 1] if f + 1 < F and f % 3 != 2 else None
                mt.append(_mkey(stepped.step(frames[f], f, dets[f], next_frame=nxt)))
            res.append(([_mkey(m) for m in ms], loop.tracks(), mt, stepped.tracks()))
    finally:
        gpu.set_option("tbd_la_defer", 0)
        gpu.set_option("tbd_la_pyr_side", 2)  # the default
        gpu.set_option("tbd_post_direct", 1)
    for r in res[1:]:
        assert r == res[0]
    assert res[0][0] == res[0][2]
    assert sum(m[7] for m in res[0][0]) > 0


def test_tbd_inline_kernel_args_match_tables(gpu):
    """The PyrLK segment lists, the fit table and the GFTT ROI tables carried
    in the kernel arguments (ctx options lk_seg_inline, tbd_fit_inline,
    gftt_inline; the defaults) and
    read from the staged tables give the same frames, zero-copy or not."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 40, 14
    frames, gt = klt.synth_render(10, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=640, bounds_ymax=360, redetect_every=3)
    res = []
    try:
        for seg, fit, gf, zc in ((1, 1, 1, 1), (0, 0, 0, 1), (1, 0, 1, 1), (0, 1, 0, 1), (1, 1, 1, 0)):
            gpu.set_option("lk_seg_inline", seg)
            gpu.set_option("tbd_fit_inline", fit)
            gpu.set_option("gftt_inline", gf)
            gpu.set_option("tbd_zero_copy", zc)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = loop.run(frames, 0, dets)
            res.append(([_mkey(m) for m in ms], loop.tracks()))
    finally:
        gpu.set_option("lk_seg_inline", 1)
        gpu.set_option("tbd_fit_inline", 1)
        gpu.set_option("gftt_inline", 1)
        gpu.set_option("tbd_zero_copy", 1)
    assert sum(m[0] > 0 for m in res[0][0]) > F // 2  # frames with true positives
    for r in res[1:]:
        assert r == res[0]


def test_tbd_run_host_matches_run(gpu):
    """tbdk_tbd_run_host (frames uploaded from pinned host memory through the
    three-frame device ring) gives the same frames as tbdk_tbd_run on the same
    frames resident in HBM, over two calls on one loop (the ring is reused)
    and from pageable memory too."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 32, 14
    frames, gt = klt.synth_render(12, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=640, bounds_ymax=360, redetect_every=4)
    ref = tbd.TbdLoop(c, ctx=gpu)
    want = [_mkey(m) for m in ref.run(frames, 0, dets)]
    host = frames.cpu().pin_memory()
    for src in (host, frames.cpu()):
        loop = tbd.TbdLoop(c, ctx=gpu)
        got = [_mkey(m) for m in loop.run_host(src[:9], 0, dets[:9])]
        got += [_mkey(m) for m in loop.run_host(src[9:], 9, dets[9:])]
        assert got == want
        assert loop.tracks() == ref.tracks()


def test_tbd_lookahead_then_no_tracks(gpu):
    """Detections vanish for a stretch, so a step that issued look-ahead PyrLK
    (speculative, and on re-detection frames the early rows') ends with every
    track deleted, and the next step has no tracks: it skips KLT and rebuilds
    the next pyramid over the frame that look-ahead PyrLK may still be reading
    (tbd_loop.hip, the wait on la_done in the no-KLT branch).  Then detections
    return and new tracks start.  Frames, predictions and tracks equal the
    same sequence with the look-ahead off, through run and per-step ahead."""
    from opencv_amd import klt, tbd

    W, H, N, F = 640, 480, 16, 40
    frames, gt = klt.synth_render(17, W, H, N, 0, F, ctx=gpu)
    dets = []
    for f in range(F):
        d = tbd.detections_from_gt(gt[f].numpy())
        dets.append(d[:0].copy() if 10 <= f < 26 else d)
    c = tbd.default_config(W, H, bounds_xmax=W, bounds_ymax=H, redetect_every=5)
    res = {}
    try:
        for spec, ela in ((1, 1), (1, 2), (0, 0)):
            gpu.set_option("tbd_spec_lookahead", spec)
            gpu.set_option("tbd_early_la", ela)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = [_mkey(m) for m in loop.run(frames, 0, dets)]
            ahead = tbd.TbdLoop(c, ctx=gpu)
            ma, pa = [], []
            for f in range(F):
                ma.append(_mkey(ahead.step(frames[f], f, dets[f], next_frame=frames[f + 1] if f + 1 < F else None)))
                pa.append(ahead.predictions())
            torch.cuda.synchronize()
            assert ms == ma, (spec, ela)
            assert loop.tracks() == ahead.tracks(), (spec, ela)
            res[spec, ela] = (ms, pa, loop.tracks())
    finally:
        gpu.set_option("tbd_spec_lookahead", 1)
        gpu.set_option("tbd_early_la", 1)
    base = res[0, 0]
    for key, r in res.items():
        assert r == base, key
    nt = [m[6] for m in base[0]]
    gap = [f for f in range(11, 26) if nt[f - 1] > 0 and nt[f] == 0]
    assert gap, f"no step ended with every track deleted: {nt}"  # the no-track step follows it
    assert nt[-1] > 0 and sum(m[7] for m in base[0][27:]) > 0  # tracking resumed after the gap


def test_tbd_async_launch_worker_matches(gpu):
    """The look-ahead PyrLK launches issued by the loop's launch worker thread
    (ctx option tbd_async_la, read at loop creation) and by the loop's own
    thread give the same frames, through tbdk_tbd_run and per-frame steps with
    and without an announced next frame, with and without the deferred
    look-ahead; with timing events on, the worker's launches are recorded
    beside the loop thread's (the context's timing state is shared)."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 40, 16
    frames, gt = klt.synth_render(13, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=640, bounds_ymax=360, redetect_every=4)
    res = []
    try:
        for asy, d in ((0, 0), (1, 0), (1, 1)):
            gpu.set_option("tbd_async_la", asy)
            gpu.set_option("tbd_la_defer", d)
            gpu.timing_select(["lk_sparse"])
            gpu.timing_enable(True)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = loop.run(frames, 0, dets)
            n_lk, _ = gpu.timing_query("lk_sparse")
            gpu.timing_enable(False)
            gpu.timing_select(None)
            stepped = tbd.TbdLoop(c, ctx=gpu)
            mt = []
            for f in range(F):
                nxt = frames[f + 1] if f + 1 < F and f % 3 != 2 else None
                mt.append(_mkey(stepped.step(frames[f], f, dets[f], next_frame=nxt)))
            res.append(([_mkey(m) for m in ms], loop.tracks(), mt, stepped.tracks(), n_lk))
            del loop, stepped
    finally:
        gpu.set_option("tbd_async_la", 0)
        gpu.set_option("tbd_la_defer", 0)
        gpu.timing_enable(False)
        gpu.timing_select(None)
    for r in res[1:]:
        assert r[:4] == res[0][:4]
    assert res[0][4] > F and res[1][4] == res[0][4]  # every PyrLK launch timed, the worker's included



def test_tbd_run_borrowed_level0_matches_copy(gpu):
    """tbdk_tbd_run's pyramids taking the caller's frame as level 0 (ctx option
    tbd_borrow_l0, A/B: no padded copy; PyrLK reads windows across the
    frame's edge by reflect-101 coordinates) give the same frames as the padded
    copy, including across consecutive run calls (the last frame's level 0 is
    copied into the loop's own buffer when a call ends) and a per-frame step
    after them; a small frame with many objects puts windows on every edge."""
    from opencv_amd import klt, tbd

    W, H, N, F = 320, 240, 48, 18
    frames, gt = klt.synth_render(15, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=W, bounds_ymax=H, redetect_every=4)
    res = []
    try:
        for b in (0, 1):
            gpu.set_option("tbd_borrow_l0", b)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = list(loop.run(frames[:7], 0, dets[:7]))
            ms += list(loop.run(frames[7:F - 1], 7, dets[7:F - 1]))
            ms.append(loop.step(frames[F - 1], F - 1, dets[F - 1]))
            res.append(([_mkey(m) for m in ms], loop.tracks(), sum(m.lk_points for m in ms)))
            del loop
    finally:
        gpu.set_option("tbd_borrow_l0", 0)
    assert res[0] == res[1] and res[0][2] > 0


def test_tbd_run_one_point_steps_match(gpu):
    """ctx option lk_solo (a wave's last stepping point on all its lanes) inside
    the frame loop: the same per-frame metrics (PyrLK iteration totals included)
    and tracks as without it, through tbdk_tbd_run and per-frame steps."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 40, 16
    frames, gt = klt.synth_render(29, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=640, bounds_ymax=360, redetect_every=4)
    res = []
    try:
        for solo in (0, 2, 5):
            gpu.set_option("lk_solo", solo)
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = loop.run(frames, 0, dets)
            stepped = tbd.TbdLoop(c, ctx=gpu)
            mt = [_mkey(stepped.step(frames[f], f, dets[f])) for f in range(F)]
            res.append(([_mkey(m) for m in ms], [m.lk_iters for m in ms], loop.tracks(), mt, stepped.tracks()))
            del loop, stepped
    finally:
        gpu.set_option("lk_solo", 4)
    assert sum(res[0][1]) > 0
    for r in res[1:]:
        assert r == res[0]


def test_tbd_run_gftt_ahead_matches(gpu):
    """ctx option tbd_gftt_ahead (tbdk_tbd_run launches the next frame's
    new-track GFTT one step ahead, over the caller's next frame): the same
    per-frame metrics and tracks as without it and as per-frame steps, with the
    bounds quirk (every frame starts new tracks beyond the filter), frequent
    re-detections, and a run split by a per-frame step (each run's last step
    has no next frame, so no launch is left ahead across calls)."""
    from opencv_amd import klt, tbd

    W, H, N, F = 960, 540, 40, 18
    frames, gt = klt.synth_render(41, W, H, N, 0, F, ctx=gpu)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(F)]
    c = tbd.default_config(W, H, bounds_xmax=640, bounds_ymax=360, redetect_every=3)
    res = []
    try:
        for ahead, at in ((0, 2), (1, 0), (1, 1), (1, 2)):
            gpu.set_option("tbd_gftt_ahead", ahead)
            gpu.set_option("tbd_ahead_at", at)  # where the step launches it
            loop = tbd.TbdLoop(c, ctx=gpu)
            ms = loop.run(frames, 0, dets)
            split = tbd.TbdLoop(c, ctx=gpu)
            mt = list(split.run(frames[:7], 0, dets[:7]))
            mt.append(split.step(frames[7], 7, dets[7]))
            mt += list(split.run(frames[8:], 8, dets[8:]))
            res.append(([_mkey(m) for m in ms], loop.tracks(), [_mkey(m) for m in mt], split.tracks()))
            del loop, split
    finally:
        gpu.set_option("tbd_gftt_ahead", 1)
        gpu.set_option("tbd_ahead_at", 0)
    stepped = tbd.TbdLoop(c, ctx=gpu)
    ref = [_mkey(stepped.step(frames[f], f, dets[f])) for f in range(F)]
    assert sum(k[10] for k in ref) > F  # re-detections / new tracks every frame
    for r in res:
        assert r[0] == ref and r[2] == ref
        assert r[1] == stepped.tracks() and r[3] == stepped.tracks()
