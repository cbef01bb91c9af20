"""End-to-end parity of the native TBD loop at the bench's own configurations.

libtbdk's loop (tbdk_tbd_run, and tbdk_tbd_step_ahead frame by frame, which
runs the same code with the same look-ahead) against an INDEPENDENT oracle
pipeline, oracle/tbd_loop_oracle.py: O.Pyramid -> O.gftt_rois (256/box, q
0.01, minDist 3, every 5 frames or < 32 points) -> O.lk -> box_fit_oracle
(getRTMatrix + cv::solve(DECOMP_EIG)) -> tbd_oracle.Tracker, driving itself
with its own predictions (samples/gpu/tbd.cpp:624-706, tbd.cpp:288-304).
Nothing of the GPU's output feeds the oracle.

Per frame:
  * KLT predictions: the same tracks predicted, centres within 1e-4 px (the
    fit's closed-form vs eigen-solve tolerance, tests/test_gpu_box_fit.py);
  * every track's id, box, predPosition (the rounded Rect), age, visible
    count and corner count: exact;
  * TP / FN / FP / GT, tracks, PyrLK points entered and tracked, predicted
    tracks, refreshed sets: exact (PyrLK in the oracle's exact-sum mode, the
    GPU's accumulation, bit-exact per point, tests/test_gpu_klt.py);
and tbdk_tbd_run's per-frame metrics equal the frame-by-frame ones.

Configurations: BASELINE configs[2] (1920x1080, 128 objects, the reference's
hard-coded 1280x720 bounds filter) and configs[3] (KITTI 1242x375, its 8
sequences seeds s..s+7).  16 / 12 frames cover three / two re-detection
frames (0, 5, 10, 15)."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tbd_loop_oracle as L  # noqa: E402

pytestmark = pytest.mark.gpu

SEED = 20261015
METRIC_KEYS = ("tp", "fn", "fp", "gt", "ntracks", "lk_points", "klt_points", "klt_predicted", "redetected")


def _gpu_rows(tracks):
    return [(t["id"], t["x"], t["y"], t["width"], t["height"], t["pred_x"], t["pred_y"], t["pred_w"],
             t["pred_h"], t["age"], t["total_visible"], t["npoints"]) for t in tracks]


def run_pair(gpu, W, H, N, F, seed, drop=0.0):
    from opencv_amd import klt, tbd

    frames, gt = klt.synth_render(seed, W, H, N, 0, F, ctx=gpu)
    ofr, ogt = L.O.synth(seed, W, H, N, 0, F)  # the oracle's own rendering of the sequence
    assert np.array_equal(frames.cpu().numpy(), ofr) and np.array_equal(gt.numpy(), ogt)
    rng = np.random.default_rng(seed)
    keep = [rng.random(N) >= drop for _ in range(F)]
    dets = []
    for f in range(F):
        d = tbd.detections_from_gt(ogt[f])
        dets.append(np.ascontiguousarray(d[keep[f][d["id"]]]))

    cfg = tbd.default_config(W, H)  # reference bounds (0, 1280, 0, 720), the bench's options
    loop = tbd.TbdLoop(cfg, ctx=gpu)
    ora = L.KltTbdLoop(W, H, nthreads=min(16, os.cpu_count() or 1))
    gms = []
    stats = {"pred_err": 0.0, "preds": 0, "refreshed": 0, "lost": 0}
    for f in range(F):
        m = loop.step(frames[f], f, dets[f], next_frame=frames[f + 1] if f + 1 < F else None)
        om = ora.step(ofr[f], f, L.detections(ogt[f], f, keep[f]))
        gm = {k: getattr(m, k) for k in METRIC_KEYS}
        gms.append(gm)
        assert gm == om, f"frame {f}: metrics {gm} vs oracle {om}"
        gp, op = loop.predictions(), ora.preds
        assert gp.keys() == op.keys(), f"frame {f}: predicted tracks differ"
        for k, (cx, cy) in gp.items():
            e = max(abs(cx - op[k][0]), abs(cy - op[k][1]))
            assert e <= 1e-4, f"frame {f} track {k}: centre {cx, cy} vs {op[k]}"
            stats["pred_err"] = max(stats["pred_err"], e)
        stats["preds"] += len(gp)
        stats["refreshed"] += om["redetected"]
        stats["lost"] += om["lk_points"] - om["klt_points"]
        assert _gpu_rows(loop.tracks()) == ora.track_rows(), f"frame {f}: tracks differ"
    # the native frame loop (tbdk_tbd_run) over the same frames: the same frames out
    batch = tbd.TbdLoop(cfg, ctx=gpu)
    ms = batch.run([frames[f] for f in range(F)], 0, dets)
    assert [{k: getattr(m, k) for k in METRIC_KEYS} for m in ms] == gms
    assert _gpu_rows(batch.tracks()) == ora.track_rows()
    torch.cuda.synchronize()
    return stats


@pytest.mark.parametrize("seed,drop", [(SEED, 0.0), (SEED + 1, 0.1)])
def test_tbd_loop_equals_oracle_pipeline_1080p_128(gpu, seed, drop):
    """BASELINE configs[2]: 1920x1080 x 128 objects, 16 frames (re-detection at 0, 5, 10, 15)."""
    s = run_pair(gpu, 1920, 1080, 128, 16, seed, drop)
    assert s["preds"] > 15 * 100  # the KLT motion model drove the tracker
    assert s["refreshed"] > 3 * 128


@pytest.mark.parametrize("k", range(8))
def test_tbd_loop_equals_oracle_pipeline_kitti(gpu, k):
    """BASELINE configs[3]: the KITTI-shaped 1242x375 sequences s..s+7, 128 objects (one per GPU in the bench)."""
    s = run_pair(gpu, 1242, 375, 128, 12, SEED + k)
    assert s["preds"] > 0


def test_tbd_loop_equals_oracle_pipeline_1080p_long(gpu):
    """configs[2] over 64 frames (13 re-detection frames, 5 % of the detections
    dropped at random): tracks born, coasting, deleted and re-created many times
    over, still frame-by-frame equal to the oracle pipeline"""
    s = run_pair(gpu, 1920, 1080, 128, 64, SEED + 7, 0.05)
    assert s["preds"] > 63 * 100
    assert s["refreshed"] > 13 * 100
