"""GPU GFTT over box ROIs vs the CPU oracle: identical corner lists (bit-exact
positions, same order, same count) per ROI."""
import numpy as np
import pytest
import torch

import _oracle as O

pytestmark = pytest.mark.gpu


def detect(gpu, frame, rois, maxc, q, md):
    from opencv_amd import klt

    det = klt.GoodFeaturesToTrackDetector(maxc, q, md)
    c, n = det.detect_rois(torch.from_numpy(np.ascontiguousarray(frame)).cuda(), rois)
    torch.cuda.synchronize()
    return c.cpu().numpy(), n.cpu().numpy()


def check(frame, rois, c, n, maxc, q, md):
    ref = O.gftt_rois(frame, rois, maxc, q, md)
    for i, r in enumerate(ref):
        assert n[i] == len(r), f"roi {i}: count {n[i]} vs {len(r)}"
        assert np.array_equal(c[i, :n[i]], r), f"roi {i}: corners differ"


@pytest.mark.parametrize("maxc,q,md", [(256, 0.01, 3.0), (1000, 0.01, 0.0), (64, 0.05, 8.0), (32, 0.3, 1.0),
                                       (33, 0.02, 5.0), (300, 0.001, 2.5), (2000, 0.001, 6.5)])
def test_gftt_rois_match_oracle(gpu, maxc, q, md):
    fr, gt = O.synth(20261015, 640, 480, 32, 0, 1)
    rois = [tuple(int(v) for v in g[1:]) for g in gt[0] if g[0]]
    c, n = detect(gpu, fr[0], rois, maxc, q, md)
    check(fr[0], rois, c, n, maxc, q, md)


def test_gftt_basketball_and_edge_rois(gpu):
    d = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "basketball_pair.npz"))
    img = d["a"]
    rois = [(0, 0, 640, 480)[:2] + (160, 120), (600, 440, 40, 40), (0, 0, 3, 3), (5, 5, 2, 50), (100, 100, 1, 1),
            (300, 200, 77, 33), (0, 0, 320, 240)]
    c, n = detect(gpu, img, rois, 500, 0.01, 2.0)
    check(img, rois, c, n, 500, 0.01, 2.0)


def test_gftt_flat_and_empty(gpu):
    img = np.full((100, 100), 77, np.uint8)
    c, n = detect(gpu, img, [(0, 0, 100, 100), (10, 10, 20, 20)], 100, 0.01, 0.0)
    assert (n == 0).all()
    c, n = detect(gpu, img, [], 100, 0.01, 0.0)
    assert n.shape == (0,)


def test_gftt_1080p_128_boxes(gpu):
    fr, gt = O.synth(20261015, 1920, 1080, 128, 0, 1)
    rois = [tuple(int(v) for v in g[1:]) for g in gt[0] if g[0]]
    c, n = detect(gpu, fr[0], rois, 256, 0.01, 3.0)
    check(fr[0], rois, c, n, 256, 0.01, 3.0)
    assert (n > 0).all()


@pytest.mark.parametrize("inline", [1, 0])
def test_gftt_roi_table_in_args_or_memory(gpu, inline):
    """The ROI table carried in the kernel arguments (ctx option gftt_inline,
    up to 128 ROIs) and read from device memory (the option off, or more ROIs
    than the arguments hold) give the oracle's corner lists."""
    fr, gt = O.synth(20261016, 1920, 1080, 128, 0, 1)
    boxes = [tuple(int(v) for v in g[1:]) for g in gt[0] if g[0]]
    halves = [(x, y, max(w // 2, 3), max(h // 2, 3)) for x, y, w, h in boxes]
    gpu.set_option("gftt_inline", inline)
    try:
        for rois in (boxes[:128], (boxes + halves)[:200]):
            c, n = detect(gpu, fr[0], rois, 128, 0.01, 3.0)
            check(fr[0], rois, c, n, 128, 0.01, 3.0)
            assert (n > 0).sum() > len(rois) // 2
    finally:
        gpu.set_option("gftt_inline", 1)


@pytest.mark.parametrize("shape", [(480, 640), (37, 61), (3, 3), (1, 7), (9, 1), (1080, 1920), (130, 121),
                                   (17, 200), (33, 58), (34, 59), (33, 56), (34, 57), (2, 2)])
@pytest.mark.parametrize("redo", [0, 1])
def test_corner_min_eig_matches_oracle(gpu, shape, redo):
    """cornerMinEigenVal map (the GFTT eigenvalue kernel over one full-image
    ROI, strips of 56 columns) bit-exact with the oracle, on the concurrent
    segment walk and with a fresh-start mismatch forced at every segment
    boundary (option gftt_eig_redo: the drift-corrected re-walk rounds)."""
    from opencv_amd import klt

    h, w = shape
    if h >= 200:
        fr, _ = O.synth(77, w, h, 12, 0, 1)
        img = np.ascontiguousarray(fr[0])
    else:
        img = np.random.default_rng(h * 1000 + w).integers(0, 256, (h, w), dtype=np.uint8)
    gpu.set_option("gftt_eig_redo", redo)
    try:
        got = klt.corner_min_eigen_val(torch.from_numpy(img).cuda(), ctx=gpu).cpu().numpy()
    finally:
        gpu.set_option("gftt_eig_redo", 0)
    ref = O.min_eig(img)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_gftt_bench_frames_many_rois(gpu):
    """GFTT over the bench's 1080p frames and boxes (several frames: the
    box-filter double rounding that makes the running sum history-dependent
    occurs in a fraction of strips) equals the oracle."""
    fr, gt = O.synth(20261015, 1920, 1080, 128, 0, 12)
    for t in range(0, 12, 3):
        rois = []
        for g in gt[t]:
            if not g[0]:
                continue
            x, y, w, h = (int(v) for v in g[1:])
            x0, y0, x1, y1 = max(x, 0), max(y, 0), min(x + w, 1920), min(y + h, 1080)
            if x1 - x0 >= 3 and y1 - y0 >= 3:
                rois.append((x0, y0, x1 - x0, y1 - y0))
        c, n = detect(gpu, fr[t], rois, 256, 0.01, 3.0)
        check(fr[t], rois, c, n, 256, 0.01, 3.0)


@pytest.mark.parametrize("maxc,q,md", [(256, 0.01, 3.0), (300, 0.001, 2.5)])
def test_gftt_rois_forced_rewalk(gpu, maxc, q, md):
    """GFTT results with a fresh-start mismatch forced at every eigenvalue
    segment boundary (the cold re-walk rounds) equal the oracle's."""
    fr, gt = O.synth(31, 1280, 720, 40, 0, 1)
    rois = []
    for x, y, w, h in (tuple(int(v) for v in g[1:]) for g in gt[0] if g[0]):
        x0, y0, x1, y1 = max(x, 0), max(y, 0), min(x + w, 1280), min(y + h, 720)
        if x1 - x0 >= 3 and y1 - y0 >= 3:
            rois.append((x0, y0, x1 - x0, y1 - y0))
    gpu.set_option("gftt_eig_redo", 1)
    try:
        c, n = detect(gpu, fr[0], rois, maxc, q, md)
    finally:
        gpu.set_option("gftt_eig_redo", 0)
    check(fr[0], rois, c, n, maxc, q, md)


@pytest.mark.parametrize("maxc,md", [(5000, 1.5), (700, 4.0), (3000, 0.0)])
def test_gftt_large_candidate_sets(gpu, maxc, md):
    """ROIs with thousands of candidates (noise texture, a flat band of ties):
    multi-thousand-key sorts and long greedy walks give the oracle's corner
    lists exactly."""
    rng = np.random.default_rng(123)
    img = rng.integers(0, 256, (300, 400), dtype=np.uint8)
    img[100:140, 50:300] = 77  # flat band: ties and empty regions
    rois = [(0, 0, 200, 150), (10, 20, 150, 120), (200, 100, 180, 190)]
    c, n = detect(gpu, img, rois, maxc, 0.001, md)
    assert (n > 0).all()
    check(img, rois, c, n, maxc, 0.001, md)


MODES = [(5, False, 0.04), (7, False, 0.04), (4, False, 0.04), (2, False, 0.04), (1, False, 0.04),
         (3, True, 0.04), (5, True, 0.06), (6, True, 0.04), (11, True, 0.04)]


@pytest.mark.parametrize("block,harris,k", MODES)
@pytest.mark.parametrize("shape", [(37, 61), (3, 3), (1, 7), (9, 1), (130, 121), (2, 2), (480, 640)])
def test_corner_response_matches_oracle(gpu, shape, block, harris, k):
    """cornerMinEigenVal / cornerHarris for blockSize != 3 and the Harris response
    (klt_gftt_resp.hip) bit-exact with the oracle, including the calcHarris code
    path split by flat index (AVX lines, one SSE2 block, scalar tail)"""
    from opencv_amd import klt

    h, w = shape
    img = np.random.default_rng(h * 1000 + w + block).integers(0, 256, (h, w), dtype=np.uint8)
    got = klt.corner_response(torch.from_numpy(img).cuda(), block, harris, k, ctx=gpu).cpu().numpy()
    ref = O.corner_response(img, block, harris, k)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("block,harris,k", MODES)
def test_gftt_block_harris_rois_match_oracle(gpu, block, harris, k):
    """createGoodFeaturesToTrackDetector(blockSize, useHarrisDetector, harrisK)
    over box ROIs: the corner lists equal the oracle's"""
    from opencv_amd import klt

    fr, gt = O.synth(20261015 + block, 640, 480, 32, 0, 1)
    rois = [tuple(int(v) for v in g[1:]) for g in gt[0] if g[0]] + [(0, 0, 3, 3), (5, 5, 2, 50), (600, 440, 40, 40)]
    for maxc, q, md in ((256, 0.01, 3.0), (1000, 0.001, 0.0)):
        det = klt.GoodFeaturesToTrackDetector(maxc, q, md, block, harris, k)
        c, n = det.detect_rois(torch.from_numpy(np.ascontiguousarray(fr[0])).cuda(), rois)
        torch.cuda.synchronize()
        c, n = c.cpu().numpy(), n.cpu().numpy()
        ref = O.gftt_rois(fr[0], rois, maxc, q, md, block, harris, k)
        for i, r in enumerate(ref):
            assert n[i] == len(r), f"roi {i}: count {n[i]} vs {len(r)}"
            assert np.array_equal(c[i, :n[i]], r), f"roi {i}: corners differ"


def test_gftt_params_rejected(gpu):
    from opencv_amd import klt, _lib

    img = torch.zeros((20, 20), dtype=torch.uint8, device="cuda")
    for kw in ({"blockSize": 0}, {"blockSize": 64}, {"harrisK": float("nan")}):
        with pytest.raises(_lib.TbdkError):
            klt.GoodFeaturesToTrackDetector(10, 0.01, 0.0, **kw).detect_rois(img, [(0, 0, 20, 20)])


@pytest.mark.parametrize("compact", [0, 1])
@pytest.mark.parametrize("maxc,q,md", [(256, 0.01, 3.0), (500, 0.001, 0.0), (64, 1.0, 2.0), (40, 1.5, 1.0)])
def test_gftt_compact_and_dense_candidates(gpu, compact, maxc, q, md):
    """GFTT with the eigenvalue plane (ctx option gftt_compact = 0) and with
    only its local maxima's values written (1, the default; used for quality
    <= 1, the dense plane above it): the same corner lists as the oracle,
    including the basketball frame's edge and degenerate ROIs and quality 1
    (the bound of the compact mode's no-candidate rule for ROIs whose max <= 0)."""
    d = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "basketball_pair.npz"))
    img = d["a"]
    rois = [(0, 0, 160, 120), (600, 440, 40, 40), (0, 0, 3, 3), (5, 5, 2, 50), (300, 200, 77, 33), (0, 0, 640, 480),
            (250, 250, 57, 121), (10, 400, 113, 80)]
    gpu.set_option("gftt_compact", compact)
    try:
        c, n = detect(gpu, img, rois, maxc, q, md)
    finally:
        gpu.set_option("gftt_compact", 1)
    check(img, rois, c, n, maxc, q, md)
