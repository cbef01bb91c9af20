"""Pin the GFTT oracle (oracle/gftt_oracle.c) against the reference test's own
independent validator, restated in numpy: test_cornerEigenValsVecs +
test_goodFeaturesToTrack of modules/imgproc/test/test_goodfeaturetotrack.cpp:68-300
(2-D Sobel filter2D, double-precision eigenvalues, same selection rules)."""
import numpy as np
import pytest

import _oracle as O
from test_oracle import np_reflect101


def ref_test_response(img, block=3, harris=False, k=0.04):
    """test_cornerEigenValsVecs (test_goodfeaturetotrack.cpp:69-159): 2-D Sobel
    filter2D, products in double, a block x block box filter (anchor block/2),
    the MINEIGENVAL or HARRIS expression in double"""
    h, w = img.shape
    ys = np_reflect101(np.arange(-1, h + 1), h)
    xs = np_reflect101(np.arange(-1, w + 1), w)
    p = img.astype(np.float64)[ys][:, xs]
    kx = np.array([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]], np.float64)
    dx = sum(kx[j, i] * p[j:j + h, i:i + w] for j in range(3) for i in range(3)).astype(np.float32)
    dy = sum(kx.T[j, i] * p[j:j + h, i:i + w] for j in range(3) for i in range(3)).astype(np.float32)
    denom = 1.0 / (((1 << 2) * block) ** 2 * 255.0)
    xv, yv = dx.astype(np.float64), dy.astype(np.float64)
    planes = [(xv * xv * denom).astype(np.float32), (xv * yv * denom).astype(np.float32),
              (yv * yv * denom).astype(np.float32)]
    anc = block // 2
    bys = np_reflect101(np.arange(-anc, h - anc + block - 1), h)
    bxs = np_reflect101(np.arange(-anc, w - anc + block - 1), w)
    boxed = []
    for q in planes:
        qp = q[bys][:, bxs].astype(np.float64)
        boxed.append(sum(qp[j:j + h, i:i + w] for j in range(block) for i in range(block)).astype(np.float32))
    a, b, c = (t.astype(np.float64) for t in boxed)
    if harris:
        return (a * c - b * b - k * (a + c) * (a + c)).astype(np.float32)
    d = np.sqrt((a - c) ** 2 + 4 * b * b)
    return (0.5 * (a + c - d)).astype(np.float32)


def ref_test_min_eig(img):
    return ref_test_response(img)


def ref_test_gftt(img, max_corners, quality, min_distance, block=3, harris=False, k=0.04):
    eig = ref_test_response(img, block, harris, k)
    thr = np.float32(eig.max() * quality)
    eig = np.where(eig > thr, eig, np.float32(0))
    h, w = eig.shape
    cands = []
    for y in range(1, h - 1):
        for x in range(1, w - 1):
            v = eig[y, x]
            if v != 0 and v == eig[y - 1:y + 2, x - 1:x + 2].max():
                cands.append((-float(v), -(y * w + x), x, y))
    cands.sort()
    out = []
    md2 = min_distance * min_distance
    for _, _, x, y in cands:
        if min_distance >= 1 and any((x - a) ** 2 + (y - b) ** 2 < md2 for a, b in out):
            continue
        out.append((x, y))
        if len(out) == max_corners:
            break
    return np.array(out, np.float32).reshape(-1, 2)


def test_min_eig_close_to_reference_validator():
    img = np.random.default_rng(5).integers(0, 256, (60, 80), dtype=np.uint8)
    got = O.min_eig(img).astype(np.float64)
    ref = ref_test_min_eig(img).astype(np.float64) / 255.0  # the test's denom omits one 255 factor
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-6 * np.abs(ref).max())


@pytest.mark.parametrize("seed,shape,maxc,md", [(0, (64, 64), 100, 0.0), (1, (96, 130), 256, 3.0),
                                                (2, (130, 90), 50, 10.0), (3, (40, 40), 1000, 1.0)])
def test_gftt_matches_reference_validator(seed, shape, maxc, md):
    fr, _ = O.synth(100 + seed, 320, 240, 6, 0, 1)
    img = fr[0][20:20 + shape[0], 30:30 + shape[1]]
    got = O.gftt(img, maxc, 0.01, md)
    ref = ref_test_gftt(img, maxc, 0.01, md)
    # same count, and (near-)identical lists: the validator's double-precision
    # eigenvalues may reorder near-ties, so compare as sets (>= 99 %, test_gftt.cpp:93-109)
    assert abs(len(got) - len(ref)) <= max(1, len(ref) // 100)
    gs = set(map(tuple, got.astype(int).tolist()))
    rs = set(map(tuple, ref.astype(int).tolist()))
    assert len(gs & rs) >= 0.99 * min(len(gs), len(rs))


def test_gftt_edge_cases():
    assert len(O.gftt(np.zeros((50, 50), np.uint8), 100, 0.01, 0)) == 0  # flat: no corners (test_gftt.cpp:112-125)
    assert len(O.gftt(np.zeros((2, 2), np.uint8), 100, 0.01, 0)) == 0
    img = np.zeros((40, 40), np.uint8)
    img[10:30, 10:30] = 200
    c = O.gftt(img, 4, 0.01, 5)
    assert len(c) == 4  # the square's four corners
    assert set(map(tuple, c.astype(int).tolist())) <= {(x, y) for x in (9, 10, 29, 30) for y in (9, 10, 29, 30)}


def test_corner_response_block3_equals_min_eig():
    fr, _ = O.synth(7, 200, 150, 5, 0, 1)
    for img in (fr[0], fr[0][3:50, 7:90], fr[0][:1, :9], fr[0][:5, :1]):
        assert np.array_equal(O.corner_response(img, 3, False), O.min_eig(img))


@pytest.mark.parametrize("block,harris", [(5, False), (7, False), (4, False), (2, False), (3, True), (5, True),
                                          (6, True)])
def test_corner_response_close_to_reference_validator(block, harris):
    """cornerMinEigenVal / cornerHarris for other block sizes against the validator
    (its denominator omits one 255 factor: eigenvalues x255, Harris x255^2)"""
    img = np.random.default_rng(block + 10 * harris).integers(0, 256, (50, 70), dtype=np.uint8)
    got = O.corner_response(img, block, harris, 0.04).astype(np.float64)
    ref = ref_test_response(img, block, harris, 0.04).astype(np.float64) / (255.0 ** (2 if harris else 1))
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())


@pytest.mark.parametrize("seed,block,harris,md", [(0, 5, False, 3.0), (1, 7, False, 0.0), (2, 4, False, 5.0),
                                                  (3, 3, True, 10.0), (4, 5, True, 3.0), (5, 3, True, 0.0)])
def test_gftt_block_harris_matches_reference_validator(seed, block, harris, md):
    """the reference test's blockSize / useHarrisDetector modes
    (test_goodfeaturetotrack.cpp:343-369: Harris with k 0.04 on test cases 2, 3)"""
    fr, _ = O.synth(200 + seed, 320, 240, 6, 0, 1)
    img = fr[0][25:25 + 110, 40:40 + 120]
    got = O.gftt_ex(img, 200, 0.01, md, block, harris, 0.04)
    ref = ref_test_gftt(img, 200, 0.01, md, block, harris, 0.04)
    assert abs(len(got) - len(ref)) <= max(1, len(ref) // 100)
    gs = set(map(tuple, got.astype(int).tolist()))
    rs = set(map(tuple, ref.astype(int).tolist()))
    assert len(gs & rs) >= 0.99 * min(len(gs), len(rs))


def test_harris_code_paths_by_flat_index():
    """calcHarris over the flattened map: AVX lines for j < N & ~7, one SSE2
    block, then the scalar double expression (corner.cpp:104-152)"""
    img = np.random.default_rng(3).integers(0, 256, (7, 9), dtype=np.uint8)  # N = 63: 56 AVX, 4 SSE2, 3 scalar
    r = O.corner_response(img, 3, True, 0.04).reshape(-1)
    assert r.shape == (63,) and np.isfinite(r).all()
