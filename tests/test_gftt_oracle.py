"""Pin the GFTT oracle (oracle/gftt_oracle.c) against the reference test's own
independent validator, restated in numpy: test_cornerEigenValsVecs +
test_goodFeaturesToTrack of modules/imgproc/test/test_goodfeaturetotrack.cpp:68-300
(2-D Sobel filter2D, double-precision eigenvalues, same selection rules)."""
import numpy as np
import pytest

import _oracle as O
from test_oracle import np_reflect101


def ref_test_min_eig(img):
    h, w = img.shape
    ys = np_reflect101(np.arange(-1, h + 1), h)
    xs = np_reflect101(np.arange(-1, w + 1), w)
    p = img.astype(np.float64)[ys][:, xs]
    kx = np.array([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]], np.float64)
    dx = sum(kx[j, i] * p[j:j + h, i:i + w] for j in range(3) for i in range(3)).astype(np.float32)
    dy = sum(kx.T[j, i] * p[j:j + h, i:i + w] for j in range(3) for i in range(3)).astype(np.float32)
    denom = 1.0 / (((1 << 2) * 3) ** 2 * 255.0)
    xv, yv = dx.astype(np.float64), dy.astype(np.float64)
    planes = [(xv * xv * denom).astype(np.float32), (xv * yv * denom).astype(np.float32),
              (yv * yv * denom).astype(np.float32)]
    boxed = []
    for q in planes:
        qp = q[ys][:, xs].astype(np.float64)
        boxed.append(sum(qp[j:j + h, i:i + w] for j in range(3) for i in range(3)).astype(np.float32))
    a, b, c = (t.astype(np.float64) for t in boxed)
    d = np.sqrt((a - c) ** 2 + 4 * b * b)
    return (0.5 * (a + c - d)).astype(np.float32)


def ref_test_gftt(img, max_corners, quality, min_distance):
    eig = ref_test_min_eig(img)
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
