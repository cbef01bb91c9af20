"""CPU checks of the HOG oracle (oracle/hog_oracle.c).

The resize is pinned to the reference's own closed form: Resize_Bitexact.Linear8U
(imgproc/test/test_resize_bitexact.cpp:21-153) asserts INTER_LINEAR_EXACT equals
eval4's 8.8 fixed-point formula with zero difference; it is restated here and
run over the test's size table.  The HOG stages are checked by identities
(gradient magnitude / angle, L2-Hys norms, SVM score = rho + <descriptor, w>,
grouping).  Parity of the full detector against the reference binaries is
unpinned: its HOG tests read opencv_extra images."""
import numpy as np
import pytest

import _oracle as O


def _eval4_resize(src, dw, dh):
    """test_resize_bitexact.cpp:110-147 (clamped 2x2 fixed-point interpolation)."""
    h, w = src.shape[:2]
    sx, sy = 1.0 / (dw / w), 1.0 / (dh / h)

    def axis(n, sc, lim):
        f = sc * (np.arange(n) + 0.5) - 0.5
        i0 = np.floor(f).astype(np.int64)
        c1 = np.rint((f - i0) * 256).astype(np.int64)
        return np.clip(i0, 0, lim - 1), np.clip(i0 + 1, 0, lim - 1), 256 - c1, c1

    x0, x1, cx0, cx1 = axis(dw, sx, w)
    y0, y1, cy0, cy1 = axis(dh, sy, h)
    s = src.astype(np.int64)
    if s.ndim == 2:
        s = s[..., None]
    cx0, cx1 = cx0[None, :, None], cx1[None, :, None]
    top = s[y0][:, x0] * cx0 + s[y0][:, x1] * cx1
    bot = s[y1][:, x0] * cx0 + s[y1][:, x1] * cx1
    v = top * cy0[:, None, None] + bot * cy1[:, None, None]
    out = ((v + (1 << 15)) >> 16).astype(np.uint8)
    return out[..., 0] if src.ndim == 2 else out


@pytest.mark.parametrize("cn,size", [(1, (512, 768)), (3, (512, 768)), (1, (1024, 384)), (4, (1024, 384)),
                                     (1, (512, 384)), (3, (512, 384)), (4, (256, 192)), (1, (4, 3)),
                                     (3, (342, 256)), (1, (146, 110)), (3, (931, 698)), (4, (853, 640)),
                                     (1, (1004, 753)), (1, (2048, 1536)), (3, (1219, 686))])
def test_resize_exact_matches_reference_closed_form(cn, size):
    rng = np.random.default_rng(cn * 1000 + size[0])
    src = rng.integers(0, 256, (768, 1024) if cn == 1 else (768, 1024, cn), dtype=np.uint8)
    got = O.hog_resize(src, size)
    assert np.array_equal(got, _eval4_resize(src, *size))


def test_gradient_magnitude_and_bins():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (40, 53), dtype=np.uint8)
    grad, qa = O.hog_gradient(img, nbins=9, gamma=True)
    lut = np.sqrt(np.arange(256, dtype=np.float64))
    p = np.pad(lut[img], 1, mode="reflect")
    dx = p[1:-1, 2:] - p[1:-1, :-2]
    dy = p[2:, 1:-1] - p[:-2, 1:-1]
    mag = np.hypot(dx, dy)
    assert np.allclose(grad.sum(axis=2), mag, rtol=1e-5, atol=1e-5)
    ang = np.mod(np.arctan2(dy, dx), np.pi) * 9 / np.pi - 0.5   # unsigned, bins centred
    frac = ang - np.floor(ang)
    ok = (mag > 1e-3) & (np.abs(frac - 0.5) < 0.45) & (np.abs(frac) > 0.02)  # away from bin edges
    hb = np.mod(np.floor(ang).astype(int), 9)
    assert np.mean(qa[..., 0][ok] == hb[ok]) > 0.99
    assert np.array_equal(qa[..., 1], np.where(qa[..., 0] + 1 < 9, qa[..., 0] + 1, 0))


@pytest.mark.parametrize("w", [1031, 2050, 1040])
def test_gradient_form_follows_cartToPolar_chunks(w):
    """cartToPolar feeds magnitude32f/fastAtan32f 1024-element chunks of each row
    (core/src/mathfuncs.cpp:285-298); a chunk under 16 elements takes the scalar forms
    (mathfuncs_core.simd.hpp:131-138,202-207). A column keeps its form when cut out
    into a crop whose single chunk has the same length class."""
    rng = np.random.default_rng(w)
    img = rng.integers(0, 256, (6, w), dtype=np.uint8)
    g, q = O.hog_gradient(img, nbins=9, gamma=True)
    base = (w - 1) // 1024 * 1024
    tail = w - base
    # the last chunk's interior columns, computed in a crop of the same length class
    lo = base - 1
    crop = np.ascontiguousarray(img[:, lo:lo + min(tail, 15) + 1 if tail < 16 else lo + 20])
    gc, qc = O.hog_gradient(crop, nbins=9, gamma=True)
    n = crop.shape[1] - 2
    assert np.array_equal(g[1:-1, base:base + n], gc[1:-1, 1:1 + n])
    assert np.array_equal(q[1:-1, base:base + n], qc[1:-1, 1:1 + n])
    # columns of a full chunk run the 8-lane forms: equal to a 20-wide (vector) crop
    gv, _ = O.hog_gradient(np.ascontiguousarray(img[:, 500:520]), nbins=9, gamma=True)
    assert np.array_equal(g[1:-1, 501:519], gv[1:-1, 1:19])
    if tail < 16:  # and the scalar tail differs from the vector form somewhere
        gs, _ = O.hog_gradient(np.ascontiguousarray(img[:, 500:515]), nbins=9, gamma=True)
        assert not np.array_equal(gs[1:-1, 1:14], g[1:-1, 501:514])


def test_gradient_three_channels_picks_the_strongest():
    rng = np.random.default_rng(2)
    gray = rng.integers(0, 256, (24, 37), dtype=np.uint8)
    bgr = np.stack([gray // 4, gray, gray // 2], 2).astype(np.uint8)  # channel 1 dominates everywhere
    g3, q3 = O.hog_gradient(bgr)
    g1, q1 = O.hog_gradient(gray)
    assert np.array_equal(g3, g1) and np.array_equal(q3, q1)


def test_block_histograms_are_l2hys_normalized():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (64, 80), dtype=np.uint8)
    prm = O.hog_params()
    grad, qa = O.hog_gradient(img)
    B = O.hog_blocks(grad, qa, prm)
    assert B.shape == ((64 - 16) // 8 + 1, (80 - 16) // 8 + 1, 36)
    n = np.linalg.norm(B.astype(np.float64), axis=2)
    assert np.all(n <= 1.0 + 1e-6) and np.all(n > 0.95)
    assert np.all(B >= 0) and B.max() < 0.3  # clipped at 0.2, then renormalized


def test_detect_score_is_the_svm_dot_product():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (160, 96), dtype=np.uint8)
    prm = O.hog_params(win=(64, 128))
    svm = rng.standard_normal(3781).astype(np.float32) * 0.05
    xy, sc = O.hog_detect(img, prm, svm, hit_threshold=-1e9)
    nwx, nwy = (96 - 64) // 8 + 1, (160 - 128) // 8 + 1
    assert len(sc) == nwx * nwy
    grad, qa = O.hog_gradient(img)
    B = O.hog_blocks(grad, qa, prm).astype(np.float64)
    for (x, y), s in zip(xy, sc):
        desc = np.concatenate([B[y // 8 + i, x // 8 + j] for j in range(7) for i in range(15)])  # x-major
        assert abs(s - (svm[3780] + desc @ svm[:3780].astype(np.float64))) < 1e-4


def test_group_rectangles_and_clip():
    rects = np.array([[10, 10, 64, 128], [12, 11, 64, 128], [11, 9, 64, 128],   # a cluster of 3
                      [300, 40, 64, 128],                                      # alone: dropped
                      [-5, 200, 64, 128], [-4, 201, 64, 128], [-6, 199, 64, 128]], np.int32)
    w = np.array([0.5, 0.9, 0.1, 2.0, 0.3, 0.4, 0.2])
    r, wt = O.hog_group(rects, w, 2, (320, 300))
    got = sorted(zip(map(tuple, r.tolist()), wt.tolist()))
    assert got == [((0, 200, 59, 100), 0.4), ((11, 10, 64, 128), 0.9)]
    r0, _ = O.hog_group(rects, w, 0, (320, 300))  # no grouping: only clipping
    assert len(r0) == 7 and r0[4].tolist() == [0, 200, 59, 100]


def test_detect_multiscale_level0_equals_detect():
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (140, 100, 3), dtype=np.uint8)
    prm = O.hog_params()
    svm = rng.standard_normal(3781).astype(np.float32) * 0.05
    xy, sc = O.hog_detect(img, prm, svm, hit_threshold=0.0)
    r, wt = O.hog_detect_multiscale(img, prm, svm, hit_threshold=0.0, nlevels=1, group_threshold=0)
    assert np.array_equal(r[:, :2], xy) and np.array_equal(wt, sc)
