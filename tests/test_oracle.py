"""Pin the CPU oracle (oracle/klt_oracle.c) before trusting it.

The reference cannot be built here and its golden data (opencv_extra) is not
vendored, so the oracle is checked against:
  * the reference's in-tree known-answer test      test_filter.cpp:2298-2304
  * the reference tests' own independent validators, restated in numpy:
      pyrDown  vs filter2D(kernel/256, REFLECT_101) + decimation, tol 1
               (test_filter.cpp:1085-1204)
      Scharr   vs cv::Scharr's separable [3 10 3] x [-1 0 1] definition
  * the reference's LK acceptance criteria on inputs with known motion
      (video/test/test_optflowpyrlk.cpp:60-228: no lost points, tiny error)
  * the reference's own image fixtures samples/data/basketball{1,2}.png.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import _oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_DATA = "/root/reference/samples/data"


def np_reflect101(idx, n):
    idx = np.asarray(idx)
    out = idx.copy()
    for _ in range(4):
        out = np.where(out < 0, -out, out)
        out = np.where(out >= n, 2 * n - 2 - out, out)
    return out


def np_pyrdown_validator(src):
    """CV_PyramidDownTest::prepare_to_validation (test_filter.cpp:1180-1204):
    cvtest::filter2D with the [1 4 6 4 1]^2/256 kernel, REFLECT_101, then every
    second pixel; float math, saturate_cast rounding."""
    h, w = src.shape
    k1 = np.array([1, 4, 6, 4, 1], np.float64)
    K = np.outer(k1, k1) / 256.0
    ys = np_reflect101(np.arange(-2, h + 2), h)
    xs = np_reflect101(np.arange(-2, w + 2), w)
    p = src.astype(np.float64)[ys][:, xs]
    acc = np.zeros((h, w))
    for j in range(5):
        for i in range(5):
            acc += K[j, i] * p[j:j + h, i:i + w]
    full = np.clip(np.rint(acc), 0, 255)
    dh, dw = (h + 1) // 2, (w + 1) // 2
    return full[0:2 * dh:2, 0:2 * dw:2][:dh, :dw].astype(np.uint8)


def np_pyrdown_exact(src):
    """Integer restatement (sum of [1 4 6 4 1]^2 products, (s+128)>>8)."""
    h, w = src.shape
    dh, dw = (h + 1) // 2, (w + 1) // 2
    k1 = np.array([1, 4, 6, 4, 1], np.int64)
    ys = np_reflect101(np.arange(-2, 2 * dh + 2), h)
    xs = np_reflect101(np.arange(-2, 2 * dw + 2), w)
    p = src.astype(np.int64)[ys][:, xs]
    acc = np.zeros((dh, dw), np.int64)
    for j in range(5):
        for i in range(5):
            acc += k1[j] * k1[i] * p[j:j + 2 * dh:2, i:i + 2 * dw:2]
    return ((acc + 128) >> 8).astype(np.uint8)


def test_pyrdown_known_answer_issue_12961():
    # TEST(Imgproc_Pyrdown, issue_12961): 9x9 zeros -> all-zero result
    out = O.pyr_down(np.zeros((9, 9), np.uint8))
    assert out.shape == (5, 5) and not out.any()


@pytest.mark.parametrize("shape", [(9, 9), (31, 17), (64, 64), (113, 128), (480, 640), (375, 1242)])
def test_pyrdown_matches_reference_validator(shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    got = O.pyr_down(img)
    ref = np_pyrdown_validator(img)
    assert got.shape == ref.shape
    assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1  # get_success_error_level: 1 for 8U
    assert np.array_equal(got, np_pyrdown_exact(img))


def test_pyramid_levels_and_borders():
    img = O.read_png_gray(os.path.join(REF_DATA, "basketball1.png")) if os.path.exists(REF_DATA) else \
        np.random.default_rng(0).integers(0, 256, (480, 640), dtype=np.uint8)
    P = O.Pyramid(img, (21, 21), 3)
    assert P.nlevels == 4  # 640x480 -> 320x240 -> 160x120 -> 80x60 (stop rule lkpyramid.cpp:782)
    cur = img
    for lvl in range(P.nlevels):
        got = P.level(lvl)
        assert np.array_equal(got, cur)
        full = P.level(lvl, with_border=True)
        pad = P.p.lv[lvl].pad
        ys = np_reflect101(np.arange(-pad, cur.shape[0] + pad), cur.shape[0])
        xs = np_reflect101(np.arange(-pad, cur.shape[1] + pad), cur.shape[1])
        assert np.array_equal(full, cur[ys][:, xs])
        cur = np_pyrdown_exact(cur)


def test_pyramid_stop_rule_small_images():
    # sizes <= winSize stop the pyramid (lkpyramid.cpp:782-787)
    P = O.Pyramid(np.zeros((50, 90), np.uint8), (21, 21), 5)
    assert P.nlevels == 2  # 90x50 -> 45x25 -> (23x13 stops)


def np_scharr(img):
    """cv::Scharr dx / dy of calcSharrDeriv: [3 10 3] smoothing x [-1 0 1], REFLECT_101."""
    h, w = img.shape
    ys = np_reflect101(np.arange(-1, h + 1), h)
    xs = np_reflect101(np.arange(-1, w + 1), w)
    p = img.astype(np.int32)[ys][:, xs]
    sm_v = 3 * (p[:-2] + p[2:]) + 10 * p[1:-1]          # vertical smoothing, (h, w+2)
    dv = p[2:] - p[:-2]                                  # vertical difference
    ix = sm_v[:, 2:] - sm_v[:, :-2]
    iy = 3 * (dv[:, 2:] + dv[:, :-2]) + 10 * dv[:, 1:-1]
    return np.stack([ix, iy], -1).astype(np.int16)


@pytest.mark.parametrize("shape", [(1, 1), (2, 7), (23, 31), (120, 160)])
def test_scharr_matches_definition(shape):
    img = np.random.default_rng(7).integers(0, 256, shape, dtype=np.uint8)
    got = O.scharr(img)
    if shape[0] > 1 and shape[1] > 1:
        assert np.array_equal(got, np_scharr(img))
    else:
        assert got.shape == (shape[0], shape[1], 2)


def shifted_pair(img, dx, dy):
    """next(x, y) = prev(x - dx, y - dy): integer shift, crop away the wrap."""
    b = np.roll(np.roll(img, dx, axis=1), dy, axis=0)
    m = 24
    return img[m:-m, m:-m].copy(), b[m:-m, m:-m].copy()


def grid_points(h, w, step, margin):
    ys, xs = np.mgrid[margin:h - margin:step, margin:w - margin:step]
    return np.stack([xs.ravel(), ys.ravel()], 1).astype(np.float32)


@pytest.mark.parametrize("accum", [O.ACCUM_SSE2, O.ACCUM_EXACT])
def test_lk_recovers_known_translation(accum):
    # the acceptance rule of Video_OpticalFlowPyrLK.accuracy (test_optflowpyrlk.cpp:140-225):
    # no lost points, at most a handful of points off by > 0.3 px, max error <= 1
    img = O.read_png_gray(os.path.join(REF_DATA, "basketball1.png"))
    a, b = shifted_pair(img, 5, -3)
    pts = grid_points(a.shape[0], a.shape[1], 16, 40)
    nx, st, err, it = O.lk(O.Pyramid(a), O.Pyramid(b), pts, accum=accum)
    e = np.abs(nx - (pts + np.float32([5, -3]))).max(1)
    textured = err < 10  # flat-region points may legitimately drift; reference counts them via its own fixture
    assert st.all()
    assert (e[textured] > 0.3).sum() <= 8
    assert np.isfinite(nx).all()


def test_lk_sse2_vs_exact_accumulation_close():
    fr, _ = O.synth(20261015, 640, 480, 32, 0, 2)
    pts = grid_points(480, 640, 8, 4)
    a = O.lk(O.Pyramid(fr[0]), O.Pyramid(fr[1]), pts, accum=O.ACCUM_SSE2)
    b = O.lk(O.Pyramid(fr[0]), O.Pyramid(fr[1]), pts, accum=O.ACCUM_EXACT)
    ok = (a[1] == 1) & (b[1] == 1)
    assert (a[1] == b[1]).mean() >= 0.995
    d = np.abs(a[0] - b[0]).max(1)[ok]
    assert (d <= 1e-2).mean() >= 0.995


def test_lk_gate_margins_and_threshold_clause():
    """orc_lk_gate's margins (every status disagreement between
    the two accumulation orders must lie within 1e-3 relative of a minEig /
    bounds threshold).  A point whose minEig IS the threshold has margin 0; a
    point far inside the frame with a strong texture has a large one; a point
    whose window walks off the frame has its bounds margin; over 1080p points
    every SSE2-vs-exact status disagreement sits at a threshold, including when
    the threshold is placed at the points' own minimum eigenvalues."""
    fr, _ = O.synth(20261015, 640, 480, 32, 0, 2)
    P0, P1 = O.Pyramid(fr[0], (21, 21), 0), O.Pyramid(fr[1], (21, 21), 0)
    pts = grid_points(480, 640, 16, 40)
    _, _, me, _ = O.lk(P0, P1, pts, max_level=0, flags=8, accum=O.ACCUM_EXACT)  # level-0 minEig per point
    i = int(np.argsort(me)[len(me) // 2])
    g = np.empty(len(pts), np.float32)
    _, st, _, _ = O.lk(P0, P1, pts, max_level=0, min_eig=float(me[i]), accum=O.ACCUM_EXACT, want_err=False, gate=g)
    assert g[i] == 0.0 and st[i] == 1  # minEig == threshold passes (the gate is minEig < threshold)
    assert (g[me > 2 * me[i]] > 0.01).all()  # 40 px inside the frame, minEig far from the threshold
    # window origins (point - 10) just inside x >= -21, at x == cols, just inside y < rows
    edge = np.float32([[-10.99, 100.0], [650.0, 200.0], [320.0, 489.995]])
    ge = np.empty(3, np.float32)
    _, st, _, _ = O.lk(P0, P1, edge, max_level=0, accum=O.ACCUM_EXACT, want_err=False, gate=ge)
    assert st[1] == 0 and ge[1] == 0.0 and (ge <= 1e-3).all()
    # the clause itself, at the 1080p loop's shape and with thresholds put among the points' minEig values
    fr, _ = O.synth(20261015, 1920, 1080, 128, 0, 2)
    A, B = O.Pyramid(fr[0], (21, 21), 2), O.Pyramid(fr[1], (21, 21), 2)
    rng = np.random.default_rng(1)
    pts = np.stack([rng.uniform(0, 1920, 8192), rng.uniform(0, 1080, 8192)], 1).astype(np.float32)
    _, _, me, _ = O.lk(A, B, pts, max_level=0, flags=8, accum=O.ACCUM_EXACT)
    for thr in (1e-4, float(np.quantile(me, 0.3)), float(np.quantile(me, 0.5))):
        ga, gb = np.empty(len(pts), np.float32), np.empty(len(pts), np.float32)
        a = O.lk(A, B, pts, max_level=2, min_eig=thr, accum=O.ACCUM_EXACT, want_err=False, gate=ga)
        b = O.lk(A, B, pts, max_level=2, min_eig=thr, accum=O.ACCUM_SSE2, want_err=False, gate=gb)
        dis = a[1] != b[1]
        assert dis.mean() <= 0.005
        assert (np.minimum(ga, gb)[dis] <= 1e-3).all()


def test_lk_edge_cases():
    fr, _ = O.synth(5, 160, 120, 4, 0, 2)
    P0, P1 = O.Pyramid(fr[0]), O.Pyramid(fr[1])
    pts = np.array([[-100, -100], [1e4, 5], [0, 0], [159.9, 119.9], [80.25, 60.75], [-21.0, 50.0]], np.float32)
    nx, st, err, it = O.lk(P0, P1, pts)
    assert st[0] == 0 and st[1] == 0 and err[0] == 0 and err[1] == 0
    # empty input
    nx, st, err, it = O.lk(P0, P1, np.zeros((0, 2), np.float32))
    assert nx.shape == (0, 2)
    # get-min-eigenvalues mode returns the eigenvalue in err
    nx, st, err, it = O.lk(P0, P1, pts[2:], flags=8)
    assert (err >= 0).all()


def test_synth_is_deterministic_and_pinned():
    fr, gt = O.synth(20261015, 640, 480, 32, 0, 3)
    fr2, gt2 = O.synth(20261015, 640, 480, 32, 0, 3)
    assert np.array_equal(fr, fr2) and np.array_equal(gt, gt2)
    golden = json.load(open(os.path.join(GOLDEN, "synth_hashes.json")))
    for f in range(3):
        assert hashlib.sha256(fr[f].tobytes()).hexdigest() == golden["640x480x32"][f]
    assert hashlib.sha256(gt.tobytes()).hexdigest() == golden["640x480x32_gt"]


# ---- the fp16 pixel path's oracle (oracle/klt16_oracle.c) ----------------------

def _h16():
    import ctypes as C

    lib = O._lib16()
    lib.orc16_f2h.restype = C.c_uint16
    lib.orc16_f2h.argtypes = [C.c_float]
    lib.orc16_h2f.restype = C.c_float
    lib.orc16_h2f.argtypes = [C.c_uint16]
    return lib


def test_f16_conversions_match_numpy():
    """binary16 <-> binary32 (round to nearest even) against numpy's float16:
    every half value, edge values, random floats over the whole range"""
    lib = _h16()
    h = np.arange(65536, dtype=np.uint16)
    ref = h.view(np.float16).astype(np.float32)
    got = np.array([lib.orc16_h2f(int(v)) for v in h], dtype=np.float32)
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan) and np.array_equal(got[~nan].view(np.uint32), ref[~nan].view(np.uint32))
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(20000) * np.exp(rng.uniform(-20, 11, 20000))).astype(np.float32)
    x = np.concatenate([x, np.float32([0, -0.0, 2 ** -24, 2 ** -25, 1.5 * 2 ** -25, 6.1e-5, 65504, 65519, 65520,
                                       1e9, -1e9, 0.1, 1 / 3, 255.0])])
    with np.errstate(over="ignore"):
        ref = x.astype(np.float16).view(np.uint16)
    got = np.array([lib.orc16_f2h(float(v)) for v in x], dtype=np.uint16)
    assert np.array_equal(got, ref)


def test_f16_pyr_down_and_scharr_definitions():
    """the fp16 pyrDown / Scharr against a numpy statement of the same fp32
    expression order (reflect-101 borders), rounded to float16"""
    rng = np.random.default_rng(4)
    img = (rng.uniform(0, 255, (37, 53)) + rng.uniform(0, 1, (37, 53))).astype(np.float16)
    f = img.astype(np.float32)
    h, w = f.shape
    ry = lambda y: O.load().orc_reflect101(y, h)  # noqa: E731
    rx = lambda x: O.load().orc_reflect101(x, w)  # noqa: E731
    dh, dw = (h + 1) // 2, (w + 1) // 2
    ref = np.empty((dh, dw), np.float16)
    for y in range(dh):
        for x in range(dw):
            r = []
            for j in range(5):
                row = f[ry(2 * y + j - 2)]
                s = [row[rx(2 * x + k - 2)] for k in range(5)]
                r.append(np.float32(np.float32(np.float32(np.float32(s[2] * np.float32(6)) +
                                                          np.float32(np.float32(s[1] + s[3]) * np.float32(4))) + s[0]) + s[4]))
            v = np.float32(np.float32(np.float32(np.float32(r[2] * np.float32(6)) +
                                                 np.float32(np.float32(r[1] + r[3]) * np.float32(4))) + r[0]) + r[4])
            ref[y, x] = np.float16(np.float32(v * np.float32(1 / 256)))
    assert np.array_equal(O.pyr_down16(img).view(np.uint16), ref.view(np.uint16))
    d = O.scharr16(img)
    y, x = 7, 11
    t0 = [np.float32(np.float32((f[y - 1, c] + f[y + 1, c]) * np.float32(3)) + np.float32(f[y, c] * np.float32(10)))
          for c in (x - 1, x, x + 1)]
    t1 = [np.float32(f[y + 1, c] - f[y - 1, c]) for c in (x - 1, x, x + 1)]
    assert d[y, x, 0] == np.float16(np.float32(t0[2] - t0[0]))
    assert d[y, x, 1] == np.float16(np.float32(np.float32(np.float32(t1[2] + t1[0]) * np.float32(3)) +
                                               np.float32(t1[1] * np.float32(10))))


def test_f16_lk_recovers_translation_and_tracks_u8_path():
    """the fp16 LK on a known translation, and against the 8-bit path on the
    same synthetic frames (different arithmetic: a sanity bound, not parity)"""
    frames, gt = O.synth(20261015, 320, 240, 12, 0, 2)
    rng = np.random.default_rng(0)
    pts = np.concatenate([np.stack([rng.uniform(x, x + bw, 24), rng.uniform(y, y + bh, 24)], 1)
                          for v, x, y, bw, bh in gt[0] if v]).astype(np.float32)
    nx, st, _, _ = O.lk(O.Pyramid(frames[0]), O.Pyramid(frames[1]), pts, accum=O.ACCUM_EXACT)
    nx16, st16, err16, _ = O.lk16(O.Pyramid16(frames[0]), O.Pyramid16(frames[1]), pts)
    both = (st == 1) & (st16 == 1)
    assert both.mean() > 0.9 and (st == st16).mean() > 0.99
    assert (np.abs(nx - nx16)[both].max(1) <= 1e-2).mean() >= 0.99
    # integer translation of a blurred noise image: recovered exactly enough
    img = frames[0]
    shifted = np.roll(np.roll(img, 2, axis=1), -1, axis=0)
    g = np.stack(np.meshgrid(np.arange(40, 280, 20), np.arange(40, 200, 20)), -1).reshape(-1, 2).astype(np.float32)
    nt, stt, _, _ = O.lk16(O.Pyramid16(img), O.Pyramid16(shifted), g)
    assert (stt == 1).all()
    assert np.abs(nt - (g + np.float32([2, -1]))).max() < 0.02


def test_f32_path_definitions_and_tracking():
    """the fp32 pixel path (16U / 32F frames): pyrDown in the fp16 path's order
    without rounding, the Scharr formula in fp32; on u8-valued frames it tracks
    as the 8-bit and fp16 paths do (a sanity bound), and a 16U frame (x257)
    tracks the same motion"""
    frames, gt = O.synth(20261016, 320, 240, 12, 0, 2)
    a = frames[0].astype(np.float32)
    d = O.pyr_down32(a)
    ref = O.pyr_down16(frames[0].astype(np.float16)).astype(np.float32)
    assert np.abs(d - ref).max() <= np.abs(ref).max() * 2 ** -10  # fp16 rounding is the only difference
    y, x = 7, 9
    c = O.scharr32(a)
    t0 = [(a[y - 1, x + k] + a[y + 1, x + k]) * np.float32(3) + a[y, x + k] * np.float32(10) for k in (-1, 0, 1)]
    assert c[y, x, 0] == np.float32(t0[2] - t0[0])
    rng = np.random.default_rng(1)
    pts = np.concatenate([np.stack([rng.uniform(x, x + bw, 24), rng.uniform(y, y + bh, 24)], 1)
                          for v, x, y, bw, bh in gt[0] if v]).astype(np.float32)
    nx, st, _, _ = O.lk(O.Pyramid(frames[0]), O.Pyramid(frames[1]), pts, accum=O.ACCUM_EXACT)
    nx32, st32, _, _ = O.lk16(O.Pyramid16(frames[0], f32=True), O.Pyramid16(frames[1], f32=True), pts)
    both = (st == 1) & (st32 == 1)
    assert both.mean() > 0.9 and (st == st32).mean() > 0.99
    assert (np.abs(nx - nx32)[both].max(1) <= 1e-2).mean() >= 0.99
    u16 = [f.astype(np.uint16) * 257 for f in frames[:2]]
    nxu, stu, _, _ = O.lk16(O.Pyramid16(u16[0], f32=True), O.Pyramid16(u16[1], f32=True), pts)
    bothu = (stu == 1) & (st32 == 1)
    assert bothu.mean() > 0.9
    assert (np.abs(nxu - nx32)[bothu].max(1) <= 1e-2).mean() >= 0.99
