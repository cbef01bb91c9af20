"""Multi-channel PyrLK in the oracle (oracle/klt_oracle.c, cn-generic): the
CPU calcOpticalFlowPyrLK on interleaved cn-channel u8 frames
(video/src/lkpyramid.cpp:55-144 calcSharrDeriv over cols*cn elements,
:178-695 LKTrackerInvoker over winW*cn window elements; pyrDown_ per channel,
imgproc/src/pyramids.cpp:746-790).

No reference-produced multi-channel vectors exist here, so the cn-generic code
is pinned to the one-channel oracle (itself pinned, tests/test_oracle.py) by
identities the reference's arithmetic implies:
  * pyrDown and calcSharrDeriv of an interleaved image are the one-channel
    results of each channel;
  * with the exact sums (ORC_ACCUM_EXACT), channels holding a constant add
    nothing to G, b or the error sum, so (gray, 0, 0) tracks exactly as gray
    and its error is gray's x 1/cn; permuting the channels changes nothing;
  * in the reference's SSE2 order, the cn copies (g, g, g) track as gray up to
    the float rounding of the sums."""
import os

import numpy as np
import pytest

import _oracle as O
from test_oracle import grid_points, shifted_pair


def _frames(seed=3, w=160, h=120):
    fr, _ = O.synth(seed, w, h, 6, 0, 2)
    return fr[0], fr[1]


@pytest.mark.parametrize("cn", [2, 3, 4])
def test_pyramid_and_scharr_are_per_channel(cn):
    a, _ = _frames()
    rng = np.random.default_rng(cn)
    chans = [a] + [rng.integers(0, 256, a.shape, dtype=np.uint8) for _ in range(cn - 1)]
    img = np.stack(chans, axis=2)
    P = O.Pyramid(img, (21, 21), 3)
    Ps = [O.Pyramid(c, (21, 21), 3) for c in chans]
    assert P.nlevels == Ps[0].nlevels
    for lvl in range(P.nlevels):
        L = P.level(lvl, with_border=True)
        for c in range(cn):
            assert np.array_equal(L[:, :, c], Ps[c].level(lvl, with_border=True)), (lvl, c)
    d = O.scharr(img)
    for c in range(cn):
        assert np.array_equal(d[:, :, 2 * c:2 * c + 2], O.scharr(chans[c]))


def _lk_pair(img0, img1, pts, accum, **kw):
    P0, P1 = O.Pyramid(img0, (21, 21), 3), O.Pyramid(img1, (21, 21), 3)
    return O.lk(P0, P1, pts, (21, 21), 3, accum=accum, **kw)


@pytest.mark.parametrize("cn", [2, 3, 4])
def test_constant_channels_track_exactly_as_gray(cn):
    a, b = _frames()
    pts = grid_points(a.shape[0], a.shape[1], 9, 4)
    z = [np.full(a.shape, 77, np.uint8)] * (cn - 1)
    g = _lk_pair(a, b, pts, O.ACCUM_EXACT)
    m = _lk_pair(np.stack([a] + z, 2), np.stack([b] + z, 2), pts, O.ACCUM_EXACT)
    assert np.array_equal(m[0], g[0]) and np.array_equal(m[1], g[1]) and np.array_equal(m[3], g[3])
    ok = g[1] == 1
    # errval is the same integer-valued sum; only the 1/(32*winW*cn*winH) scale differs
    assert np.allclose(m[2][ok] * cn, g[2][ok], rtol=1e-6, atol=1e-7)
    # LK_GET_MIN_EIGENVALS: minEig is normalised by 2*winW*winH (no cn)
    gm = _lk_pair(a, b, pts, O.ACCUM_EXACT, flags=O.OPTFLOW_LK_GET_MIN_EIGENVALS)
    mm = _lk_pair(np.stack([a] + z, 2), np.stack([b] + z, 2), pts, O.ACCUM_EXACT, flags=O.OPTFLOW_LK_GET_MIN_EIGENVALS)
    assert np.array_equal(gm[2], mm[2])


def test_channel_permutation_is_invariant_with_exact_sums():
    a, b = _frames()
    rng = np.random.default_rng(9)
    c1 = np.clip(a.astype(int) + rng.integers(-20, 20, a.shape), 0, 255).astype(np.uint8)
    c2 = np.clip(b.astype(int) + 5, 0, 255).astype(np.uint8)
    c1b = np.clip(b.astype(int) + rng.integers(-20, 20, b.shape), 0, 255).astype(np.uint8)
    c2b = np.clip(a.astype(int) + 5, 0, 255).astype(np.uint8)
    pts = grid_points(a.shape[0], a.shape[1], 11, 4)
    r0 = _lk_pair(np.stack([a, c1, c2], 2), np.stack([b, c1b, c2b], 2), pts, O.ACCUM_EXACT)
    r1 = _lk_pair(np.stack([c2, a, c1], 2), np.stack([c2b, b, c1b], 2), pts, O.ACCUM_EXACT)
    for x, y in zip(r0, r1):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("accum", [O.ACCUM_SSE2, O.ACCUM_EXACT])
def test_replicated_channels_track_as_gray(accum):
    a, b = _frames(5)
    pts = grid_points(a.shape[0], a.shape[1], 9, 4)
    g = _lk_pair(a, b, pts, accum)
    m = _lk_pair(np.stack([a] * 3, 2), np.stack([b] * 3, 2), pts, accum)
    both = (g[1] == 1) & (m[1] == 1)
    assert (g[1] == m[1]).mean() >= 0.99
    assert np.abs(m[0][both] - g[0][both]).max() < 1e-2


@pytest.mark.parametrize("dx,dy", [(2, 1), (-3, 4)])
def test_multichannel_known_translation(dx, dy):
    rng = np.random.default_rng(abs(dx * 7 + dy))
    base = rng.integers(0, 256, (140, 180, 3), dtype=np.uint8)
    import scipy.ndimage as nd
    base = np.stack([nd.gaussian_filter(base[:, :, c].astype(float), 2.0) for c in range(3)], 2)
    base = np.clip((base - base.min()) * 4, 0, 255).astype(np.uint8)
    pairs = [shifted_pair(base[:, :, c], dx, dy) for c in range(3)]
    a = np.stack([p[0] for p in pairs], 2)
    b = np.stack([p[1] for p in pairs], 2)
    pts = grid_points(a.shape[0], a.shape[1], 12, 16)
    nxt, st, err, _ = _lk_pair(a, b, pts, O.ACCUM_SSE2)
    ok = st == 1
    assert ok.mean() > 0.95
    assert np.abs(nxt[ok] - (pts[ok] + np.float32([dx, dy]))).max() < 0.05


# ---- the fp32 pixel path on cn channels (oracle/klt16_oracle.c, CV_16UC3/C4 and
# CV_32FC3/C4 frames of cv::cuda::SparsePyrLKOpticalFlow, cudaoptflow/src/pyrlk.cpp:197-205)


def _f32_frames(cn, seed=5, w=160, h=120):
    a, b = _frames(seed, w, h)
    rng = np.random.default_rng(seed)
    noise = [rng.normal(0, 3, a.shape).astype(np.float32) for _ in range(cn - 1)]
    fa = np.stack([a.astype(np.float32)] + [a * 0.5 + 20 + n for n in noise], 2).astype(np.float32)
    fb = np.stack([b.astype(np.float32)] + [b * 0.5 + 20 + n for n in noise], 2).astype(np.float32)
    return fa, fb


@pytest.mark.parametrize("cn", [2, 3, 4])
def test_f32_pyramid_and_scharr_are_per_channel(cn):
    fa, _ = _f32_frames(cn)
    P = O.Pyramid16(fa, (21, 21), 3, f32=True)
    Ps = [O.Pyramid16(np.ascontiguousarray(fa[:, :, c]), (21, 21), 3, f32=True) for c in range(cn)]
    assert P.nlevels == Ps[0].nlevels and P.cn == cn
    for lvl in range(P.nlevels):
        for c in range(cn):
            assert np.array_equal(P.levels[lvl][:, :, c].view(np.uint32), Ps[c].levels[lvl].view(np.uint32))
            assert np.array_equal(P.derivs[lvl][:, :, 2 * c:2 * c + 2].view(np.uint32),
                                  Ps[c].derivs[lvl].view(np.uint32))


@pytest.mark.parametrize("cn", [2, 3, 4])
def test_f32_constant_channels_track_exactly_as_gray(cn):
    """a constant channel's interpolated derivatives are exactly 0, so its G and b
    terms are +0 and every running sum keeps its value: points, status,
    iterations and minEig equal the one-channel run bit for bit, wherever the
    constant channels sit"""
    a, b = _frames()
    fa, fb = a.astype(np.float32), b.astype(np.float32)
    pts = grid_points(a.shape[0], a.shape[1], 9, 4)
    g = O.lk16(O.Pyramid16(fa, f32=True), O.Pyramid16(fb, f32=True), pts)
    gm = O.lk16(O.Pyramid16(fa, f32=True), O.Pyramid16(fb, f32=True), pts, flags=O.OPTFLOW_LK_GET_MIN_EIGENVALS)
    z = np.full(a.shape, 77.25, np.float32)
    for pos in range(cn):
        chans_a, chans_b = [z] * cn, [z] * cn
        chans_a[pos], chans_b[pos] = fa, fb
        A, B = O.Pyramid16(np.stack(chans_a, 2), f32=True), O.Pyramid16(np.stack(chans_b, 2), f32=True)
        m = O.lk16(A, B, pts)
        assert np.array_equal(m[0].view(np.uint32), g[0].view(np.uint32)), pos
        assert np.array_equal(m[1], g[1]) and np.array_equal(m[3], g[3])
        mm = O.lk16(A, B, pts, flags=O.OPTFLOW_LK_GET_MIN_EIGENVALS)
        assert np.array_equal(mm[2].view(np.uint32), gm[2].view(np.uint32))


@pytest.mark.parametrize("cn,dx,dy", [(3, 3, -2), (4, -2, 1)])
def test_f32_multichannel_known_translation(cn, dx, dy):
    img = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "basketball_pair.npz"))["a"]
    a, b = shifted_pair(img, dx, dy)
    fa = np.stack([a.astype(np.float32) * (c + 1) / cn for c in range(cn)], 2).astype(np.float32)
    fb = np.stack([b.astype(np.float32) * (c + 1) / cn for c in range(cn)], 2).astype(np.float32)
    pts = grid_points(a.shape[0], a.shape[1], 24, 48)
    nx, st, err, _ = O.lk16(O.Pyramid16(fa, f32=True), O.Pyramid16(fb, f32=True), pts)
    e = np.abs(nx - (pts + np.float32([dx, dy]))).max(1)
    assert st.mean() > 0.95 and np.median(e[st == 1]) < 0.05
