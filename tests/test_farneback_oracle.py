"""CPU checks of the Farneback oracle (oracle/farneback_oracle.c): known answers
the reference's algorithm must reproduce.  The reference's own Farneback
fixtures (opencv_extra rubberwhale1/2.png, video/test/test_optflowgf.cpp) are
not vendored, so the restatement is pinned by these identities and by its
line-by-line citations (parity of the full flow field against the reference
is unpinned)."""
import numpy as np
import pytest

import _oracle as O


def test_gaussian_kernel_matches_get_gaussian_kernel():
    # getGaussianKernel small fixed table for sigma <= 0 (smooth.dispatch.cpp:70-122)
    assert np.array_equal(O.gaussian_kernel(3, 0), np.float32([0.25, 0.5, 0.25]))
    assert np.array_equal(O.gaussian_kernel(5, -1), np.float32([0.0625, 0.25, 0.375, 0.25, 0.0625]))
    k = O.gaussian_kernel(9, 1.5)
    assert abs(float(k.astype(np.float64).sum()) - 1) < 1e-6 and np.array_equal(k, k[::-1])
    x = np.arange(9) - 4.0
    ref = np.exp(-x * x / (2 * 1.5 * 1.5))
    assert np.allclose(k, ref / ref.sum(), rtol=1e-6)


@pytest.mark.parametrize("n,sigma", [(5, 1.1), (7, 1.5)])
def test_poly_exp_recovers_quadratic(n, sigma):
    """FarnebackPolyExp is a weighted least-squares fit of a quadratic: on an
    exact quadratic image it returns the coefficients (away from borders):
    R = [b_y, b_x, a_yy, a_xx, a_xy] (optflowgf.cpp:193-198)."""
    h, w = 48, 64
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    cx, cy = 32, 24
    I = (10 + 0.5 * (x - cx) - 0.25 * (y - cy) + 0.01 * (x - cx) ** 2 + 0.02 * (y - cy) ** 2
         + 0.005 * (x - cx) * (y - cy)).astype(np.float32)
    R = O.fb_poly_exp(I, n, sigma)
    # linear coefficients vary with position: at (x, y) b_x = 0.5 + 2*0.01*(x-cx) + 0.005*(y-cy)
    yy, xx = slice(n + 2, h - n - 2), slice(n + 2, w - n - 2)
    bx = 0.5 + 0.02 * (x - cx) + 0.005 * (y - cy)
    by = -0.25 + 0.04 * (y - cy) + 0.005 * (x - cx)
    assert np.allclose(R[yy, xx, 1], bx[yy, xx], atol=2e-4)
    assert np.allclose(R[yy, xx, 0], by[yy, xx], atol=2e-4)
    assert np.allclose(R[yy, xx, 3], 0.01, atol=2e-5)
    assert np.allclose(R[yy, xx, 2], 0.02, atol=2e-5)
    assert np.allclose(R[yy, xx, 4], 0.005, atol=2e-5)


def test_level_image_identity_and_halving():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    # level 0: the 3x3 fixed-kernel blur, no resize
    out = O.fb_level_image(img, (53, 37), 3, 0.0)
    f = img.astype(np.float64)
    pad = np.pad(f, 1, mode="reflect")  # numpy "reflect" == BORDER_REFLECT_101
    k = np.array([0.25, 0.5, 0.25])
    rows = pad[:, :-2] * k[0] + pad[:, 1:-1] * k[1] + pad[:, 2:] * k[2]
    ref = rows[:-2] * k[0] + rows[1:-1] * k[1] + rows[2:] * k[2]
    assert np.allclose(out, ref, atol=1e-4)
    # a constant image stays constant through blur + any resize
    c = np.full((60, 80), 77, np.uint8)
    for size in [(40, 30), (24, 18), (64, 48), (20, 15)]:
        assert np.allclose(O.fb_level_image(c, size, 9, 1.5), 77.0, atol=1e-4)


@pytest.mark.parametrize("flags", [0, O.FARNEBACK_GAUSSIAN])
@pytest.mark.parametrize("shift", [(3, 2), (-1, 4)])
def test_farneback_recovers_translation(flags, shift):
    fr, _ = O.synth(20261015, 320, 240, 6, 0, 1)
    a = fr[0]
    b = np.roll(a, (shift[1], shift[0]), axis=(0, 1))
    f = O.farneback(a, b, flags=flags)
    inner = f[24:-24, 24:-24]
    assert abs(np.median(inner[..., 0]) - shift[0]) < 0.01
    assert abs(np.median(inner[..., 1]) - shift[1]) < 0.01
    assert np.mean(np.abs(inner[..., 0] - shift[0]) < 0.1) > 0.95


def test_farneback_zero_motion_and_levels():
    fr, _ = O.synth(7, 160, 120, 3, 0, 1)
    f = O.farneback(fr[0], fr[0], levels=3)
    # the last row/column take UpdateMatrices' out-of-range branch (R1 = 0,
    # optflowgf.cpp:278-284), so only the interior is exactly still
    assert np.abs(f[16:-16, 16:-16]).max() < 1e-3
    with pytest.raises(ValueError):
        O.farneback(fr[0], fr[0], pyr_scale=1.0)


@pytest.mark.parametrize("pyr_scale,poly_n,winsize", [(0.5, 5, 13), (0.3, 7, 13), (0.8, 5, 15)])
def test_direct_order_box_sums_vs_running_sums(pyr_scale, poly_n, winsize):
    """The exact-order box sums the GPU uses (box_direct) differ from the
    reference's running sums only by the latter's accumulated float rounding:
    similarity far below the reference's own 1e-4 bound (test_optflow.cpp:347)."""
    fr, _ = O.synth(13, 640, 480, 6, 0, 2)
    sigma = 1.1 if poly_n <= 5 else 1.5
    kw = dict(pyr_scale=pyr_scale, levels=5, winsize=winsize, iterations=10, poly_n=poly_n, poly_sigma=sigma)
    r = O.farneback(fr[0], fr[1], **kw)
    d = O.farneback(fr[0], fr[1], box_direct=True, **kw)
    e = np.abs(r - d).max(axis=2)
    a, b = r.astype(np.float64).ravel(), d.astype(np.float64).ravel()
    assert abs(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)) - 1) < 1e-5
    assert np.mean(e <= 1e-2) >= 0.99 and e.max() <= 0.5
    # the Gaussian variant has no running sums: the two modes are identical
    g0 = O.farneback(fr[0], fr[1], flags=O.FARNEBACK_GAUSSIAN, **kw)
    g1 = O.farneback(fr[0], fr[1], flags=O.FARNEBACK_GAUSSIAN, box_direct=True, **kw)
    assert np.array_equal(g0, g1)


# ---- INTER_AREA resize (the USE_INITIAL_FLOW input of the coarsest level) ----

def test_resize_area_matches_reference_known_answer():
    """Imgproc_resize_area.regression (imgproc/test/test_imgwarp.cpp:1536-1571):
    16x16 CV_16UC1 at fx = fy = 0.3 through the table path (ResizeArea_Invoker
    with a float accumulator; ushort -> float is exact, saturate_cast rounds)."""
    import json
    import os

    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "resize_area_regression.json")))
    src = np.float32(g["input"]).reshape(16, 16)
    out = np.rint(O.resize_area(src, (5, 5), inv_scale=(0.3, 0.3)))
    exp = np.float32(g["expected"]).reshape(5, 5)
    assert np.abs(out - exp).max() <= 1.0  # the reference test's tolerance
    assert np.array_equal(out, exp)


def test_resize_area_half_matches_reference_formula():
    """Resize.Area_half (test_imgwarp.cpp:1671-1709) for float: within 7e-5 of
    ((a+b) + (c+d)) * 0.25 on values in [-1000, 1000]; here with 2 channels."""
    rng = np.random.default_rng(17)
    src = rng.uniform(-1000, 1000, (100, 100, 2)).astype(np.float32)
    out = O.resize_area(src, (50, 50))
    s = src.astype(np.float32)
    ref = ((s[0::2, 0::2] + s[0::2, 1::2]) + (s[1::2, 0::2] + s[1::2, 1::2])) * np.float32(0.25)
    assert np.abs(out - ref).max() <= 7e-5


@pytest.mark.parametrize("size", [(17, 13), (40, 30), (7, 5)])
def test_resize_area_general_is_the_cell_average(size):
    """The table path averages each output cell over the fractional source area:
    each source pixel [s, s+1) weighs its overlap with the cell [d*scale,
    (d+1)*scale) (computed here in double, independently of the tables), and a
    constant image stays constant."""
    h, w = 60, 80
    dw, dh = size
    rng = np.random.default_rng(dw)
    img = rng.uniform(0, 255, (h, w)).astype(np.float32)
    out = O.resize_area(img, (dw, dh))

    def weights(ss, ds):
        sc = ss / ds
        W = np.zeros((ds, ss))
        for d in range(ds):
            lo, hi = d * sc, min((d + 1) * sc, ss)
            for s_ in range(int(np.floor(lo)), int(np.ceil(hi))):
                W[d, s_] = max(0.0, min(hi, s_ + 1) - max(lo, s_))
            W[d] /= W[d].sum()
        return W

    ref = weights(h, dh) @ img.astype(np.float64) @ weights(w, dw).T
    assert np.allclose(out, ref, atol=2e-3)
    const = np.full((h, w, 2), 1.75, np.float32)
    assert np.allclose(O.resize_area(const, (dw, dh)), 1.75, atol=1e-5)


def test_farneback_initial_flow_is_used_and_exact_at_one_level():
    """OPTFLOW_USE_INITIAL_FLOW: with 0 iterations and one level the output is
    the input flow (resize to the same size is a copy, *= 1 a no-op); with several
    levels and 0 iterations it is the area-downscaled, rescaled, then linearly
    upscaled input; iterating from the true motion keeps it."""
    rng = np.random.default_rng(3)
    h, w = 64, 96
    a = rng.integers(0, 256, (h, w), dtype=np.uint8)
    init = rng.uniform(-2, 2, (h, w, 2)).astype(np.float32)
    out = O.farneback(a, a, levels=0, iterations=0, flags=O.OPTFLOW_USE_INITIAL_FLOW, init_flow=init)
    assert np.array_equal(out, init)
    zero = O.farneback(a, a, levels=0, iterations=0, flags=0, init_flow=init)
    assert not zero.any()
    const = np.full((h, w, 2), 0.5, np.float32)
    out = O.farneback(a, a, levels=1, iterations=0, flags=O.OPTFLOW_USE_INITIAL_FLOW, init_flow=const)
    assert np.allclose(out, 0.5, atol=1e-6)  # 0.5 -> area -> *0.5 -> linear up -> *2
