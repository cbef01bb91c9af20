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
