"""Dense Farneback on the GPU (libtbdk farneback.hip) vs the CPU oracle.

Bit-exact: the level images (GaussianBlur + resize), the polynomial expansion
and the whole flow field of the OPTFLOW_FARNEBACK_GAUSSIAN variant.  The box
variant (flags 0) sums its windows in exact order where the reference keeps
running sums whose float-rounded row differences accumulate over the image:
it is bit-exact against the oracle's exact-order mode, and within a stated
tolerance of the reference's running sums, well inside the reference's own
GPU-vs-CPU criterion (cudaoptflow/test/test_optflow.cpp:336-348:
CCORR_NORMED similarity within 1e-4)."""
import numpy as np
import pytest
import torch

import _oracle as O

pytestmark = pytest.mark.gpu


def _frames(seed, w, h, shift=(2.5, -1.25), nobj=6):
    fr, _ = O.synth(seed, w, h, nobj, 0, 2)
    return fr[0], fr[1]


def _gpu_flow(gpu, a, b, init=None, **kw):
    from opencv_amd import farneback as F

    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    fb = F.FarnebackOpticalFlow.create(ctx=gpu, **kw)
    out = fb.calc(ta, tb, None if init is None else torch.from_numpy(init.copy()).cuda())
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _similarity(a, b):
    """1 - CCORR_NORMED of two equal-size fields (cvtest checkSimilarity)."""
    a = a.astype(np.float64).ravel()
    b = b.astype(np.float64).ravel()
    return abs(float(a @ b) / (np.linalg.norm(a) * np.linalg.norm(b)) - 1.0)


@pytest.mark.parametrize("src,dst,ks,sigma", [
    ((97, 61), (97, 61), 3, 0.0),          # level 0: blur only
    ((96, 64), (48, 32), 3, 0.5),          # exact 2x: INTER_AREA fast path
    ((200, 120), (50, 30), 9, 1.5),        # 4x: INTER_LINEAR
    ((201, 121), (60, 36), 19, 3.5),       # ragged: INTER_LINEAR, both axes
    ((333, 250), (266, 200), 3, 0.125),    # pyr_scale 0.8
    ((640, 480), (58, 43), 25, 5.05),      # pyr_scale 0.3, level 2
    ((1242, 375), (621, 188), 3, 0.5),     # KITTI level 1: x exact 2, y not
])
def test_level_image_bit_exact(gpu, src, dst, ks, sigma):
    from opencv_amd import farneback as F

    rng = np.random.default_rng(sum(src) + ks)
    img = rng.integers(0, 256, (src[1], src[0]), dtype=np.uint8)
    got = F.level_image(torch.from_numpy(img).cuda(), dst, ks, sigma, ctx=gpu)
    torch.cuda.synchronize()
    ref = O.fb_level_image(img, dst, ks, sigma)
    assert np.array_equal(got.cpu().numpy(), ref)


@pytest.mark.parametrize("n,sigma", [(5, 1.1), (7, 1.5), (3, 0.0), (15, 2.0)])
@pytest.mark.parametrize("shape", [(61, 97), (240, 320), (5, 7)])
def test_poly_exp_bit_exact(gpu, n, sigma, shape):
    from opencv_amd import farneback as F

    rng = np.random.default_rng(n * 100 + shape[0])
    src = (rng.random(shape, dtype=np.float32) * 255).astype(np.float32)
    got = F.poly_exp(torch.from_numpy(src).cuda(), n, sigma, ctx=gpu)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), O.fb_poly_exp(src, n, sigma))


@pytest.mark.parametrize("pyr_scale,poly_n,winsize", [(0.5, 5, 13), (0.3, 7, 13), (0.8, 5, 9), (0.5, 7, 21),
                                                       (0.5, 5, 4)])
def test_gaussian_variant_bit_exact(gpu, pyr_scale, poly_n, winsize):
    a, b = _frames(11, 320, 240)
    sigma = 1.1 if poly_n <= 5 else 1.5
    kw = dict(pyr_scale=pyr_scale, levels=5, winsize=winsize, iterations=10, poly_n=poly_n, poly_sigma=sigma,
              flags=O.FARNEBACK_GAUSSIAN)
    ref = O.farneback(a, b, **kw)
    got = _gpu_flow(gpu, a, b, numLevels=5, pyrScale=pyr_scale, winSize=winsize, numIters=10, polyN=poly_n,
                    polySigma=sigma, flags=O.FARNEBACK_GAUSSIAN)
    assert np.array_equal(got, ref), np.abs(got - ref).max()


@pytest.mark.parametrize("pyr_scale,poly_n,winsize", [(0.5, 5, 13), (0.3, 7, 13), (0.8, 5, 15), (0.5, 5, 1),
                                                       (0.5, 7, 21), (0.5, 5, 4)])
def test_box_variant_bit_exact_vs_direct_order(gpu, pyr_scale, poly_n, winsize):
    """flags 0 (the default): bit-exact against the oracle's exact-order box
    sums (box_direct), every level, every iteration."""
    a, b = _frames(12, 320, 240)
    sigma = 1.1 if poly_n <= 5 else 1.5
    ref = O.farneback(a, b, pyr_scale=pyr_scale, levels=5, winsize=winsize, iterations=10, poly_n=poly_n,
                      poly_sigma=sigma, flags=0, box_direct=True)
    got = _gpu_flow(gpu, a, b, numLevels=5, pyrScale=pyr_scale, winSize=winsize, numIters=10, polyN=poly_n,
                    polySigma=sigma, flags=0)
    assert np.array_equal(got, ref), np.abs(got - ref).max()


@pytest.mark.parametrize("pyr_scale,poly_n,winsize", [(0.5, 5, 13), (0.3, 7, 13), (0.8, 5, 15)])
def test_box_variant_vs_reference_running_sums(gpu, pyr_scale, poly_n, winsize):
    """flags 0 vs the reference's running sums.  Stated tolerance: similarity
    (1 - CCORR_NORMED) < 1e-5, ten times tighter than the reference's own
    CUDA-vs-CPU bound 1e-4 (test_optflow.cpp:347); >= 99 % of pixels within
    1e-2 px; max 0.5 px.  (The two differ only by the reference's float-rounded
    running-sum differences, tests/test_farneback_oracle.py.)"""
    a, b = _frames(13, 640, 480)
    sigma = 1.1 if poly_n <= 5 else 1.5
    ref = O.farneback(a, b, pyr_scale=pyr_scale, levels=5, winsize=winsize, iterations=10, poly_n=poly_n,
                      poly_sigma=sigma, flags=0)
    got = _gpu_flow(gpu, a, b, numLevels=5, pyrScale=pyr_scale, winSize=winsize, numIters=10, polyN=poly_n,
                    polySigma=sigma, flags=0)
    d = np.abs(got - ref).max(axis=2)
    assert _similarity(ref, got) < 1e-5
    assert np.mean(d <= 1e-2) >= 0.99, np.mean(d <= 1e-2)
    assert d.max() <= 0.5, d.max()


@pytest.mark.parametrize("w,h", [(33, 33), (64, 40), (130, 70), (1242, 375)])
def test_odd_sizes_and_iterations(gpu, w, h):
    a, b = _frames(w + h, w, h, nobj=2)
    for iters in (0, 1, 3):
        for flags in (0, O.FARNEBACK_GAUSSIAN):
            ref = O.farneback(a, b, iterations=iters, flags=flags, box_direct=True)
            got = _gpu_flow(gpu, a, b, numIters=iters, flags=flags)
            assert np.array_equal(got, ref), (iters, flags)


def test_prep_ahead_equal(gpu):
    """ctx option fb_prep_ahead: the level preps on the side stream (default) and inline
    give identical flows, at two sizes back to back (the per-level regions and events
    are reused) and for one level (no side stream)"""
    runs = []
    for ahead in (1, 0):
        gpu.set_option("fb_prep_ahead", ahead)
        try:
            out = []
            for (w, h), kw in (((641, 359), {}), ((333, 250), dict(flags=O.FARNEBACK_GAUSSIAN)),
                               ((200, 120), dict(numLevels=0))):
                a, b = _frames(w * h, w, h, nobj=3)
                out.append(_gpu_flow(gpu, a, b, **kw))
            runs.append(out)
        finally:
            gpu.set_option("fb_prep_ahead", 1)
    for x, y in zip(*runs):
        assert np.array_equal(x, y)


def test_1080p_translation(gpu):
    """Full-size known motion: a 1080p synthetic frame shifted by (5, -3)."""
    fr, _ = O.synth(20261015, 1920, 1080, 24, 0, 1)
    a = fr[0]
    b = np.roll(a, (-3, 5), axis=(0, 1))
    got = _gpu_flow(gpu, a, b)
    inner = got[40:-40, 40:-40]
    assert abs(np.median(inner[..., 0]) - 5) < 0.01 and abs(np.median(inner[..., 1]) + 3) < 0.01
    assert np.mean(np.abs(inner - np.float32([5, -3])).max(axis=2) < 0.1) > 0.95


@pytest.mark.parametrize("w,h,pyr_scale,levels", [
    (320, 240, 0.5, 5),    # coarsest 80x60: integer factor 4 (resizeAreaFast_, area 16)
    (96, 64, 0.5, 5),      # coarsest 48x32: factor 2 (area 4)
    (320, 240, 0.3, 5),    # fractional factors: the computeResizeAreaTab path
    (1242, 375, 0.5, 5),   # 1242 -> 310 after a .5 rounding: the table path in x
    (130, 70, 0.5, 0),     # one level: copy, *= 1 skipped
])
@pytest.mark.parametrize("iters", [0, 10])
def test_use_initial_flow_bit_exact(gpu, w, h, pyr_scale, levels, iters):
    """OPTFLOW_USE_INITIAL_FLOW (optflowgf.cpp:1151-1157): the coarsest level
    starts from resize(flow0, INTER_AREA) * scale.  Gaussian variant against the
    reference order, box variant against the exact-order mode."""
    a, b = _frames(w * 7 + h, w, h, nobj=3)
    rng = np.random.default_rng(w + levels)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    init = np.stack([2.5 + 0.01 * xx, -1.25 - 0.005 * yy], 2) + rng.uniform(-0.5, 0.5, (h, w, 2))
    init = init.astype(np.float32)
    for flags, direct in ((O.FARNEBACK_GAUSSIAN, False), (0, True)):
        f = flags | O.OPTFLOW_USE_INITIAL_FLOW
        ref = O.farneback(a, b, pyr_scale=pyr_scale, levels=levels, iterations=iters, flags=f, box_direct=direct,
                          init_flow=init)
        got = _gpu_flow(gpu, a, b, init=init, numLevels=levels, pyrScale=pyr_scale, numIters=iters, flags=f)
        assert np.array_equal(got, ref), (flags, np.abs(got - ref).max())


def test_use_initial_flow_converges_from_the_true_motion(gpu):
    """Seeded with the true shift, one level and a few iterations keep it."""
    fr, _ = O.synth(77, 640, 480, 12, 0, 1)
    a = fr[0]
    b = np.roll(a, (-3, 5), axis=(0, 1))
    init = np.broadcast_to(np.float32([5, -3]), (480, 640, 2))
    from opencv_amd import farneback as F

    got = _gpu_flow(gpu, a, b, init=init, numLevels=0, numIters=3, flags=F.OPTFLOW_USE_INITIAL_FLOW)
    inner = got[40:-40, 40:-40]
    assert np.mean(np.abs(inner - np.float32([5, -3])).max(axis=2) < 0.1) > 0.95


def test_rejects_bad_arguments(gpu):
    from opencv_amd import _lib
    from opencv_amd import farneback as F

    a = torch.zeros((64, 64), dtype=torch.uint8, device="cuda")
    for kw in (dict(pyrScale=1.0), dict(fastPyramids=True), dict(winSize=0), dict(winSize=23), dict(polyN=0),
               dict(polyN=16), dict(numIters=-1), dict(flags=F.OPTFLOW_USE_INITIAL_FLOW), dict(flags=1)):
        with pytest.raises(_lib.TbdkError):
            F.FarnebackOpticalFlow.create(ctx=gpu, **kw).calc(a, a)
    with pytest.raises(_lib.TbdkError):
        F.FarnebackOpticalFlow.create(ctx=gpu).calc(a, a[:32])


@pytest.mark.parametrize("flags,direct", [(0, True), ("gauss", False)])
def test_4k_pair_bit_exact(gpu, flags, direct):
    """BASELINE configs[4] at its full size: the bench's 3840x2160 synthetic pair
    (seed + 7, 512 objects) with cv::cuda::FarnebackOpticalFlow's defaults
    (5 levels, pyrScale 0.5, winSize 13, 10 iterations, polyN 5, sigma 1.1).
    Box variant (the bench's) against the oracle's exact-order mode, the
    Gaussian variant against the reference order: bit-exact over all 8.3 Mpx
    (optflowgf.cpp:1096-1191)."""
    f = O.FARNEBACK_GAUSSIAN if flags == "gauss" else 0
    fr, _ = O.synth(20261015 + 7, 3840, 2160, 512, 0, 2)
    ref = O.farneback(fr[0], fr[1], flags=f, box_direct=direct)
    got = _gpu_flow(gpu, fr[0], fr[1], flags=f)
    assert np.array_equal(got, ref), np.abs(got - ref).max()
    assert np.isfinite(ref).all() and np.abs(ref).max() > 0.5  # real motion, not a trivial field


def test_calls_on_alternating_streams(gpu):
    """Back-to-back calls on different streams share the context's scratch: a
    call on another stream waits for the previous call's completion (the
    prep-ahead fork orders only the caller's own stream), so every flow equals
    the one computed alone."""
    from opencv_amd import farneback as F

    pairs = [_frames(900 + i, 640, 360, nobj=5) for i in range(4)]
    fb = F.FarnebackOpticalFlow.create(ctx=gpu)
    want = []
    for a, b in pairs:
        want.append(fb.calc(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()))
        torch.cuda.synchronize()
    want = [w.cpu().numpy() for w in want]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dev = [(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()) for a, b in pairs]
    outs = [torch.empty((360, 640, 2), dtype=torch.float32, device="cuda") for _ in pairs]
    torch.cuda.synchronize()
    for rep in range(3):
        for i, (a, b) in enumerate(dev):
            st = streams[(i + rep) % 2]
            with torch.cuda.stream(st):
                fb.calc(a, b, outs[i], stream=st)
        torch.cuda.synchronize()
        for o, w in zip(outs, want):
            assert np.array_equal(o.cpu().numpy(), w)
