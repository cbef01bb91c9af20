"""PyrLK on multi-channel frames (klt_cn.hip) vs the oracle's cn-generic
calcOpticalFlowPyrLK (tests/test_klt_cn_oracle.py pins it to the one-channel
path): pyramid levels and CV_16SC(2cn) Scharr planes bit-exact; tracked points,
status, error and iteration counts bit-exact with the exact-sum mode and within
SURVEY §8c's tolerance of the reference's SSE2 order."""
import numpy as np
import pytest
import torch

import _oracle as O
from test_gpu_klt import assert_exact, assert_tolerance, grid_points

pytestmark = pytest.mark.gpu


def _frames(cn, w, h, seed=11):
    fr, _ = O.synth(seed, w, h, 12, 0, 2)
    rng = np.random.default_rng(seed + cn)
    extra = []
    for c in range(1, cn):  # other channels: shifted / rescaled copies with noise, so they carry texture
        a = np.clip(fr[0].astype(int) * (c + 1) // (c + 2) + rng.integers(-8, 8, fr[0].shape), 0, 255)
        b = np.clip(fr[1].astype(int) * (c + 1) // (c + 2) + rng.integers(-8, 8, fr[1].shape), 0, 255)
        extra.append((np.roll(a, c, 1).astype(np.uint8), np.roll(b, c, 1).astype(np.uint8)))
    A = np.stack([fr[0]] + [e[0] for e in extra], 2)
    B = np.stack([fr[1]] + [e[1] for e in extra], 2)
    return np.ascontiguousarray(A), np.ascontiguousarray(B)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("cn", [2, 3, 4])
@pytest.mark.parametrize("shape,maxlev,win", [((120, 160), 3, (21, 21)), ((77, 301), 2, (15, 9)),
                                              ((480, 640), 3, (21, 21))])
def test_pyramid_cn_bit_exact(gpu, cn, shape, maxlev, win):
    from opencv_amd import klt

    A, _ = _frames(cn, shape[1], shape[0])
    P = klt.build_pyramid(_dev(A), win, maxlev, ctx=gpu)
    torch.cuda.synchronize()
    R = O.Pyramid(A, win, maxlev, P.pyr.lv[0].pad)
    assert P.nlevels == R.nlevels and P.channels == cn
    for lvl in range(P.nlevels):
        assert np.array_equal(P.level(lvl, with_border=True), R.level(lvl, with_border=True)), lvl
        assert np.array_equal(P.deriv(lvl), O.scharr(R.level(lvl))), lvl


def run_pair_cn(gpu, A, B, pts, win=(21, 21), maxlev=3, iters=30, eps=0.01, flags=0, init=None):
    from opencv_amd import klt

    lk = klt.SparsePyrLKOpticalFlow(win, maxlev, iters, bool(flags & 4), epsilon=eps, getMinEigenVals=bool(flags & 8))
    Pa = klt.build_pyramid(_dev(A), win, maxlev, ctx=gpu)
    Pb = klt.build_pyramid(_dev(B), win, maxlev, ctx=gpu)
    r = lk.calc(Pa, Pb, _dev(pts), None if init is None else _dev(init), want_iters=True)
    torch.cuda.synchronize()
    g = (r.next_pts.cpu().numpy(), r.status.cpu().numpy(), r.err.cpu().numpy(), r.iters.cpu().numpy())
    pad = Pa.pyr.lv[0].pad
    Ra, Rb = O.Pyramid(A, win, maxlev, pad), O.Pyramid(B, win, maxlev, pad)
    ex = O.lk(Ra, Rb, pts, win, maxlev, iters, eps, flags, accum=O.ACCUM_EXACT, init=init)
    sse = O.lk(Ra, Rb, pts, win, maxlev, iters, eps, flags, accum=O.ACCUM_SSE2, init=init)
    return g, ex, sse


@pytest.mark.parametrize("cn", [2, 3, 4])
@pytest.mark.parametrize("win,maxlev", [((21, 21), 3), ((15, 9), 2), ((31, 31), 1), ((63, 63), 0)])
def test_lk_cn_matches_oracle(gpu, cn, win, maxlev):
    A, B = _frames(cn, 320, 240)
    pts = grid_points(240, 320, 9, 3)
    pts = np.concatenate([pts, np.float32([[-5, 10], [330, 20], [0.5, 0.5], [319.5, 239.5]])])
    g, ex, sse = run_pair_cn(gpu, A, B, pts, win, maxlev)
    assert_exact(g, ex)
    assert_tolerance(g, sse)


@pytest.mark.parametrize("cn", [3, 4])
def test_lk_cn_flags(gpu, cn):
    A, B = _frames(cn, 200, 150, seed=5)
    pts = grid_points(150, 200, 11, 2)
    rng = np.random.default_rng(cn)
    init = pts + rng.uniform(-2, 2, pts.shape).astype(np.float32)
    g, ex, _ = run_pair_cn(gpu, A, B, pts, flags=O.OPTFLOW_USE_INITIAL_FLOW, init=init)
    assert_exact(g, ex)
    g, ex, _ = run_pair_cn(gpu, A, B, pts, flags=O.OPTFLOW_LK_GET_MIN_EIGENVALS)
    assert_exact(g, ex)


def test_lk_cn_rejects_mixed_inputs(gpu):
    from opencv_amd import klt, _lib

    A, B = _frames(3, 160, 120)
    P3 = klt.build_pyramid(_dev(A), (21, 21), 2, ctx=gpu)
    P1 = klt.build_pyramid(_dev(np.ascontiguousarray(B[:, :, 0])), (21, 21), 2, ctx=gpu)
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 2)
    with pytest.raises(_lib.TbdkError):
        lk.calc(P3, P1, _dev(grid_points(120, 160, 20, 10)))
    with pytest.raises(_lib.TbdkError):
        klt.Pyramid(gpu, 160, 120, 2, (21, 21), channels=5)
