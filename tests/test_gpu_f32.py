"""GPU parity of the fp32 pixel path (16U and 32F frames, the other depths
cv::cuda::SparsePyrLKOpticalFlow takes, cudaoptflow/src/pyrlk.cpp:189-205;
the CPU PyrLK has no such path).  The checker is oracle/klt16_oracle.c in its
fp32 mode (the fp16 path's algorithm with nothing rounded to fp16): fp32
levels, their reflect-101 frames and fp32 derivative pairs bit-exact from u8,
u16 and fp32 frames; sparse LK bit-exact (points, status, error, iterations)."""
import numpy as np
import pytest
import torch

import _oracle as O
from test_gpu_f16 import box_points, edge_points, to_dev

pytestmark = pytest.mark.gpu


def _frames(kind, w, h, seed=7):
    frames, gt = O.synth(seed, w, h, 8, 0, 2)
    if kind == "u8":
        return frames[0], frames[1], gt
    if kind == "u16":
        rng = np.random.default_rng(seed)
        return [(f.astype(np.uint16) * 257 + rng.integers(0, 257, f.shape)).astype(np.uint16) for f in frames[:2]] + [gt]
    rng = np.random.default_rng(seed + 1)
    return [(f.astype(np.float32) / 255.0 + rng.normal(0, 1e-3, f.shape)).astype(np.float32) for f in frames[:2]] + [gt]


def _dev_pyr(ctx, img, win, max_level):
    from opencv_amd import klt

    return klt.Pyramid(ctx, img.shape[1], img.shape[0], max_level, win, torch.float32).build(to_dev(img))


@pytest.mark.parametrize("kind", ["u8", "u16", "f32"])
@pytest.mark.parametrize("shape", [(480, 640), (217, 333), (97, 131)])
def test_f32_pyramid_bit_exact(gpu, kind, shape):
    h, w = shape
    a, _, _ = _frames(kind, w, h)
    P = _dev_pyr(gpu, a, (21, 21), 3)
    R = O.Pyramid16(a, (21, 21), 3, f32=True)
    assert P.nlevels == R.nlevels
    for i in range(P.nlevels):
        got = P.level(i)
        assert got.dtype == np.float32
        assert np.array_equal(got.view(np.uint32), R.levels[i].view(np.uint32)), f"level {i}"
        assert np.array_equal(P.deriv(i).view(np.uint32), R.derivs[i].view(np.uint32)), f"deriv {i}"
        full = P.level(i, with_border=True)
        pad = P.pyr.lv[i].pad
        ref = R.levels[i]
        hh, ww = ref.shape
        ry = [O.load().orc_reflect101(y - pad, hh) for y in range(hh + 2 * pad)]
        rx = [O.load().orc_reflect101(x - pad, ww) for x in range(ww + 2 * pad)]
        assert np.array_equal(full.view(np.uint32), ref[np.ix_(ry, rx)].view(np.uint32)), f"border {i}"


@pytest.mark.parametrize("kind", ["u8", "u16", "f32"])
@pytest.mark.parametrize("win,maxlev", [(21, 3), (7, 0), (15, 2), (31, 1)])
def test_f32_lk_bit_exact(gpu, kind, win, maxlev):
    from opencv_amd import klt

    a, b, gt = _frames(kind, 640, 480, seed=win)
    pts = np.concatenate([box_points(gt[0], 32, seed=win), edge_points(640, 480)])
    Pa, Pb = _dev_pyr(gpu, a, (win, win), maxlev), _dev_pyr(gpu, b, (win, win), maxlev)
    lk = klt.SparsePyrLKOpticalFlow((win, win), maxlev, 30)
    r = lk.calc(Pa, Pb, to_dev(pts), want_iters=True)
    torch.cuda.synchronize()
    Ra, Rb = O.Pyramid16(a, (win, win), maxlev, f32=True), O.Pyramid16(b, (win, win), maxlev, f32=True)
    nx, st, er, it = O.lk16(Ra, Rb, pts, (win, win), maxlev)
    g_st = r.status.cpu().numpy()
    assert np.array_equal(g_st, st)
    ok = st == 1
    assert np.array_equal(r.next_pts.cpu().numpy()[ok].view(np.uint32), nx[ok].view(np.uint32))
    assert np.array_equal(r.err.cpu().numpy()[ok].view(np.uint32), er[ok].view(np.uint32))
    assert np.array_equal(r.iters.cpu().numpy(), it)


def test_f32_lk_flags_and_frames_from_torch(gpu):
    """initial flow / min-eigenvalue output; calc() on uint16 / float32 frames
    builds fp32 pyramids itself"""
    from opencv_amd import klt

    a, b, gt = _frames("u16", 320, 240, seed=3)
    pts = box_points(gt[0], 24, seed=3)
    init = pts + np.float32([1.5, -0.75])
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 3, 30, True)
    r = lk.calc(to_dev(a.view(np.int16)).view(torch.uint16), to_dev(b.view(np.int16)).view(torch.uint16),
                to_dev(pts), to_dev(init))
    torch.cuda.synchronize()
    nx, st, er, _ = O.lk16(O.Pyramid16(a, (21, 21), 3, f32=True), O.Pyramid16(b, (21, 21), 3, f32=True), pts,
                           flags=O.OPTFLOW_USE_INITIAL_FLOW, init=init)
    ok = st == 1
    assert np.array_equal(r.status.cpu().numpy(), st)
    assert np.array_equal(r.next_pts.cpu().numpy()[ok].view(np.uint32), nx[ok].view(np.uint32))
    lk2 = klt.SparsePyrLKOpticalFlow((21, 21), 3, 30, getMinEigenVals=True)
    af, bf, _ = _frames("f32", 320, 240, seed=3)
    r2 = lk2.calc(to_dev(af), to_dev(bf), to_dev(pts))
    torch.cuda.synchronize()
    nx2, st2, er2, _ = O.lk16(O.Pyramid16(af, (21, 21), 3, f32=True), O.Pyramid16(bf, (21, 21), 3, f32=True), pts,
                              flags=O.OPTFLOW_LK_GET_MIN_EIGENVALS)
    assert np.array_equal(r2.status.cpu().numpy(), st2)
    assert np.array_equal(r2.err.cpu().numpy().view(np.uint32), er2.view(np.uint32))


# ---- CV_16UC3/C4 and CV_32FC3/C4: the fp32 pixel path on cn interleaved channels
# (tbdk_pyr_create_f32_cn, klt_cn_f32.hip), bit-exact vs orc16_lk with cn channels


def _cn_frames(kind, cn, w, h, seed=11):
    frames, gt = O.synth(seed, w, h, 8, 0, 2)
    rng = np.random.default_rng(seed)
    out = []
    for f in frames[:2]:
        chans = [f.astype(np.float32)] + [(f.astype(np.float32) * (0.3 + 0.2 * c) + 25 * c) for c in range(1, cn)]
        img = np.stack(chans, 2)
        if kind == "u16":
            out.append((img * 257 + rng.integers(0, 200, img.shape)).clip(0, 65535).astype(np.uint16))
        elif kind == "u8":
            out.append(img.clip(0, 255).astype(np.uint8))
        else:  # fractional values at the u8 scale (minEig's 1e-4 gate is scale dependent)
            out.append((img + rng.normal(0, 0.25, img.shape)).astype(np.float32))
    return out[0], out[1], gt


def _cn_pyr(ctx, img, win, max_level):
    from opencv_amd import klt

    P = klt.Pyramid(ctx, img.shape[1], img.shape[0], max_level, win, torch.float32, channels=img.shape[2])
    t = to_dev(img.view(np.int16)).view(torch.uint16) if img.dtype == np.uint16 else to_dev(img)
    return P.build(t)


@pytest.mark.parametrize("kind,cn", [("f32", 3), ("f32", 4), ("u16", 3), ("u16", 4), ("u8", 3), ("f32", 2)])
def test_f32_cn_pyramid_bit_exact(gpu, kind, cn):
    a, _, _ = _cn_frames(kind, cn, 333, 217)
    P = _cn_pyr(gpu, a, (21, 21), 3)
    R = O.Pyramid16(a, (21, 21), 3, f32=True)
    assert P.nlevels == R.nlevels and P.channels == cn
    for i in range(P.nlevels):
        got = P.level(i)
        assert got.shape == R.levels[i].shape
        assert np.array_equal(got.view(np.uint32), R.levels[i].view(np.uint32)), f"level {i}"
        assert np.array_equal(P.deriv(i).view(np.uint32), R.derivs[i].view(np.uint32)), f"deriv {i}"
        full = P.level(i, with_border=True)
        pad = P.pyr.lv[i].pad
        hh, ww = R.levels[i].shape[:2]
        ry = [O.load().orc_reflect101(y - pad, hh) for y in range(hh + 2 * pad)]
        rx = [O.load().orc_reflect101(x - pad, ww) for x in range(ww + 2 * pad)]
        assert np.array_equal(full.view(np.uint32), R.levels[i][np.ix_(ry, rx)].view(np.uint32)), f"border {i}"


@pytest.mark.parametrize("kind,cn,win,maxlev", [("f32", 3, 21, 3), ("f32", 4, 21, 2), ("u16", 3, 15, 2),
                                                ("u16", 4, 31, 1), ("f32", 3, 7, 0), ("u16", 4, 9, 3),
                                                ("u16", 4, 45, 1)])  # > 64 KB of LDS: the opt-in path
def test_f32_cn_lk_bit_exact(gpu, kind, cn, win, maxlev):
    from opencv_amd import klt

    a, b, gt = _cn_frames(kind, cn, 320, 240, seed=win)
    pts = np.concatenate([box_points(gt[0], 24, seed=win), edge_points(320, 240)])
    Pa, Pb = _cn_pyr(gpu, a, (win, win), maxlev), _cn_pyr(gpu, b, (win, win), maxlev)
    Ra, Rb = O.Pyramid16(a, (win, win), maxlev, f32=True), O.Pyramid16(b, (win, win), maxlev, f32=True)
    for flags, init in ((0, None), (4, pts + np.float32([1.25, -0.5])), (8, None)):
        lk = klt.SparsePyrLKOpticalFlow((win, win), maxlev, 30, bool(flags & 4), getMinEigenVals=bool(flags & 8))
        r = lk.calc(Pa, Pb, to_dev(pts), None if init is None else to_dev(init), want_iters=True)
        torch.cuda.synchronize()
        nx, st, er, it = O.lk16(Ra, Rb, pts, (win, win), maxlev, flags=flags, init=init)
        assert np.array_equal(r.status.cpu().numpy(), st), flags
        ok = st == 1
        assert np.array_equal(r.next_pts.cpu().numpy()[ok].view(np.uint32), nx[ok].view(np.uint32)), flags
        assert np.array_equal(r.err.cpu().numpy()[ok].view(np.uint32), er[ok].view(np.uint32)), flags
        assert np.array_equal(r.iters.cpu().numpy(), it), flags
        if flags == 0:
            assert st.mean() > 0.7


def test_f32_cn_calc_on_frames_and_vs_u8_cn(gpu):
    """calc() on (H, W, 3) float32 frames builds the fp32 cn pyramids itself; the
    same frames as u8 through the u8 multi-channel path (exact integer sums,
    different arithmetic): >= 99 % of the points tracked by both within 1e-2 px"""
    from opencv_amd import klt

    a, b, gt = _cn_frames("u8", 3, 640, 480, seed=4)
    pts = box_points(gt[0], 48, seed=4)
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 3, 30)
    r32 = lk.calc(to_dev(a.astype(np.float32)), to_dev(b.astype(np.float32)), to_dev(pts))
    r8 = lk.calc(to_dev(a), to_dev(b), to_dev(pts))
    torch.cuda.synchronize()
    nx, st, _, _ = O.lk16(O.Pyramid16(a.astype(np.float32), f32=True), O.Pyramid16(b.astype(np.float32), f32=True),
                          pts)
    assert np.array_equal(r32.status.cpu().numpy(), st)
    s8, s32 = r8.status.cpu().numpy(), r32.status.cpu().numpy()
    both = (s8 == 1) & (s32 == 1)
    d = np.abs(r8.next_pts.cpu().numpy() - r32.next_pts.cpu().numpy())[both].max(1)
    assert (s8 == s32).mean() >= 0.99 and (d <= 1e-2).mean() >= 0.99


def test_f32_4k_bit_exact_sample(gpu):
    """the fp32 pixel path at configs[4]'s size: 4K float32 frames (u8 scale plus
    noise), 512 objects x 256 points, 3 levels; both pyramids whole (the
    role-split build, klt_pyr_fp.hip) and LK on a seeded 8192-point sample"""
    from opencv_amd import klt

    W, H, nobj = 3840, 2160, 512
    fr, gt = klt.synth_render(20261015, W, H, nobj, 0, 2, ctx=gpu)
    rng = np.random.default_rng(5)
    f = [(x.cpu().numpy().astype(np.float32) + rng.normal(0, 0.25, (H, W))).astype(np.float32) for x in fr]
    pts = box_points(gt[0].numpy(), 256)
    assert len(pts) == nobj * 256
    P0, P1 = _dev_pyr(gpu, f[0], (21, 21), 2), _dev_pyr(gpu, f[1], (21, 21), 2)
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)
    r = lk.calc(P0, P1, to_dev(pts), want_iters=True)
    torch.cuda.synchronize()
    R0, R1 = O.Pyramid16(f[0], (21, 21), 2, f32=True), O.Pyramid16(f[1], (21, 21), 2, f32=True)
    for P, R in ((P0, R0), (P1, R1)):
        assert P.nlevels == R.nlevels == 3
        for i in range(3):
            assert np.array_equal(P.level(i).view(np.uint32), R.levels[i].view(np.uint32)), f"level {i}"
            assert np.array_equal(P.deriv(i).view(np.uint32), R.derivs[i].view(np.uint32)), f"deriv {i}"
    idx = np.sort(np.random.default_rng(4).choice(len(pts), 8192, replace=False))
    nx, st, er, it = O.lk16(R0, R1, pts[idx], (21, 21), 2, nthreads=16)
    g_st = r.status.cpu().numpy()[idx]
    assert np.array_equal(g_st, st)
    ok = st == 1
    assert np.array_equal(r.next_pts.cpu().numpy()[idx][ok].view(np.uint32), nx[ok].view(np.uint32))
    assert np.array_equal(r.err.cpu().numpy()[idx][ok].view(np.uint32), er[ok].view(np.uint32))
    assert np.array_equal(r.iters.cpu().numpy()[idx], it)
    assert st.mean() > 0.9
