"""GPU parity tests of the fp16 pixel path (BASELINE configs[4]).

The reference has no fp16 (or fp32) CPU PyrLK, so the checker is the fp32
restatement oracle/klt16_oracle.c (LKTrackerInvoker's algorithm on fp16 pixels,
one fixed operation order).  Bars:
  * fp16 levels (interior + reflect-101 frame) and fp16 derivative planes:
    bit-exact vs the oracle, from u8 and from fp16 frames, odd sizes included;
  * sparse LK: bit-exact next_pts / status / err / iteration counts vs the
    oracle (every window size the kernel has, level counts 0-3, initial flow,
    min-eigenvalue output, points outside the image);
  * the fp16 path against the 8-bit path on the same frames (different
    arithmetic): >= 99 % of points tracked by both within 1e-2 px, status
    agreement >= 99.5 % — at 640x480 and at BASELINE configs[4]'s 4K size;
  * BASELINE configs[4] itself (3840x2160, 512 objects x 256 points, the
    bench's lk_f16 leg): both fp16 pyramids bit-exact, and the GPU's LK over
    all 131k points bit-exact vs the oracle on a seeded 8192-point sample
    (every point's result depends only on its own inputs).
"""
import ctypes as C

import numpy as np
import pytest
import torch

import _oracle as O

pytestmark = pytest.mark.gpu


def K():
    from opencv_amd import klt

    return klt


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def box_points(gt, n_per_box, seed=0):
    rng = np.random.default_rng(seed)
    pts = []
    for v, x, y, w, h in gt:
        if v:
            pts.append(np.stack([rng.uniform(x, x + w, n_per_box), rng.uniform(y, y + h, n_per_box)], 1))
    return np.concatenate(pts).astype(np.float32)


def edge_points(w, h):
    """points at and beyond the borders (bounds gates, reflect-101 / zero frames)"""
    xs = np.array([-30.0, -10.5, -0.3, 0.0, 3.25, w / 2, w - 4.5, w - 1.0, w - 0.01, w + 2.0, w + 25.0])
    ys = np.array([-25.0, -1.0, 0.0, 9.75, h / 3, h - 1.5, h - 0.2, h + 12.0])
    gx, gy = np.meshgrid(xs, ys)
    return np.stack([gx.ravel(), gy.ravel()], 1).astype(np.float32)


def dev_pyr(ctx, img, win, max_level):
    return K().Pyramid(ctx, img.shape[1], img.shape[0], max_level, win, torch.float16).build(to_dev(img))


@pytest.mark.parametrize("shape", [(480, 640), (217, 333), (97, 131)])
def test_f16_pyramid_bit_exact_from_u8(gpu, shape):
    h, w = shape
    frames, _ = O.synth(7, w, h, 6, 0, 1)
    img = frames[0]
    P = dev_pyr(gpu, img, (21, 21), 3)
    R = O.Pyramid16(img, (21, 21), 3)
    assert P.nlevels == R.nlevels
    for i in range(P.nlevels):
        got = P.level(i)
        assert got.dtype == np.float16
        assert np.array_equal(got.view(np.uint16), R.levels[i].view(np.uint16)), f"level {i}"
        assert np.array_equal(P.deriv(i).view(np.uint16), R.derivs[i].view(np.uint16)), f"deriv {i}"
        # the padded frame holds BORDER_REFLECT_101 values of the level
        full = P.level(i, with_border=True)
        pad = P.pyr.lv[i].pad
        ref = R.levels[i]
        hh, ww = ref.shape
        ry = [O.load().orc_reflect101(y - pad, hh) for y in range(hh + 2 * pad)]
        rx = [O.load().orc_reflect101(x - pad, ww) for x in range(ww + 2 * pad)]
        assert np.array_equal(full.view(np.uint16), ref[np.ix_(ry, rx)].view(np.uint16)), f"border {i}"


def test_f16_pyramid_bit_exact_from_f16(gpu):
    rng = np.random.default_rng(3)
    h, w = 301, 455
    img = (rng.uniform(0, 255, (h, w)) + rng.uniform(0, 1, (h, w))).astype(np.float16)
    img[:5, :7] = np.float16(1e-6)  # fp16 subnormals
    P = K().Pyramid(gpu, w, h, 3, (15, 15), torch.float16).build(to_dev(img))
    R = O.Pyramid16(img, (15, 15), 3)
    assert P.nlevels == R.nlevels
    for i in range(P.nlevels):
        assert np.array_equal(P.level(i).view(np.uint16), R.levels[i].view(np.uint16)), f"level {i}"
        assert np.array_equal(P.deriv(i).view(np.uint16), R.derivs[i].view(np.uint16)), f"deriv {i}"


def run_gpu_lk(ctx, P0, P1, pts, win, max_level, flags=0, init=None, max_count=30, eps=0.01, min_eig=1e-4):
    lk = K().SparsePyrLKOpticalFlow(win, max_level, max_count, useInitialFlow=bool(flags & 4), epsilon=eps,
                                    minEigThreshold=min_eig, getMinEigenVals=bool(flags & 8))
    r = lk.calc(P0, P1, to_dev(pts), None if init is None else to_dev(init), want_iters=True)
    torch.cuda.synchronize()
    return r.next_pts.cpu().numpy(), r.status.cpu().numpy(), r.err.cpu().numpy(), r.iters.cpu().numpy()


def assert_same(got, ref, tag=""):
    g_nx, g_st, g_er, g_it = got
    nx, st, er, it = ref
    assert np.array_equal(g_st, st), f"{tag} status"
    assert np.array_equal(g_nx.view(np.uint32), nx.view(np.uint32)), f"{tag} next_pts"
    assert np.array_equal(g_er.view(np.uint32), er.view(np.uint32)), f"{tag} err"
    assert np.array_equal(g_it, it), f"{tag} iters"


@pytest.mark.parametrize("win,max_level", [(21, 3), (21, 0), (7, 2), (15, 1), (31, 3), (9, 3)])
def test_f16_lk_bit_exact(gpu, win, max_level):
    frames, gt = O.synth(20261015, 640, 480, 32, 0, 2)
    pts = np.concatenate([box_points(gt[0], 24), edge_points(640, 480)])
    P0 = dev_pyr(gpu, frames[0], (win, win), max_level)
    P1 = dev_pyr(gpu, frames[1], (win, win), max_level)
    R0, R1 = O.Pyramid16(frames[0], (win, win), max_level), O.Pyramid16(frames[1], (win, win), max_level)
    got = run_gpu_lk(gpu, P0, P1, pts, (win, win), max_level)
    ref = O.lk16(R0, R1, pts, (win, win), max_level)
    assert_same(got, ref, f"win {win} L{max_level}")
    assert got[1].mean() > 0.8


def test_f16_lk_flags_bit_exact(gpu):
    frames, gt = O.synth(11, 640, 480, 24, 5, 2)
    pts = box_points(gt[0], 32, seed=1)
    P0, P1 = dev_pyr(gpu, frames[0], (21, 21), 3), dev_pyr(gpu, frames[1], (21, 21), 3)
    R0, R1 = O.Pyramid16(frames[0]), O.Pyramid16(frames[1])
    init = pts + np.float32([1.5, -0.75])
    for flags, init_ in ((4, init), (8, None), (12, init)):
        got = run_gpu_lk(gpu, P0, P1, pts, (21, 21), 3, flags=flags, init=init_)
        ref = O.lk16(R0, R1, pts, (21, 21), 3, flags=flags, init=init_)
        assert_same(got, ref, f"flags {flags}")
    # criteria: one iteration, tight and loose eps, a high min-eigenvalue gate
    for mc, eps, me in ((1, 0.01, 1e-4), (30, 0.0, 1e-4), (30, 1.0, 1e-4), (30, 0.01, 5e-3)):
        got = run_gpu_lk(gpu, P0, P1, pts, (21, 21), 3, max_count=mc, eps=eps, min_eig=me)
        ref = O.lk16(R0, R1, pts, (21, 21), 3, max_count=mc, eps=eps, min_eig=me)
        assert_same(got, ref, f"criteria {mc} {eps} {me}")


def test_f16_lk_from_f16_frames_bit_exact(gpu):
    """fp16 frames with fractional values (build_f16) through the same kernel"""
    frames, gt = O.synth(5, 640, 480, 16, 0, 2)
    rng = np.random.default_rng(2)
    f16 = [(f.astype(np.float32) + rng.uniform(-0.5, 0.5, f.shape)).clip(0, 255).astype(np.float16) for f in frames]
    pts = box_points(gt[0], 48)
    P0 = K().build_pyramid(to_dev(f16[0]), (21, 21), 3, ctx=gpu)
    P1 = K().build_pyramid(to_dev(f16[1]), (21, 21), 3, ctx=gpu)
    assert P0.dtype == torch.float16
    got = run_gpu_lk(gpu, P0, P1, pts, (21, 21), 3)
    ref = O.lk16(O.Pyramid16(f16[0]), O.Pyramid16(f16[1]), pts)
    assert_same(got, ref, "fp16 frames")


def compare_with_u8_path(gpu, W, H, nobj, per_box, max_level):
    frames, gt = K().synth_render(20261015, W, H, nobj, 0, 2, ctx=gpu)
    pts = box_points(gt[0].numpy(), per_box)
    lk = K().SparsePyrLKOpticalFlow((21, 21), max_level, 30)
    r8 = lk.calc(frames[0], frames[1], to_dev(pts))
    P0 = K().build_pyramid(frames[0], (21, 21), max_level, ctx=gpu, dtype=torch.float16)
    P1 = K().build_pyramid(frames[1], (21, 21), max_level, ctx=gpu, dtype=torch.float16)
    r16 = lk.calc(P0, P1, to_dev(pts))
    torch.cuda.synchronize()
    s8, s16 = r8.status.cpu().numpy(), r16.status.cpu().numpy()
    both = (s8 == 1) & (s16 == 1)
    d = np.abs(r8.next_pts.cpu().numpy() - r16.next_pts.cpu().numpy())[both].max(1)
    assert (s8 == s16).mean() >= 0.995
    assert (d <= 1e-2).mean() >= 0.99, f"{(d <= 1e-2).mean()}"
    return len(pts), d


def test_f16_vs_u8_path_640(gpu):
    n, d = compare_with_u8_path(gpu, 640, 480, 32, 64, 3)
    assert n > 1500 and np.median(d) < 1e-3


def test_f16_vs_u8_path_4k(gpu):
    """BASELINE configs[4] shape: 3840x2160, 512 objects x 256 points, 3 levels"""
    n, d = compare_with_u8_path(gpu, 3840, 2160, 512, 256, 2)
    assert n > 100000


def test_f16_4k_bit_exact_sample(gpu):
    """configs[4]: 4K, 512 objects x 256 points (131,072), 3 levels (max_level 2 as the
    bench's lk_f16 leg); pyramids whole, LK on a seeded 8192-point sample"""
    W, H, nobj = 3840, 2160, 512
    frames, gt = K().synth_render(20261015, W, H, nobj, 0, 2, ctx=gpu)
    pts = box_points(gt[0].numpy(), 256)
    assert len(pts) == nobj * 256
    P0 = K().build_pyramid(frames[0], (21, 21), 2, ctx=gpu, dtype=torch.float16)
    P1 = K().build_pyramid(frames[1], (21, 21), 2, ctx=gpu, dtype=torch.float16)
    got = run_gpu_lk(gpu, P0, P1, pts, (21, 21), 2)
    f = frames.cpu().numpy()
    R0, R1 = O.Pyramid16(f[0], (21, 21), 2), O.Pyramid16(f[1], (21, 21), 2)
    for P, R in ((P0, R0), (P1, R1)):
        assert P.nlevels == R.nlevels == 3
        for i in range(3):
            assert np.array_equal(P.level(i).view(np.uint16), R.levels[i].view(np.uint16)), f"level {i}"
            assert np.array_equal(P.deriv(i).view(np.uint16), R.derivs[i].view(np.uint16)), f"deriv {i}"
    idx = np.sort(np.random.default_rng(4).choice(len(pts), 8192, replace=False))
    ref = O.lk16(R0, R1, pts[idx], (21, 21), 2, nthreads=16)
    assert_same(tuple(a[idx] for a in got), ref, "4K sample")
    assert got[1].mean() > 0.9


def test_f16_argument_checks(gpu):
    from opencv_amd import _lib

    k = K()
    frames, _ = O.synth(1, 320, 240, 4, 0, 2)
    P8 = k.Pyramid(gpu, 320, 240, 2, (21, 21)).build(to_dev(frames[0]))
    P16 = dev_pyr(gpu, frames[1], (21, 21), 2)
    pts = to_dev(np.float32([[100, 100], [50, 60]]))
    with pytest.raises(_lib.TbdkError):  # mixed depths
        k.SparsePyrLKOpticalFlow((21, 21), 2).calc(P8, P16, pts)
    with pytest.raises(_lib.TbdkError):  # the fp16 path has one kernel
        k.SparsePyrLKOpticalFlow((21, 21), 2, impl=3).calc(P16, P16, pts)
    with pytest.raises(_lib.TbdkError):  # no instantiation for even windows
        k.SparsePyrLKOpticalFlow((20, 20), 2).calc(P16, P16, pts)
    img16 = to_dev(frames[0].astype(np.float16))
    rc = gpu.lib.tbdk_pyr_build_f16(gpu.handle, C.c_void_p(img16.data_ptr()), 640, C.byref(P8.pyr), None)
    assert rc == -1  # TBDK_EINVAL: fp16 frame into a u8 pyramid
    rc = gpu.lib.tbdk_pyr_build_f16(gpu.handle, C.c_void_p(img16.data_ptr()), 639, C.byref(P16.pyr), None)
    assert rc == -1  # odd / short pitch
