"""HOG people detector on the GPU (libtbdk hog.hip) vs the CPU oracle
(oracle/hog_oracle.c, the HOGDescriptor restatement): bit-exact at every stage
(INTER_LINEAR_EXACT levels, gradients and bins, normalized block histograms,
window scores as doubles) and equal detection sets after grouping."""
import numpy as np
import pytest
import torch

import _oracle as O

pytestmark = pytest.mark.gpu


def _bgr(seed, w, h, cn=3):
    fr, _ = O.synth(seed, w, h, 8, 0, 1)
    g = fr[0].astype(np.int32)
    if cn == 1:
        return g.astype(np.uint8)
    rng = np.random.default_rng(seed)
    chans = [np.clip(g + rng.integers(-30, 30, g.shape), 0, 255) for _ in range(cn)]
    return np.stack(chans, 2).astype(np.uint8)


def _hog(gpu, win=(64, 128), **kw):
    from opencv_amd import hog

    h = hog.HOG.create(win, ctx=gpu, **kw)
    h.setSVMDetector(h.getDefaultPeopleDetector())
    return h


def _prm(h):
    p = h.p
    return O.hog_params(win=(p.win_w, p.win_h), block=(p.block_w, p.block_h),
                        bstride=(p.block_stride_x, p.block_stride_y), cell=(p.cell_w, p.cell_h), nbins=p.nbins,
                        win_sigma=p.win_sigma, l2hys=p.l2hys_threshold, gamma=bool(p.gamma_correction),
                        signed=bool(p.signed_gradient), wstride=(p.win_stride_x, p.win_stride_y))


@pytest.mark.parametrize("cn", [1, 3, 4])
@pytest.mark.parametrize("src,dst", [((640, 480), (610, 457)), ((1242, 375), (1183, 357)), ((97, 61), (31, 20)),
                                     ((50, 40), (123, 77))])
def test_resize_exact_bit_exact(gpu, cn, src, dst):
    from opencv_amd import hog

    img = _bgr(sum(src) + cn, *src, cn=cn)
    got = hog.resize_exact(torch.from_numpy(img).cuda(), dst, ctx=gpu).cpu().numpy()
    assert np.array_equal(got, O.hog_resize(img, dst))


@pytest.mark.parametrize("cn", [1, 3, 4])
@pytest.mark.parametrize("w,h", [(640, 480), (130, 77), (15, 33), (6, 5), (1031, 9), (2050, 7), (1040, 5)])
@pytest.mark.parametrize("gamma,signed", [(True, False), (False, True)])
def test_gradient_bit_exact(gpu, cn, w, h, gamma, signed):
    from opencv_amd import hog

    img = _bgr(w * h + cn, w, h, cn=cn)
    hg = _hog(gpu)
    hg.setGammaCorrection(gamma)
    hg.setSignedGradient(signed)
    g, q = hog.gradient(torch.from_numpy(img).cuda(), hg, ctx=gpu)
    og, oq = O.hog_gradient(img[..., :3] if cn == 4 else img, nbins=9, gamma=gamma, signed=signed)
    assert np.array_equal(q.cpu().numpy(), oq)
    assert np.array_equal(g.cpu().numpy(), og)


@pytest.mark.parametrize("geom", [dict(), dict(block_size=(16, 16), cell_size=(4, 4), nbins=9, win_size=(64, 128)),
                                  dict(nbins=18, win_size=(64, 128)), dict(block_stride=(4, 4), win_size=(48, 96))])
def test_blocks_bit_exact(gpu, geom):
    from opencv_amd import hog

    img = _bgr(7, 200, 150, cn=1)
    hg = hog.HOG.create(ctx=gpu, **geom)
    og, oq = O.hog_gradient(img, nbins=hg.p.nbins)
    B = hog.blocks(torch.from_numpy(og).cuda(), torch.from_numpy(oq).cuda(), hg, ctx=gpu).cpu().numpy()
    assert np.array_equal(B, O.hog_blocks(og, oq, _prm(hg)))


@pytest.mark.parametrize("w,h,bstride", [(300, 170, (8, 8)), (16, 16, (8, 8)), (151, 97, (4, 4)), (777, 41, (8, 8))])
def test_blocks_tiled_kernel_bit_exact(gpu, w, h, bstride):
    """hog_block_tile_kernel (2x2 cells, 9 bins): ragged last tiles in x and y, a single
    block, block stride 4; equal to the oracle, to the register-bin variant (option 2) and
    to the per-cell kernel (option 0)"""
    from opencv_amd import hog

    img = _bgr(w + 3 * h, w, h, cn=1)
    hg = hog.HOG.create(ctx=gpu, block_stride=bstride, win_size=(48, 96) if bstride[0] == 4 else (64, 128))
    og, oq = O.hog_gradient(img, nbins=9)
    G, Q = torch.from_numpy(og).cuda(), torch.from_numpy(oq).cuda()
    B = hog.blocks(G, Q, hg, ctx=gpu).cpu().numpy()
    assert np.array_equal(B, O.hog_blocks(og, oq, _prm(hg)))
    try:
        for opt in (0, 2):
            gpu.set_option("hog_block_tiled", opt)
            assert np.array_equal(B, hog.blocks(G, Q, hg, ctx=gpu).cpu().numpy()), opt
    finally:
        gpu.set_option("hog_block_tiled", 1)


@pytest.mark.parametrize("win", [(64, 128), (48, 96)])
@pytest.mark.parametrize("cn", [1, 3])
def test_detect_scores_bit_exact(gpu, win, cn):
    img = _bgr(11 + cn, 320, 240, cn=cn)
    hg = _hog(gpu, win)
    hg.setHitThreshold(-1e9)  # every window
    xy, sc = hg.detect(torch.from_numpy(img).cuda(), confidences=True)
    oxy, osc = O.hog_detect(img, _prm(hg), hg.svm, hit_threshold=-1e9)
    assert len(xy) == len(oxy)
    assert np.array_equal(np.array(xy), oxy) and np.array_equal(np.array(sc), osc)


@pytest.mark.parametrize("win,cn,hit,group", [((64, 128), 3, -2.2, 2), ((48, 96), 3, -1.0, 2), ((64, 128), 1, -1.6, 0),
                                              ((48, 96), 4, -0.9, 4)])
def test_detect_multiscale_equals_oracle(gpu, win, cn, hit, group):
    """The sample's call: 15 levels, scale 1.05, win stride 8 (tbd.cpp:425-431, 596-606)."""
    img = _bgr(20 + cn, 640, 360, cn=cn)
    hg = _hog(gpu, win)
    hg.setNumLevels(15)
    hg.setHitThreshold(hit)
    hg.setGroupThreshold(group)
    rects, wts = hg.detectMultiScale(torch.from_numpy(img).cuda(), confidences=True)
    ref = img[..., :3] if cn == 4 else img
    orects, owts = O.hog_detect_multiscale(ref, _prm(hg), hg.svm, hit_threshold=hit, nlevels=15, scale0=1.05,
                                           group_threshold=group)
    got = sorted(zip(rects, wts))
    exp = sorted(zip(map(tuple, orects.tolist()), owts.tolist()))
    assert len(exp) > 0
    assert got == exp


def test_detector_change_between_calls(gpu):
    """The detector and the cell plan are uploaded only when they change (host copies
    compared): a new detector of the same size, then the old one again, each equal to
    the oracle's scores"""
    img = _bgr(5, 320, 240, cn=3)
    hg = _hog(gpu)
    hg.setHitThreshold(-1e9)
    d0 = list(hg.svm)
    d1 = [v * 0.5 for v in d0]
    for d in (d0, d1, d0):
        hg.setSVMDetector(d)
        xy, sc = hg.detect(torch.from_numpy(img).cuda(), confidences=True)
        oxy, osc = O.hog_detect(img, _prm(hg), hg.svm, hit_threshold=-1e9)
        assert np.array_equal(np.array(xy), oxy) and np.array_equal(np.array(sc), osc)


@pytest.mark.parametrize("lanes", [1, 2, 4])
def test_detect_multiscale_level_streams_equal(gpu, lanes):
    """ctx option hog_level_streams: the levels' chains on 1, 2 or 4 streams give the
    default (3 streams) result, here on frames of two sizes back to back"""
    hg = _hog(gpu, (48, 96))
    hg.setNumLevels(15)
    hg.setHitThreshold(-0.5)
    imgs = [torch.from_numpy(_bgr(31, 640, 360, cn=4)).cuda(), torch.from_numpy(_bgr(32, 800, 450, cn=4)).cuda()]
    ref = [hg.detectMultiScale(im, confidences=True) for im in imgs]
    assert sum(len(r[0]) for r in ref) > 0
    try:
        gpu.set_option("hog_level_streams", lanes)
        got = [hg.detectMultiScale(im, confidences=True) for im in imgs]
    finally:
        gpu.set_option("hog_level_streams", 3)
    assert got == ref
    with pytest.raises(Exception):
        gpu.set_option("hog_level_streams", 5)


@pytest.mark.parametrize("win", [(64, 128), (48, 96)])
def test_window_pass_tiled_equals_per_window(gpu, win):
    """ctx option hog_window_tiled: the LDS-tiled window pass (rows of 16 windows,
    ragged last tiles) and the per-window pass give the same rects and weights;
    the tiled pass really runs for both detectors (the 64 x 128 default's tile
    takes ~76 KB of LDS), counted through the "hog_window_tile" timing name"""
    hg = _hog(gpu, win)
    hg.setNumLevels(15)
    hg.setHitThreshold(-1.5)
    hg.setGroupThreshold(0)
    im = torch.from_numpy(_bgr(41, 700, 420, cn=3)).cuda()

    def run():
        gpu.timing_select(["hog_window_tile"])
        gpu.timing_enable(True)
        try:
            r = hg.detectMultiScale(im, confidences=True)
            return r, gpu.timing_calls("hog_window_tile")
        finally:
            gpu.timing_enable(False)
            gpu.timing_select(None)

    ref, tiled = run()
    assert len(ref[0]) > 0 and tiled > 0
    try:
        gpu.set_option("hog_window_tiled", 0)
        got, tiled0 = run()
    finally:
        gpu.set_option("hog_window_tiled", 1)
    assert got == ref and tiled0 == 0


def test_rejects_bad_arguments(gpu):
    from opencv_amd import _lib, hog

    with pytest.raises(_lib.TbdkError):
        hog.HOG.create((60, 128))                        # (win - block) % stride != 0
    hg = _hog(gpu)
    with pytest.raises(_lib.TbdkError):
        hg.setSVMDetector(np.zeros(100, np.float32))     # wrong detector size
    with pytest.raises(_lib.TbdkError):
        hg.detectMultiScale(torch.zeros((64, 64, 2), dtype=torch.uint8, device="cuda"))
    with pytest.raises(_lib.TbdkError):
        hog.HOG.create((32, 32)).getDefaultPeopleDetector()
    small = torch.zeros((60, 40), dtype=torch.uint8, device="cuda")  # smaller than the window
    assert hg.detectMultiScale(small) == []
