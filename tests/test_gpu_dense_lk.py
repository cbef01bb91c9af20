"""Dense PyrLK (tbdk_lk_dense, cv::cuda::DensePyrLKOpticalFlow's interface) vs
the CPU oracle's calcOpticalFlowPyrLK at every pixel: bit-exact against the
oracle's exact-sum mode, as the sparse path (tests/test_gpu_klt.py)."""
import numpy as np
import pytest
import torch

import _oracle as O

pytestmark = pytest.mark.gpu


def _grid(w, h):
    ys, xs = np.mgrid[0:h, 0:w]
    return np.stack([xs.ravel(), ys.ravel()], 1).astype(np.float32)


@pytest.mark.parametrize("w,h,win,max_level", [(160, 120, 13, 3), (96, 72, 21, 2), (131, 77, 9, 1)])
def test_dense_matches_oracle_at_every_pixel(gpu, w, h, win, max_level):
    from opencv_amd import klt

    fr, _ = O.synth(31 + w, w, h, 4, 0, 2)
    lk = klt.DensePyrLKOpticalFlow.create((win, win), max_level, 30)
    flow, status = lk.calc(torch.from_numpy(fr[0]).cuda(), torch.from_numpy(fr[1]).cuda(), want_status=True)
    torch.cuda.synchronize()
    flow, status = flow.cpu().numpy(), status.cpu().numpy()
    pts = _grid(w, h)
    # the dense interface has no err output: calcOpticalFlowPyrLK with err = noArray()
    nx, st, _, _ = O.lk(O.Pyramid(fr[0], (win, win), max_level), O.Pyramid(fr[1], (win, win), max_level), pts,
                        win=(win, win), max_level=max_level, accum=O.ACCUM_EXACT, want_err=False)
    assert np.array_equal(status.ravel(), st)
    ok = st == 1
    ref = (nx - pts).astype(np.float32)
    assert np.array_equal(flow.reshape(-1, 2)[ok], ref[ok])


def test_dense_recovers_translation(gpu):
    from opencv_amd import klt

    fr, _ = O.synth(5, 640, 480, 12, 0, 1)
    a = fr[0]
    b = np.roll(a, (2, -3), axis=(0, 1))  # content moves by (-3, +2)
    flow, status = klt.DensePyrLKOpticalFlow.create().calc(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(),
                                                           want_status=True)
    torch.cuda.synchronize()
    f = flow.cpu().numpy()[32:-32, 32:-32]
    s = status.cpu().numpy()[32:-32, 32:-32] == 1
    assert s.mean() > 0.9
    assert abs(np.median(f[..., 0][s]) + 3) < 0.01 and abs(np.median(f[..., 1][s]) - 2) < 0.01


def test_dense_rejects_bad_arguments(gpu):
    from opencv_amd import _lib, klt

    a = torch.zeros((64, 64), dtype=torch.uint8, device="cuda")
    with pytest.raises(_lib.TbdkError):  # CV_Assert(winSize > 2), pyrlk.cpp:243
        klt.DensePyrLKOpticalFlow.create((2, 13)).calc(a, a)
    with pytest.raises(_lib.TbdkError):
        klt.DensePyrLKOpticalFlow.create().calc(a, a, flow=torch.empty((64, 64, 2), device="cuda")[:, :32])


def test_dense_ignores_use_initial_flow(gpu):
    """PyrLKOpticalFlowBase::dense never reads the incoming flow (pyrlk.cpp:238-299)."""
    from opencv_amd import klt

    fr, _ = O.synth(7, 96, 64, 4, 0, 2)
    a, b = torch.from_numpy(fr[0]).cuda(), torch.from_numpy(fr[1]).cuda()
    ref = klt.DensePyrLKOpticalFlow.create().calc(a, b)
    seeded = torch.full((64, 96, 2), 5.0, device="cuda")
    out = klt.DensePyrLKOpticalFlow.create(useInitialFlow=True).calc(a, b, flow=seeded)
    torch.cuda.synchronize()
    assert torch.equal(ref, out)


@pytest.mark.parametrize("w,h,win,max_level", [(640, 480, 13, 3), (331, 187, 21, 2), (200, 150, 7, 4), (160, 120, 31, 5),
                                                (64, 48, 9, 0), (97, 61, 15, 3)])
def test_dense_case_images_equal_per_point_setup(gpu, w, h, win, max_level):
    """The dense path's case images (every window read from the per-phase
    interpolated images, ctx option lk_dense_case = 1, the default) against the
    per-point setup of the sparse kernels over the pixel grid (lk_dense_case =
    0): the same flow and status at every pixel, the flow of failed points
    included."""
    from opencv_amd import klt

    fr, _ = O.synth(7 + w, w, h, 12, 0, 2)
    a, b = torch.from_numpy(fr[0]).cuda(), torch.from_numpy(fr[1]).cuda()
    out = {}
    try:
        for mode in (1, 0):
            gpu.set_option("lk_dense_case", mode)
            lk = klt.DensePyrLKOpticalFlow.create((win, win), max_level, 30)
            flow, status = lk.calc(a, b, want_status=True)
            torch.cuda.synchronize()
            out[mode] = (flow.cpu().numpy(), status.cpu().numpy())
    finally:
        gpu.set_option("lk_dense_case", 1)
    assert np.array_equal(out[1][1], out[0][1])
    assert np.array_equal(out[1][0].view(np.uint32), out[0][0].view(np.uint32))
    assert out[1][1].mean() > 0.5
