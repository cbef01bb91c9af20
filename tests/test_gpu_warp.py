"""warpAffine on the GPU vs the CPU oracle: bit-exact (integer fixed-point path)."""
import numpy as np
import pytest
import torch

import _oracle as O
from test_warp_oracle import rotation_matrix

pytestmark = pytest.mark.gpu


def run(gpu, src, M, dsize, flags, border, bval, init=None):
    from opencv_amd import klt

    s = torch.from_numpy(src).cuda()
    d = None if init is None else torch.from_numpy(init).cuda()
    out = klt.warp_affine(s, M, dsize, flags, border, bval, dst=d, ctx=gpu)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("inter", [O.INTER_NEAREST, O.INTER_LINEAR, O.INTER_CUBIC, O.INTER_AREA])
@pytest.mark.parametrize("border", [O.BORDER_CONSTANT, O.BORDER_REPLICATE, O.BORDER_REFLECT, O.BORDER_WRAP,
                                    O.BORDER_REFLECT_101, O.BORDER_TRANSPARENT])
@pytest.mark.parametrize("inverse", [False, True])
def test_warp_matches_oracle(gpu, inter, border, inverse):
    rng = np.random.default_rng(100 + inter * 17 + border * 3 + inverse)
    for _ in range(3):
        sw, sh = int(rng.integers(8, 300)), int(rng.integers(8, 200))
        dw, dh = int(rng.integers(1, 320)), int(rng.integers(1, 220))
        src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
        M = rotation_matrix(sw / 2.0, sh / 2.0, float(rng.uniform(-180, 180)), float(rng.uniform(0.4, 2.0)))
        M[:, 2] += rng.uniform(-20, 20, 2)
        flags = inter | (O.WARP_INVERSE_MAP if inverse else 0)
        bval = int(rng.integers(0, 256))
        init = rng.integers(0, 256, (dh, dw), dtype=np.uint8)
        got = run(gpu, src, M, (dw, dh), flags, border, bval, init)
        ref = O.warp_affine(src, M, (dw, dh), flags, border, bval, dst=init)
        assert np.array_equal(got, ref)


def test_warp_1080p_box_propagation(gpu):
    """Full-frame warp of a synthetic 1080p frame by a small similarity (the TBD
    box-propagation shape), plus degenerate and extreme matrices."""
    fr, _ = O.synth(20261015, 1920, 1080, 16, 0, 1)
    src = fr[0]
    a = np.deg2rad(0.8)
    M = np.array([[1.01 * np.cos(a), -1.01 * np.sin(a), 2.5], [1.01 * np.sin(a), 1.01 * np.cos(a), -1.75]])
    for flags in (O.INTER_LINEAR, O.INTER_NEAREST | O.WARP_INVERSE_MAP, O.INTER_CUBIC):
        got = run(gpu, src, M, (1920, 1080), flags, O.BORDER_REFLECT_101, 0)
        assert np.array_equal(got, O.warp_affine(src, M, (1920, 1080), flags, O.BORDER_REFLECT_101, 0))
    for M in (np.zeros((2, 3)), np.array([[1e6, 0, 0], [0, 1e-7, 5e9]]), np.array([[0, 1, 0], [1, 0, 0]])):
        small = src[:64, :96].copy()
        for inter in (O.INTER_LINEAR, O.INTER_CUBIC):
            got = run(gpu, small, M, (70, 50), inter, O.BORDER_CONSTANT, 3)
            assert np.array_equal(got, O.warp_affine(small, M, (70, 50), inter, O.BORDER_CONSTANT, 3))


def test_warp_rejects_bad_arguments(gpu):
    from opencv_amd import _lib, klt

    s = torch.zeros((10, 10), dtype=torch.uint8, device="cuda")
    with pytest.raises(_lib.TbdkError):
        klt.warp_affine(s, np.eye(2, 3), (10, 10), flags=4, ctx=gpu)  # INTER_LANCZOS4 unsupported
    with pytest.raises(_lib.TbdkError):
        klt.warp_affine(s, np.eye(2, 3), (10, 10), borderMode=7, ctx=gpu)
    with pytest.raises(_lib.TbdkError):
        klt.warp_affine(s, np.eye(2, 3), (10, 10), dst=s, ctx=gpu)  # aliasing
