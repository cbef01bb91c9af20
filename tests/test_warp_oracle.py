"""Pin the warpAffine oracle (oracle/warp_oracle.c) against the reference
test's own validator, restated in numpy: CV_WarpAffine_Test::warpAffine
(modules/imgproc/test/test_imgwarp_strict.cpp:1105-1156) builds the same
10-bit fixed-point map, and CV_Remap_Test::remap_nearest / remap_generic
(:881-1003) resample it with float weights and borderInterpolate; accepted
within get_success_error_level (:233-245, 1 LSB).  Test matrices follow
generate_test_data (:1058-1082): getRotationMatrix2D about the centre, angle in
[-180, 180), scale in [0.4, 2), optionally WARP_INVERSE_MAP."""
import math

import numpy as np
import pytest

import _oracle as O


def rotation_matrix(cx, cy, angle_deg, scale):
    """cv::getRotationMatrix2D (imgproc/src/imgwarp.cpp getRotationMatrix2D)."""
    a = math.radians(angle_deg)
    alpha, beta = math.cos(a) * scale, math.sin(a) * scale
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy],
                     [-beta, alpha, beta * cx + (1 - alpha) * cy]], np.float64)


def border_interp(p, n, border):
    if 0 <= p < n:
        return p
    if border == O.BORDER_CONSTANT:
        return -1
    if border == O.BORDER_REPLICATE:
        return 0 if p < 0 else n - 1
    if border in (O.BORDER_REFLECT, O.BORDER_REFLECT_101):
        d = 1 if border == O.BORDER_REFLECT_101 else 0
        if n == 1:
            return 0
        while not 0 <= p < n:
            p = -p - 1 + d if p < 0 else n - 1 - (p - n) - d
        return p
    raise ValueError("WRAP is handled by border_interp_c")


def c_div(a, b):  # C integer division (truncation toward zero)
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def border_interp_c(p, n, border):
    if border == O.BORDER_WRAP and not 0 <= p < n:
        if p < 0:
            p -= c_div(p - n + 1, n) * n
        if p >= n:
            p %= n
        return p
    return border_interp(p, n, border)


def ref_test_maps(M, dsize, inter, inverse):
    """CV_WarpAffine_Test::warpAffine map generation (:1126-1152)."""
    tM = np.asarray(M, np.float64).reshape(2, 3)
    if not inverse:
        tM = O.invert_affine(tM)
    t = tM.reshape(6)
    rd = 512 if inter == O.INTER_NEAREST else 16
    dw, dh = dsize
    mx = np.zeros((dh, dw, 2), np.int64)
    fa = np.zeros((dh, dw), np.int64)
    for dy in range(dh):
        for dx in range(dw):
            v1 = int(np.rint(t[0] * dx * 1024)) + int(np.rint((t[1] * dy + t[2]) * 1024)) + rd
            v2 = int(np.rint(t[3] * dx * 1024)) + int(np.rint((t[4] * dy + t[5]) * 1024)) + rd
            if inter == O.INTER_NEAREST:
                mx[dy, dx] = (np.clip(v1 >> 10, -32768, 32767), np.clip(v2 >> 10, -32768, 32767))
            else:
                v1 >>= 5
                v2 >>= 5
                mx[dy, dx] = (np.clip(v1 >> 5, -32768, 32767), np.clip(v2 >> 5, -32768, 32767))
                fa[dy, dx] = (v2 & 31) * 32 + (v1 & 31)
    return mx, fa


def cubic_coeffs(x):
    """interpolateCubic of the reference test (test_imgwarp_strict.cpp:379-387), float32"""
    f = np.float32
    x = f(x)
    A = f(-0.75)
    c0 = ((A * (x + f(1)) - f(5) * A) * (x + f(1)) + f(8) * A) * (x + f(1)) - f(4) * A
    c1 = ((A + f(2)) * x - (A + f(3))) * x * x + f(1)
    c2 = ((A + f(2)) * (f(1) - x) - (A + f(3))) * (f(1) - x) * (f(1) - x) + f(1)
    return [c0, c1, c2, f(1) - c0 - c1 - c2]


def ref_test_remap_cubic(src, mx, fa, border, bval):
    """remap_generic with ksize 4, ofs 1 (test_imgwarp_strict.cpp:928-1017)"""
    sh, sw = src.shape
    dh, dw = fa.shape
    out = np.zeros((dh, dw), np.float64)
    s = src.astype(np.float32)
    f = np.float32
    for dy in range(dh):
        for dx in range(dw):
            isx, isy = int(mx[dy, dx, 0]) - 1, int(mx[dy, dx, 1]) - 1
            w = cubic_coeffs((fa[dy, dx] & 31) / f(32))
            wy = cubic_coeffs(((fa[dy, dx] >> 5) & 31) / f(32))
            if 0 <= isx < sw - 3 and 0 <= isy < sh - 3:
                ix = []
                for y in range(4):
                    acc = f(0)
                    for i in range(4):
                        acc = f(acc + w[i] * s[isy + y, isx + i])
                    ix.append(acc)
            else:
                ax = [border_interp_c(isx + k, sw, border) for k in range(4)]
                ay = [border_interp_c(isy + k, sh, border) for k in range(4)]
                ix = []
                for i in range(4):
                    acc = f(0)
                    for j in range(4):
                        v = s[ay[i], ax[j]] if (ay[i] >= 0 and ax[j] >= 0) else f(bval)
                        acc = f(acc + f(v * w[j]))
                    ix.append(acc)
            acc = f(0)
            for i in range(4):
                acc = f(acc + f(wy[i] * ix[i]))
            out[dy, dx] = acc
    return out


def ref_test_remap(src, mx, fa, inter, border, bval):
    """remap_nearest / remap_generic (float weights, ksize 2) of the reference test."""
    if inter == O.INTER_CUBIC:
        return ref_test_remap_cubic(src, mx, fa, border, bval)
    sh, sw = src.shape
    dh, dw = fa.shape
    out = np.zeros((dh, dw), np.float64)
    s = src.astype(np.float32)
    for dy in range(dh):
        for dx in range(dw):
            sx, sy = int(mx[dy, dx, 0]), int(mx[dy, dx, 1])
            if inter == O.INTER_NEAREST:
                if 0 <= sx < sw and 0 <= sy < sh:
                    out[dy, dx] = s[sy, sx]
                elif border == O.BORDER_CONSTANT:
                    out[dy, dx] = bval
                else:
                    out[dy, dx] = s[border_interp_c(sy, sh, border), border_interp_c(sx, sw, border)]
                continue
            wx1 = np.float32((fa[dy, dx] & 31) / 32.0)
            wy1 = np.float32(((fa[dy, dx] >> 5) & 31) / 32.0)
            w = [np.float32(1) - wx1, wx1]
            wy = [np.float32(1) - wy1, wy1]
            if 0 <= sx < sw - 1 and 0 <= sy < sh - 1:
                ix = [w[0] * s[sy + k, sx] + w[1] * s[sy + k, sx + 1] for k in range(2)]
            else:
                ax = [border_interp_c(sx + k, sw, border) for k in range(2)]
                ay = [border_interp_c(sy + k, sh, border) for k in range(2)]
                ix = []
                for i in range(2):
                    acc = np.float32(0)
                    for j in range(2):
                        v = s[ay[i], ax[j]] if (ay[i] >= 0 and ax[j] >= 0) else np.float32(bval)
                        acc += np.float32(v * w[j])
                    ix.append(acc)
            out[dy, dx] = wy[0] * ix[0] + wy[1] * ix[1]
    return out


CASES = [
    # (seed, src (w, h), dst (w, h), angle, scale, inter, inverse, border)
    (1, (37, 29), (41, 33), 30.0, 1.3, O.INTER_LINEAR, False, O.BORDER_CONSTANT),
    (2, (40, 31), (40, 31), -115.0, 0.7, O.INTER_LINEAR, True, O.BORDER_REPLICATE),
    (3, (23, 45), (30, 30), 170.0, 1.9, O.INTER_LINEAR, False, O.BORDER_REFLECT),
    (4, (33, 33), (29, 35), 64.0, 0.45, O.INTER_LINEAR, False, O.BORDER_WRAP),
    (5, (50, 20), (44, 26), -33.0, 1.1, O.INTER_LINEAR, True, O.BORDER_REFLECT_101),
    (6, (37, 29), (41, 33), 12.0, 1.6, O.INTER_NEAREST, False, O.BORDER_CONSTANT),
    (7, (31, 27), (35, 35), -150.0, 0.9, O.INTER_NEAREST, True, O.BORDER_REFLECT_101),
    (8, (26, 38), (32, 32), 95.0, 1.4, O.INTER_NEAREST, False, O.BORDER_WRAP),
    (9, (37, 29), (41, 33), 30.0, 1.3, O.INTER_CUBIC, False, O.BORDER_CONSTANT),
    (10, (40, 31), (40, 31), -115.0, 0.7, O.INTER_CUBIC, True, O.BORDER_REPLICATE),
    (11, (23, 45), (30, 30), 170.0, 1.9, O.INTER_CUBIC, False, O.BORDER_REFLECT),
    (12, (33, 33), (29, 35), 64.0, 0.45, O.INTER_CUBIC, False, O.BORDER_WRAP),
    (13, (50, 20), (44, 26), -33.0, 1.1, O.INTER_CUBIC, True, O.BORDER_REFLECT_101),
]


@pytest.mark.parametrize("seed,ssz,dsz,angle,scale,inter,inverse,border", CASES)
def test_warp_oracle_matches_reference_validator(seed, ssz, dsz, angle, scale, inter, inverse, border):
    rng = np.random.default_rng(seed)
    sw, sh = ssz
    src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    M = rotation_matrix(sw / 2.0, sh / 2.0, angle, scale)
    bval = int(rng.integers(0, 255))
    flags = inter | (O.WARP_INVERSE_MAP if inverse else 0)
    got = O.warp_affine(src, M, dsz, flags, border, bval)
    mx, fa = ref_test_maps(M, dsz, inter, inverse)
    ref = ref_test_remap(src, mx, fa, inter, border, bval)
    # validate_results (:247-266) ignores reference values outside [0, 255] (cubic overshoot)
    inside = (ref >= 0.0) & (ref <= 255.0)
    diff = np.abs(got.astype(np.float64) - ref) * inside
    assert diff.max() <= 1.0, diff.max()
    if inter == O.INTER_NEAREST:
        assert diff.max() == 0


def test_warp_known_answers():
    rng = np.random.default_rng(9)
    src = rng.integers(0, 256, (24, 40), dtype=np.uint8)
    ident = np.array([[1, 0, 0], [0, 1, 0]], np.float64)
    for inter in (O.INTER_NEAREST, O.INTER_LINEAR):
        assert np.array_equal(O.warp_affine(src, ident, (40, 24), inter), src)
    # integer translation by (+3, -2): dst(x, y) = src(x - 3, y + 2)
    T = np.array([[1, 0, 3], [0, 1, -2]], np.float64)
    out = O.warp_affine(src, T, (40, 24), O.INTER_LINEAR, O.BORDER_CONSTANT, 7)
    assert np.array_equal(out[0:22, 3:40], src[2:24, 0:37])
    assert (out[:, :3] == 7).all() and (out[22:, :] == 7).all()
    # half-pixel shift: exact average of neighbours with the 15-bit weights
    H = np.array([[1, 0, -0.5], [0, 1, 0]], np.float64)
    out = O.warp_affine(src, H, (40, 24), O.INTER_LINEAR | O.WARP_INVERSE_MAP, O.BORDER_REPLICATE)
    exp = (src[:, :-1].astype(np.int64) * 16384 + src[:, 1:].astype(np.int64) * 16384 + 16384) >> 15
    assert np.array_equal(out[:, 1:], exp.astype(np.uint8))


def test_warp_transparent_keeps_destination():
    rng = np.random.default_rng(11)
    src = rng.integers(0, 256, (20, 20), dtype=np.uint8)
    M = rotation_matrix(10, 10, 45, 1.5)
    init = np.full((30, 30), 99, np.uint8)
    out = O.warp_affine(src, M, (30, 30), O.INTER_LINEAR, O.BORDER_TRANSPARENT, 0, dst=init)
    assert (out == 99).any() and (out != 99).any()


def test_bicubic_table_sums_and_known_answers():
    """BicubicTab_i: every entry's 16 weights sum to 2^15 (initInterTab2D's
    correction, imgwarp.cpp:251-264); integer shifts and the identity warp
    reproduce the source with INTER_CUBIC"""
    import ctypes as C

    lib = O.load()
    lib.orc_bicubic_tab.argtypes = [C.c_int, C.c_int, C.c_void_p]
    for ay in range(32):
        for ax in range(32):
            w = np.zeros(16, np.int16)
            lib.orc_bicubic_tab(ay, ax, w.ctypes.data_as(C.c_void_p))
            assert int(w.astype(np.int64).sum()) == 32768
            if ax == 0 and ay == 0:
                # 1.0 * 2^15 saturates to 32767 and the sum correction searches
                # taps (2..3, 2..3), so the missing unit lands on tap (2, 2)
                assert w[5] == 32767 and w[10] == 1 and (np.delete(w, [5, 10]) == 0).all()
    rng = np.random.default_rng(21)
    src = rng.integers(0, 256, (24, 40), dtype=np.uint8)
    ident = np.array([[1, 0, 0], [0, 1, 0]], np.float64)
    assert np.array_equal(O.warp_affine(src, ident, (40, 24), O.INTER_CUBIC, O.BORDER_REFLECT_101), src)
    T = np.array([[1, 0, 3], [0, 1, -2]], np.float64)
    out = O.warp_affine(src, T, (40, 24), O.INTER_CUBIC, O.BORDER_CONSTANT, 7)
    assert np.array_equal(out[0:22, 3:40], src[2:24, 0:37])
    init = np.full((30, 30), 99, np.uint8)
    out = O.warp_affine(src, rotation_matrix(10, 10, 45, 1.5), (30, 30), O.INTER_CUBIC, O.BORDER_TRANSPARENT, 0,
                        dst=init)
    assert (out == 99).any() and (out != 99).any()
