/*
 * warp_oracle.c — CPU restatement of cv::warpAffine for CV_8UC1
 * (INTER_NEAREST / INTER_LINEAR, every border mode).  TEST INFRASTRUCTURE ONLY.
 *
 *   M inversion unless WARP_INVERSE_MAP        imgproc/src/imgwarp.cpp:2606-2616
 *   fixed-point source map, AB_BITS = 10:
 *     adelta[x] = saturate_cast<int>(M0*x*1024)                     :2555-2559
 *     X0 = saturate_cast<int>((M1*y + M2)*1024) + round_delta       :2198-2199
 *     LINEAR : X = (X0 + adelta) >> 5; sx = sat16(X >> 5); ax = X & 31   :2266-2274
 *     NEAREST: sx = sat16((X0 + adelta) >> 10)                      :2226-2232
 *   remapBilinear<FixedPtCast<int,uchar,15>> with BilinearTab_i (15-bit
 *     weights (32-a)(32-b)*32 ..., exact for INTER_LINEAR)            :649-866, 211-268
 *   remapNearest                                                    :330-440
 *   borderInterpolate (core/src/copy.cpp) for REFLECT/REFLECT_101/WRAP,
 *     clip() for REPLICATE, cval for CONSTANT, skip for TRANSPARENT.
 * saturate_cast<int>(double) is cvRound (SSE2 cvtsd2si: round half to even,
 * 0x80000000 when out of range); int sums wrap as on x86.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "klt_oracle.h"

static int cv_round_sat(double v)
{
    const double r = nearbyint(v);
    if (!(r >= -2147483648.0 && r <= 2147483647.0)) return INT32_MIN;
    return (int)r;
}

static int sat16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

static int wrap_add(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }

int orc_border_interpolate(int p, int len, int border)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (border == ORC_BORDER_REPLICATE) return p < 0 ? 0 : len - 1;
    if (border == ORC_BORDER_REFLECT || border == ORC_BORDER_REFLECT_101) {
        const int delta = border == ORC_BORDER_REFLECT_101;
        if (len == 1) return 0;
        do {
            if (p < 0) p = -p - 1 + delta;
            else p = len - 1 - (p - len) - delta;
        } while ((unsigned)p >= (unsigned)len);
        return p;
    }
    if (border == ORC_BORDER_WRAP) {
        if (p < 0) p -= ((p - len + 1) / len) * len;
        if (p >= len) p %= len;
        return p;
    }
    return -1; /* CONSTANT */
}

static int clipi(int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; }

void orc_invert_affine(const double* M, double* out)
{
    double m[6];
    for (int i = 0; i < 6; ++i) m[i] = M[i];
    double D = m[0] * m[4] - m[1] * m[3];
    D = D != 0 ? 1. / D : 0;
    const double A11 = m[4] * D, A22 = m[0] * D;
    m[0] = A11;
    m[1] *= -D;
    m[3] *= -D;
    m[4] = A22;
    const double b1 = -m[0] * m[2] - m[1] * m[5];
    const double b2 = -m[3] * m[2] - m[4] * m[5];
    m[2] = b1;
    m[5] = b2;
    for (int i = 0; i < 6; ++i) out[i] = m[i];
}

int orc_warp_affine_u8(const uint8_t* src, int sw, int sh, int spitch, uint8_t* dst, int dw, int dh, int dpitch,
                       const double* M0, int flags, int border, int bval)
{
    int inter = flags & 7;
    if (inter == 3) inter = 1; /* INTER_AREA -> INTER_LINEAR (:2600-2601) */
    if (inter != 0 && inter != 1) return -1;
    double M[6];
    if (flags & ORC_WARP_INVERSE_MAP) {
        for (int i = 0; i < 6; ++i) M[i] = M0[i];
    } else {
        orc_invert_affine(M0, M);
    }
    const int round_delta = inter == 0 ? 512 : 16;
    const uint8_t cval = (uint8_t)(bval < 0 ? 0 : (bval > 255 ? 255 : bval));
    const unsigned width1 = sw > 1 ? (unsigned)(sw - 1) : 0u, height1 = sh > 1 ? (unsigned)(sh - 1) : 0u;
    for (int y = 0; y < dh; ++y) {
        const int X0 = wrap_add(cv_round_sat((M[1] * y + M[2]) * 1024), round_delta);
        const int Y0 = wrap_add(cv_round_sat((M[4] * y + M[5]) * 1024), round_delta);
        uint8_t* D = dst + (size_t)y * dpitch;
        for (int x = 0; x < dw; ++x) {
            const int ad = cv_round_sat(M[0] * x * 1024), bd = cv_round_sat(M[3] * x * 1024);
            if (inter == 0) {
                const int sx = sat16(wrap_add(X0, ad) >> 10), sy = sat16(wrap_add(Y0, bd) >> 10);
                if ((unsigned)sx < (unsigned)sw && (unsigned)sy < (unsigned)sh) {
                    D[x] = src[(size_t)sy * spitch + sx];
                } else if (border == ORC_BORDER_REPLICATE) {
                    D[x] = src[(size_t)clipi(sy, 0, sh) * spitch + clipi(sx, 0, sw)];
                } else if (border == ORC_BORDER_CONSTANT) {
                    D[x] = cval;
                } else if (border != ORC_BORDER_TRANSPARENT) {
                    const int bx = orc_border_interpolate(sx, sw, border), by = orc_border_interpolate(sy, sh, border);
                    D[x] = src[(size_t)by * spitch + bx];
                }
                continue;
            }
            const int X = wrap_add(X0, ad) >> 5, Y = wrap_add(Y0, bd) >> 5;
            const int sx = sat16(X >> 5), sy = sat16(Y >> 5);
            const int ax = X & 31, ay = Y & 31;
            /* BilinearTab_i[ay*32+ax] = {(32-ay)(32-ax), (32-ay)ax, ay(32-ax), ay*ax} * 32 */
            const int w0 = (32 - ay) * (32 - ax) * 32, w1 = (32 - ay) * ax * 32;
            const int w2 = ay * (32 - ax) * 32, w3 = ay * ax * 32;
            int v0, v1, v2, v3;
            if ((unsigned)sx < width1 && (unsigned)sy < height1) {
                const uint8_t* S = src + (size_t)sy * spitch + sx;
                v0 = S[0]; v1 = S[1]; v2 = S[spitch]; v3 = S[spitch + 1];
            } else {
                if (border == ORC_BORDER_TRANSPARENT) continue;
                if (border == ORC_BORDER_CONSTANT && (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0)) {
                    D[x] = cval;
                    continue;
                }
                int sx0, sx1, sy0, sy1;
                if (border == ORC_BORDER_REPLICATE) {
                    sx0 = clipi(sx, 0, sw); sx1 = clipi(sx + 1, 0, sw);
                    sy0 = clipi(sy, 0, sh); sy1 = clipi(sy + 1, 0, sh);
                } else {
                    sx0 = orc_border_interpolate(sx, sw, border); sx1 = orc_border_interpolate(sx + 1, sw, border);
                    sy0 = orc_border_interpolate(sy, sh, border); sy1 = orc_border_interpolate(sy + 1, sh, border);
                }
                v0 = sx0 >= 0 && sy0 >= 0 ? src[(size_t)sy0 * spitch + sx0] : cval;
                v1 = sx1 >= 0 && sy0 >= 0 ? src[(size_t)sy0 * spitch + sx1] : cval;
                v2 = sx0 >= 0 && sy1 >= 0 ? src[(size_t)sy1 * spitch + sx0] : cval;
                v3 = sx1 >= 0 && sy1 >= 0 ? src[(size_t)sy1 * spitch + sx1] : cval;
            }
            int r = (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << 14)) >> 15;
            D[x] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
        }
    }
    return 0;
}
