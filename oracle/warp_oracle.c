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
 *   INTER_CUBIC: the same map (5-bit table index); remapBicubic<FixedPtCast<int,
 *     uchar,15>> (:860-958) with BicubicTab_i built as initInterTab2D does
 *     (:152-160 interpolateCubic in float, A = -0.75; :213-268 products
 *     rounded to short, the sum corrected to 2^15 on the central 2x2)
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

/* interpolateCubic (imgwarp.cpp:152-160), float */
static void cubic_coeffs(float x, float* c)
{
    const float A = -0.75f;
    c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    c[3] = 1.f - c[0] - c[1] - c[2];
}

/* BicubicTab_i[ay*32 + ax] (initInterTab2D, imgwarp.cpp:213-268) */
void orc_bicubic_tab(int ay, int ax, short* w)
{
    const float scale = 1.f / 32;
    float cy[4], cx[4];
    cubic_coeffs(ay * scale, cy);
    cubic_coeffs(ax * scale, cx);
    int isum = 0;
    for (int k1 = 0; k1 < 4; ++k1)
        for (int k2 = 0; k2 < 4; ++k2) {
            const float v = cy[k1] * cx[k2];
            int iv = (int)nearbyintf(v * 32768); /* saturate_cast<short>(float): cvRound, then clamp */
            iv = iv < -32768 ? -32768 : (iv > 32767 ? 32767 : iv);
            w[k1 * 4 + k2] = (short)iv;
            isum += iv;
        }
    if (isum != 32768) {
        const int diff = isum - 32768;
        int Mk1 = 2, Mk2 = 2, mk1 = 2, mk2 = 2;
        for (int k1 = 2; k1 < 4; ++k1)
            for (int k2 = 2; k2 < 4; ++k2) {
                if (w[k1 * 4 + k2] < w[mk1 * 4 + mk2]) mk1 = k1, mk2 = k2;
                else if (w[k1 * 4 + k2] > w[Mk1 * 4 + Mk2]) Mk1 = k1, Mk2 = k2;
            }
        if (diff < 0) w[Mk1 * 4 + Mk2] = (short)(w[Mk1 * 4 + Mk2] - diff);
        else w[mk1 * 4 + mk2] = (short)(w[mk1 * 4 + mk2] - diff);
    }
}

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
    if (inter != 0 && inter != 1 && inter != 2) return -1;
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
            if (inter == 2) { /* remapBicubic (imgwarp.cpp:860-958) */
                short w[16];
                orc_bicubic_tab(ay, ax, w);
                const int bx = sx - 1, by = sy - 1;
                int sum;
                if ((unsigned)bx < (unsigned)(sw - 3 > 0 ? sw - 3 : 0) && (unsigned)by < (unsigned)(sh - 3 > 0 ? sh - 3 : 0)) {
                    const uint8_t* S = src + (size_t)by * spitch + bx;
                    sum = 0;
                    for (int r = 0; r < 4; ++r, S += spitch)
                        sum += S[0] * w[4 * r] + S[1] * w[4 * r + 1] + S[2] * w[4 * r + 2] + S[3] * w[4 * r + 3];
                } else {
                    if (border == ORC_BORDER_TRANSPARENT &&
                        ((unsigned)(bx + 1) >= (unsigned)sw || (unsigned)(by + 1) >= (unsigned)sh))
                        continue;
                    const int b1 = border != ORC_BORDER_TRANSPARENT ? border : ORC_BORDER_REFLECT_101;
                    if (b1 == ORC_BORDER_CONSTANT && (bx >= sw || bx + 4 <= 0 || by >= sh || by + 4 <= 0)) {
                        D[x] = cval;
                        continue;
                    }
                    int xs[4], ys[4];
                    for (int i = 0; i < 4; ++i) {
                        xs[i] = orc_border_interpolate(bx + i, sw, b1);
                        ys[i] = orc_border_interpolate(by + i, sh, b1);
                    }
                    const int cv = cval;
                    sum = cv * 32768;
                    for (int i = 0; i < 4; ++i) {
                        if (ys[i] < 0) continue;
                        const uint8_t* S = src + (size_t)ys[i] * spitch;
                        for (int j = 0; j < 4; ++j)
                            if (xs[j] >= 0) sum += (S[xs[j]] - cv) * w[4 * i + j];
                    }
                }
                const int r = (sum + (1 << 14)) >> 15; /* FixedPtCast<int, uchar, 15> */
                D[x] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
                continue;
            }
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
