// warp.hip — cv::warpAffine for u8 gray images (INTER_NEAREST / INTER_LINEAR /
// INTER_CUBIC, every border mode) on gfx950, bit-exact with the CPU
// implementation's fixed-point path (imgproc/src/imgwarp.cpp:2155-2290 map
// generation, remapBilinear :649-866 / remapNearest :330-440 / remapBicubic
// :860-958; see oracle/warp_oracle.c).  INTER_CUBIC derives each pixel's 16
// BicubicTab_i weights in the kernel (interpolateCubic in float, the products
// rounded to short, initInterTab2D's sum correction, :152-160, 213-268)
// instead of reading a table: the same integers, no device globals.
//
// One thread per 4 destination pixels of a row: the per-row term
// (M1*y + M2)*1024 is formed once per thread in double exactly as the
// reference does, the per-column term M0*x*1024 per pixel (no FMA: the file
// is built with -ffp-contract=off), then the 5-bit sub-pixel table index and
// the 15-bit bilinear weights (exact integers for INTER_LINEAR).  Stores are
// one 32-bit word per thread; source taps are L1/L2 gathers.
#include "tbdk_internal.hpp"

namespace tbdk {

namespace {

// saturate_cast<int>(double) == cvRound (cvtsd2si: half to even, 0x80000000 out of range)
__device__ __forceinline__ int cv_round_sat(double v)
{
    const double r = rint(v);
    return (r >= -2147483648.0 && r <= 2147483647.0) ? (int)r : INT_MIN;
}
__device__ __forceinline__ int sat16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
__device__ __forceinline__ int wrap_add(int a, int b) { return (int)((unsigned)a + (unsigned)b); }
__device__ __forceinline__ int clipi(int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; }

// cv::borderInterpolate (core/src/copy.cpp) for the non-trivial modes
__device__ __forceinline__ int border_interp(int p, int len, int border)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (border == TBDK_BORDER_REPLICATE) return p < 0 ? 0 : len - 1;
    if (border == TBDK_BORDER_REFLECT || border == TBDK_BORDER_REFLECT_101) {
        const int delta = border == TBDK_BORDER_REFLECT_101;
        if (len == 1) return 0;
        do {
            if (p < 0) p = -p - 1 + delta;
            else p = len - 1 - (p - len) - delta;
        } while ((unsigned)p >= (unsigned)len);
        return p;
    }
    if (border == TBDK_BORDER_WRAP) {
        if (p < 0) p -= ((p - len + 1) / len) * len;
        if (p >= len) p %= len;
        return p;
    }
    return -1;
}

// interpolateCubic (imgwarp.cpp:152-160)
__device__ __forceinline__ void cubic_coeffs(float x, float* c)
{
    const float A = -0.75f;
    c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    c[3] = 1.f - c[0] - c[1] - c[2];
}

// BicubicTab_i[ay*32 + ax] (initInterTab2D, imgwarp.cpp:213-268)
__device__ __forceinline__ void bicubic_tab(int ay, int ax, int* w)
{
    const float scale = 1.f / 32;
    float cy[4], cx[4];
    cubic_coeffs(ay * scale, cy);
    cubic_coeffs(ax * scale, cx);
    int isum = 0;
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) {
            int iv = __float2int_rn(cy[k1] * cx[k2] * 32768);  // saturate_cast<short>(float)
            iv = iv < -32768 ? -32768 : (iv > 32767 ? 32767 : iv);
            w[k1 * 4 + k2] = iv;
            isum += iv;
        }
    if (isum != 32768) {  // the correction searches taps (2..3, 2..3), as the reference does
        const int diff = isum - 32768;
        int M = 10, m = 10;
#pragma unroll
        for (int k1 = 2; k1 < 4; ++k1)
#pragma unroll
            for (int k2 = 2; k2 < 4; ++k2) {
                const int t = k1 * 4 + k2;
                if (w[t] < w[m]) m = t;
                else if (w[t] > w[M]) M = t;
            }
        // w[] is indexed by runtime values here: keep it in registers via selects
#pragma unroll
        for (int t = 10; t < 16; ++t) {
            if (diff < 0 && t == M) w[t] -= diff;
            if (diff >= 0 && t == m) w[t] -= diff;
        }
    }
}

struct WarpArgs {
    const uint8_t* src;
    int sw, sh, spitch;
    uint8_t* dst;
    int dw, dh, dpitch;
    double m[6];  // inverse map (dst -> src)
    int inter, border, cval;
};

template <int INTER>
__global__ __launch_bounds__(256) void warp_affine_kernel(WarpArgs a)
{
    const int y = blockIdx.y;
    const int x0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (x0 >= a.dw) return;
    constexpr int round_delta = INTER == 0 ? 512 : 16;
    const int X0 = wrap_add(cv_round_sat((a.m[1] * y + a.m[2]) * 1024), round_delta);
    const int Y0 = wrap_add(cv_round_sat((a.m[4] * y + a.m[5]) * 1024), round_delta);
    const uint8_t cval = (uint8_t)a.cval;
    uint8_t* D = a.dst + (size_t)y * a.dpitch;
    uint8_t out[4];
    bool keep[4];  // BORDER_TRANSPARENT: leave the destination pixel untouched
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int x = x0 + k;
        keep[k] = false;
        out[k] = 0;
        if (x >= a.dw) continue;
        const int ad = cv_round_sat(a.m[0] * x * 1024), bd = cv_round_sat(a.m[3] * x * 1024);
        if (INTER == 0) {
            const int sx = sat16(wrap_add(X0, ad) >> 10), sy = sat16(wrap_add(Y0, bd) >> 10);
            if ((unsigned)sx < (unsigned)a.sw && (unsigned)sy < (unsigned)a.sh) {
                out[k] = a.src[(size_t)sy * a.spitch + sx];
            } else if (a.border == TBDK_BORDER_REPLICATE) {
                out[k] = a.src[(size_t)clipi(sy, 0, a.sh) * a.spitch + clipi(sx, 0, a.sw)];
            } else if (a.border == TBDK_BORDER_CONSTANT) {
                out[k] = cval;
            } else if (a.border == TBDK_BORDER_TRANSPARENT) {
                keep[k] = true;
            } else {
                out[k] = a.src[(size_t)border_interp(sy, a.sh, a.border) * a.spitch + border_interp(sx, a.sw, a.border)];
            }
            continue;
        }
        const int X = wrap_add(X0, ad) >> 5, Y = wrap_add(Y0, bd) >> 5;
        const int sx = sat16(X >> 5), sy = sat16(Y >> 5);
        const int ax = X & 31, ay = Y & 31;
        if (INTER == 2) {  // remapBicubic (imgwarp.cpp:860-958)
            int w[16];
            bicubic_tab(ay, ax, w);
            const int bx = sx - 1, by = sy - 1;
            int sum;
            if ((unsigned)bx < (unsigned)(a.sw - 3 > 0 ? a.sw - 3 : 0) &&
                (unsigned)by < (unsigned)(a.sh - 3 > 0 ? a.sh - 3 : 0)) {
                const uint8_t* S = a.src + (size_t)by * a.spitch + bx;
                sum = 0;
#pragma unroll
                for (int r = 0; r < 4; ++r, S += a.spitch)
                    sum += S[0] * w[4 * r] + S[1] * w[4 * r + 1] + S[2] * w[4 * r + 2] + S[3] * w[4 * r + 3];
            } else {
                if (a.border == TBDK_BORDER_TRANSPARENT &&
                    ((unsigned)(bx + 1) >= (unsigned)a.sw || (unsigned)(by + 1) >= (unsigned)a.sh)) {
                    keep[k] = true;
                    continue;
                }
                const int b1 = a.border != TBDK_BORDER_TRANSPARENT ? a.border : TBDK_BORDER_REFLECT_101;
                if (b1 == TBDK_BORDER_CONSTANT && (bx >= a.sw || bx + 4 <= 0 || by >= a.sh || by + 4 <= 0)) {
                    out[k] = cval;
                    continue;
                }
                int xs[4], ys[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    xs[q] = border_interp(bx + q, a.sw, b1);
                    ys[q] = border_interp(by + q, a.sh, b1);
                }
                const int cv = cval;
                sum = cv * 32768;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (ys[r] < 0) continue;
                    const uint8_t* S = a.src + (size_t)ys[r] * a.spitch;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (xs[q] >= 0) sum += (S[xs[q]] - cv) * w[4 * r + q];
                }
            }
            const int r = (sum + (1 << 14)) >> 15;  // FixedPtCast<int, uchar, 15>
            out[k] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
            continue;
        }
        // BilinearTab_i (imgwarp.cpp:211-268): 15-bit weights, exact for INTER_LINEAR
        const int w0 = (32 - ay) * (32 - ax) * 32, w1 = (32 - ay) * ax * 32;
        const int w2 = ay * (32 - ax) * 32, w3 = ay * ax * 32;
        int v0, v1, v2, v3;
        if ((unsigned)sx < (unsigned)(a.sw - 1) && (unsigned)sy < (unsigned)(a.sh - 1)) {
            const uint8_t* S = a.src + (size_t)sy * a.spitch + sx;
            v0 = S[0];
            v1 = S[1];
            v2 = S[a.spitch];
            v3 = S[a.spitch + 1];
        } else {
            if (a.border == TBDK_BORDER_TRANSPARENT) {
                keep[k] = true;
                continue;
            }
            if (a.border == TBDK_BORDER_CONSTANT && (sx >= a.sw || sx + 1 < 0 || sy >= a.sh || sy + 1 < 0)) {
                out[k] = cval;
                continue;
            }
            int sx0, sx1, sy0, sy1;
            if (a.border == TBDK_BORDER_REPLICATE) {
                sx0 = clipi(sx, 0, a.sw);
                sx1 = clipi(sx + 1, 0, a.sw);
                sy0 = clipi(sy, 0, a.sh);
                sy1 = clipi(sy + 1, 0, a.sh);
            } else {
                sx0 = border_interp(sx, a.sw, a.border);
                sx1 = border_interp(sx + 1, a.sw, a.border);
                sy0 = border_interp(sy, a.sh, a.border);
                sy1 = border_interp(sy + 1, a.sh, a.border);
            }
            v0 = sx0 >= 0 && sy0 >= 0 ? a.src[(size_t)sy0 * a.spitch + sx0] : cval;
            v1 = sx1 >= 0 && sy0 >= 0 ? a.src[(size_t)sy0 * a.spitch + sx1] : cval;
            v2 = sx0 >= 0 && sy1 >= 0 ? a.src[(size_t)sy1 * a.spitch + sx0] : cval;
            v3 = sx1 >= 0 && sy1 >= 0 ? a.src[(size_t)sy1 * a.spitch + sx1] : cval;
        }
        const int r = (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << 14)) >> 15;  // FixedPtCast<int,uchar,15>
        out[k] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
    const bool full = x0 + 4 <= a.dw && !(keep[0] | keep[1] | keep[2] | keep[3]);
    if (full && ((reinterpret_cast<uintptr_t>(D + x0) & 3) == 0)) {
        *reinterpret_cast<uint32_t*>(D + x0) =
            (uint32_t)out[0] | ((uint32_t)out[1] << 8) | ((uint32_t)out[2] << 16) | ((uint32_t)out[3] << 24);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (x0 + k < a.dw && !keep[k]) D[x0 + k] = out[k];
    }
}

}  // namespace

// M inversion of cv::warpAffine (imgwarp.cpp:2606-2616), host double arithmetic
void invert_affine(const double* M, double* out)
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

hipError_t launch_warp_affine(const uint8_t* src, int sw, int sh, int spitch, uint8_t* dst, int dw, int dh, int dpitch,
                              const double* minv, int inter, int border, int cval, hipStream_t s)
{
    WarpArgs a;
    a.src = src;
    a.sw = sw;
    a.sh = sh;
    a.spitch = spitch;
    a.dst = dst;
    a.dw = dw;
    a.dh = dh;
    a.dpitch = dpitch;
    for (int i = 0; i < 6; ++i) a.m[i] = minv[i];
    a.inter = inter;
    a.border = border;
    a.cval = cval;
    const dim3 grid((dw + 4 * 256 - 1) / (4 * 256), dh), block(256);
    if (inter == 0) hipLaunchKernelGGL(warp_affine_kernel<0>, grid, block, 0, s, a);
    else if (inter == 2) hipLaunchKernelGGL(warp_affine_kernel<2>, grid, block, 0, s, a);
    else hipLaunchKernelGGL(warp_affine_kernel<1>, grid, block, 0, s, a);
    return hipGetLastError();
}

}  // namespace tbdk
