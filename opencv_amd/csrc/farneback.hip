// farneback.hip — dense Farneback optical flow on gfx950, the numerics of the
// CPU cv::calcOpticalFlowFarneback (video/src/optflowgf.cpp:57-578, 1096-1190)
// behind the cv::cuda::FarnebackOpticalFlow interface
// (cudaoptflow/include/opencv2/cudaoptflow.hpp:210-252, impl
// cudaoptflow/src/farneback.cpp:164-474).
//
// Per pyramid level k (coarsest first), for each of the two frames:
//   fb_rowpass / fb_colpass  GaussianBlur(float(img), smooth_sz, sigma) then
//                            resize(INTER_LINEAR) to the level size, evaluated
//                            only at the source rows/columns the resize samples
//                            (the blur's separable row filter, its column
//                            filter, then the resize's weights, each in the
//                            reference's float operation order).
//   fb_polyexp               FarnebackPolyExp (optflowgf.cpp:116-202): float
//                            vertical pass, double horizontal pass -> R (5 planes).
// then flow init (zeros, or the previous level's flow resized INTER_LINEAR and
// scaled by 1/pyrScale) and numIters launches of
//   fb_iter                  one Jacobi step: M = FarnebackUpdateMatrices(R0, R1,
//                            flow) (optflowgf.cpp:217-312) recomputed on the fly
//                            for a 128-column strip walking down a row segment
//                            (ring of the last 2m+1 rows of M in registers), the
//                            vertical window sum (box: exact-order float sum;
//                            FARNEBACK_GAUSSIAN: the reference's float weighted
//                            sum), the horizontal window from LDS, the 2x2 solve
//                            in double -> next flow (optflowgf.cpp:341-403, 446-569).
// The reference interleaves UpdateMatrices with the blur in row stripes; the
// rows it updates are never read again by that pass (y1 = y - block_size), so it
// is exactly flow_{i+1} = solve(blur(M(flow_i))): M is never stored here, each
// iteration reads flow + R0 + R1 (48 B/px) and writes flow (8 B/px).
//
// Numerics: every float/double expression is written as the reference's (this
// file is compiled with -ffp-contract=off), so the level images, R, M, the
// Gaussian-variant blur and the solve round exactly as the reference's scalar/SSE2
// code.  The box variant's vertical/horizontal sums are exact-order float
// window sums instead of the reference's running double sums, whose
// float-rounded row differences accumulate over the whole image: bit-exact
// with the oracle's box_direct mode, which is compared to the reference's
// running sums within a stated tolerance.
#include <cfloat>
#include <cmath>
#include <cstring>
#include <new>
#include <type_traits>
#include <utility>

#include <cstdlib>
#include "tbdk_internal.hpp"

namespace tbdk {

struct FbScratch {
    float* R0 = nullptr;  // 5 planes
    float* R1 = nullptr;  // 5 planes
    float* F[2] = {nullptr, nullptr};  // flow ping-pong, 2 planes each
    float* T = nullptr;   // row-pass buffer
    float* I = nullptr;   // level image
    int64_t cap_px = 0;   // floats per plane
    int64_t cap_T = 0;
    // prep-ahead (ctx option fb_prep_ahead): every level's R0 / R1 in its own
    // region of Rl, computed on the prep stream while coarser levels iterate
    float* Rl = nullptr;
    int64_t cap_Rl = 0;
    hipStream_t prep = nullptr;
    hipEvent_t fork = nullptr;
    hipEvent_t lev_ev[64] = {};
    // the last tbdk_farneback call's stream and its completion: a call on
    // another stream waits for it before reusing the scratch
    hipStream_t last_stream = nullptr;
    hipEvent_t done = nullptr;
};

namespace {

constexpr int kFbMaxKs = 255;   // GaussianBlur ksize of the level images
constexpr int kFbMaxPolyN = 15;
constexpr int kFbMaxHalf = 10;  // winsize <= 21
constexpr int kFbStrip = 128;   // fb_iter strip width (columns, incl. the 2m halo)
// output columns of a strip: a multiple of 4, so every strip starts on an
// image column divisible by 4 (the box sums restart there)
__host__ __device__ constexpr int fb_ow(int m) { return (kFbStrip - 2 * m) & ~3; }

enum { kModeNone = 0, kModeArea2 = 1, kModeLinear = 2 };

__host__ __device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
}

// cvFloor(float): x86 cvttss2si yields INT_MIN for NaN / out of range
__device__ __forceinline__ int cv_floorf(float v)
{
    if (!(v >= -2147483648.f && v < 2147483648.f)) return INT_MIN;
    const int i = (int)v;
    return i - (i > v);
}

// resize INTER_LINEAR source column / weight of destination column dx
// (imgproc/src/resize.cpp:3600-3640, ksize2 = 1)
struct LinX {
    int sx;
    float fx;
    bool inner;  // dx < xmax: two taps
};
__device__ __forceinline__ LinX lin_x(int dx, double scale_x, int sw)
{
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cv_floorf(fx);
    fx -= sx;
    if (sx < 0) fx = 0, sx = 0;
    LinX r;
    r.inner = !(sx + 1 >= sw);
    if (sx + 1 >= sw && sx >= sw - 1) fx = 0, sx = sw - 1;
    r.sx = sx;
    r.fx = fx;
    return r;
}

// ---------------------------------------------------------------------------
// level image: GaussianBlur (sepFilter2D, REFLECT_101) + resize INTER_LINEAR

struct FbRowArgs {
    const uint8_t* img;
    int W, H, pitch;
    float* T;
    int tpitch, nc;
    int mode;        // kMode*
    double scale_x;  // LINEAR: W / dw
    int ks;
    float k[kFbMaxKs];
};

// source column of sample j of a row
__device__ __forceinline__ int fb_row_col(const FbRowArgs& a, int j)
{
    if (a.mode != kModeLinear) return j;
    const LinX lx = lin_x(j >> 1, a.scale_x, a.W);
    return (j & 1) && lx.inner ? lx.sx + 1 : lx.sx;
}

// row filter of row y at source column c (filter.simd.hpp SymmRowSmallFilter /
// RowFilter scalar and SSE orders, see oracle/farneback_oracle.c).  Kernels
// wider than 5 taps (the coarse levels: up to ~90 taps) read the block's span of
// the row from LDS, staged once with its reflect-101 border, instead of one
// global byte load and one reflect per tap.
__global__ __launch_bounds__(256) void fb_rowpass_kernel(FbRowArgs a)
{
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    const uint8_t* S = a.img + (size_t)y * a.pitch;
    const int r = a.ks >> 1;
    if (a.ks > 5) {
        extern __shared__ uint8_t srow[];
        // the samples of this block read columns [c0 - r, c1 + r] (columns are
        // monotonic in j)
        const int j0 = blockIdx.x * 256, j1 = min(j0 + 255, a.nc - 1);
        const int c0 = fb_row_col(a, j0 & ~1), c1 = fb_row_col(a, (j1 | 1) < a.nc ? (j1 | 1) : j1);
        const int base = c0 - r, len = c1 - c0 + 1 + 2 * r;
        for (int i = threadIdx.x; i < len; i += 256) srow[i] = S[reflect101(base + i, a.W)];
        __syncthreads();
        if (j >= a.nc) return;
        const uint8_t* R = srow + (fb_row_col(a, j) - r - base);  // R[t] = column c - r + t
        float s = a.k[0] * (float)R[0];
        for (int t = 1; t < a.ks; ++t) s += a.k[t] * (float)R[t];
        a.T[(size_t)y * a.tpitch + j] = s;
        return;
    }
    if (j >= a.nc) return;
    const int c = fb_row_col(a, j);
#define SX(o) ((float)S[reflect101(c + (o), a.W)])
    float s;
    if (a.ks == 3) {
        s = SX(0) * a.k[1] + (SX(-1) + SX(1)) * a.k[0];
    } else if (a.ks == 5) {
        s = SX(0) * a.k[2] + (SX(-1) + SX(1)) * a.k[1] + (SX(-2) + SX(2)) * a.k[0];
    } else {
        s = a.k[0] * SX(-r);
        for (int t = 1; t < a.ks; ++t) s += a.k[t] * SX(t - r);
    }
#undef SX
    a.T[(size_t)y * a.tpitch + j] = s;
}

struct FbColArgs {
    const float* T;
    int tpitch, H;  // source rows
    int W;          // source columns (LINEAR bounds)
    float* I;
    int w, h, ipitch;
    int mode;
    double scale_x, scale_y;
    int ks;
    float k[kFbMaxKs];
};

// column filter at source row y over T column j (SymmColumnSmallFilter /
// SymmColumnFilter, delta 0)
__device__ __forceinline__ float fb_colf(const FbColArgs& a, int y, int j)
{
    const float* T = a.T + j;
    const int r = a.ks >> 1;
#define SY(o) T[(size_t)reflect101(y + (o), a.H) * a.tpitch]
    float s;
    if (a.ks == 3) {
        s = (SY(-1) + SY(1)) * a.k[0] + SY(0) * a.k[1] + 0.0f;
    } else {
        s = a.k[r] * SY(0) + 0.0f;
        for (int t = 1; t <= r; ++t) s += a.k[r + t] * (SY(t) + SY(-t));
    }
#undef SY
    return s;
}

__global__ __launch_bounds__(256) void fb_colpass_kernel(FbColArgs a)
{
    const int dx = blockIdx.x * 256 + threadIdx.x;
    const int dy = blockIdx.y;
    if (dx >= a.w) return;
    float v;
    if (a.mode == kModeNone) {
        v = fb_colf(a, dy, dx);
    } else if (a.mode == kModeArea2) {
        // resizeAreaFast 2x (resize.cpp:2471-2497 SIMD part, 2626-2640 scalar tail)
        const float p0 = fb_colf(a, 2 * dy, 2 * dx), p1 = fb_colf(a, 2 * dy, 2 * dx + 1);
        const float q0 = fb_colf(a, 2 * dy + 1, 2 * dx), q1 = fb_colf(a, 2 * dy + 1, 2 * dx + 1);
        if (dx < (a.w & ~3)) {
            v = ((p0 + p1) + (q0 + q1)) * 0.25f;
        } else {
            float sum = 0;
            sum += p0 + p1 + q0 + q1;
            v = sum * 0.25f;
        }
    } else {
        const LinX lx = lin_x(dx, a.scale_x, a.W);
        float fy = (float)((dy + 0.5) * a.scale_y - 0.5);
        const int sy = cv_floorf(fy);
        fy -= sy;
        const float b0 = 1.f - fy, b1 = fy;
        const float a0 = 1.f - lx.fx, a1 = lx.fx;
        float hrow[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int yy = clampi(sy + t, 0, a.H - 1);
            const float s0 = fb_colf(a, yy, 2 * dx);
            hrow[t] = lx.inner ? s0 * a0 + fb_colf(a, yy, 2 * dx + 1) * a1 : s0;
        }
        v = hrow[0] * b0 + hrow[1] * b1;
    }
    a.I[(size_t)dy * a.ipitch + dx] = v;
}

// ---------------------------------------------------------------------------
// FarnebackPolyExp (optflowgf.cpp:116-202); R planes: R[c][y][x]

struct FbPolyArgs {
    const float* I;
    int w, h, ipitch;
    float* R;
    int rpitch;
    int64_t rplane;
    int n;
    float g[kFbMaxPolyN + 1], xg[kFbMaxPolyN + 1], xxg[kFbMaxPolyN + 1];  // index 0..n
    double ig11, ig03, ig33, ig55;
};

__global__ __launch_bounds__(256) void fb_polyexp_kernel(FbPolyArgs a)
{
    __shared__ float tr[3][256 + 2 * kFbMaxPolyN];
    const int x0 = blockIdx.x * 256;
    const int y = blockIdx.y;
    const int n = a.n;
    // vertical part of the convolution, replicated borders (row[-1-x] = row[2-x])
    for (int i = threadIdx.x; i < 256 + 2 * n; i += 256) {
        const int c = clampi(x0 - n + i, 0, a.w - 1);
        const float* col = a.I + c;
        float t0 = col[(size_t)y * a.ipitch] * a.g[0], t1 = 0.f, t2 = 0.f;
        for (int k = 1; k <= n; ++k) {
            const float s0 = col[(size_t)(y - k < 0 ? 0 : y - k) * a.ipitch];
            const float s1 = col[(size_t)(y + k > a.h - 1 ? a.h - 1 : y + k) * a.ipitch];
            const float p = s0 + s1;
            t0 = t0 + a.g[k] * p;
            t1 = t1 + a.xg[k] * (s1 - s0);
            t2 = t2 + a.xxg[k] * p;
        }
        tr[0][i] = t0;
        tr[1][i] = t1;
        tr[2][i] = t2;
    }
    __syncthreads();
    const int x = x0 + threadIdx.x;
    if (x >= a.w) return;
    const int o = threadIdx.x + n;
    float g0 = a.g[0];
    double b1 = tr[0][o] * g0, b2 = 0, b3 = tr[1][o] * g0, b4 = 0, b5 = tr[2][o] * g0, b6 = 0;
    for (int k = 1; k <= n; ++k) {
        const double tg = tr[0][o + k] + tr[0][o - k];
        g0 = a.g[k];
        b1 += tg * g0;
        b4 += tg * a.xxg[k];
        b2 += (tr[0][o + k] - tr[0][o - k]) * a.xg[k];
        b3 += (tr[1][o + k] + tr[1][o - k]) * g0;
        b6 += (tr[1][o + k] - tr[1][o - k]) * a.xg[k];
        b5 += (tr[2][o + k] + tr[2][o - k]) * g0;
    }
    float* R = a.R + (size_t)y * a.rpitch + x;
    R[a.rplane] = (float)(b2 * a.ig11);
    R[0] = (float)(b3 * a.ig11);
    R[3 * a.rplane] = (float)(b1 * a.ig03 + b4 * a.ig33);
    R[2 * a.rplane] = (float)(b1 * a.ig03 + b5 * a.ig33);
    R[4 * a.rplane] = (float)(b6 * a.ig55);
}

// ---------------------------------------------------------------------------
// flow between levels: resize(prevFlow, INTER_LINEAR) then *= 1/pyrScale

struct FbFlowUpArgs {
    const float* src;
    int sw, sh, spitch;
    int64_t splane;
    float* dst;
    int w, h, dpitch;
    int64_t dplane;
    double scale_x, scale_y;
    float alpha;
};

__global__ __launch_bounds__(256) void fb_flow_up_kernel(FbFlowUpArgs a)
{
    const int dx = blockIdx.x * 256 + threadIdx.x;
    const int dy = blockIdx.y;
    if (dx >= a.w) return;
    const LinX lx = lin_x(dx, a.scale_x, a.sw);
    float fy = (float)((dy + 0.5) * a.scale_y - 0.5);
    const int sy = cv_floorf(fy);
    fy -= sy;
    const float b0 = 1.f - fy, b1 = fy, a0 = 1.f - lx.fx, a1 = lx.fx;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        float hrow[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const float* S = a.src + c * a.splane + (size_t)clampi(sy + t, 0, a.sh - 1) * a.spitch;
            hrow[t] = lx.inner ? S[lx.sx] * a0 + S[lx.sx + 1] * a1 : S[lx.sx];
        }
        const float v = hrow[0] * b0 + hrow[1] * b1;
        a.dst[c * a.dplane + (size_t)dy * a.dpitch + dx] = v * a.alpha + 0.0f;  // convertTo(alpha, 0)
    }
}

// OPTFLOW_USE_INITIAL_FLOW: the coarsest level starts from
// resize(flow0, INTER_AREA) *= scale (optflowgf.cpp:1151-1157), read from the
// caller's interleaved CV_32FC2 flow and written to the planar level flow.
// Modes follow cv::resize (imgproc/src/resize.cpp): same size -> copy (:3745);
// integer factors -> resizeAreaFast_'s scalar loop for cn 2 (:2626-2640, sums
// in unrolled groups of 4, then * 1.f/area); otherwise the computeResizeAreaTab
// tables (:2853-2892), which each thread derives for its own cell in double, and
// ResizeArea_Invoker's accumulation order (:2724-2813).  `*= scale` is
// convertTo(alpha = scale, beta = 0), skipped when scale == 1.

enum FbAreaMode { kAreaCopy = 0, kAreaFast = 1, kAreaTable = 2 };

struct FbFlowAreaArgs {
    const float* src;  // interleaved, spitch floats per row
    int sw, sh, spitch;
    float* dst;        // planar: dplane floats between the two components
    int w, h, dpitch;
    int64_t dplane;
    int mode, isx, isy;
    double scale_x, scale_y;
    float alpha;
    int apply_alpha;
};

// one output cell's source span: the entries (s1-1, a_first), (s, a_mid) for
// s in [s1, s2), (s2, a_last) that computeResizeAreaTab emits for it
struct AreaSpan {
    int s1, s2;
    float a_first, a_mid, a_last;
    bool first, last;
};

__device__ __forceinline__ AreaSpan area_span(int d, double scale, int ss)
{
    AreaSpan r;
    const double f1 = d * scale, f2 = f1 + scale;
    const double cell = fmin(scale, ss - f1);
    int s1 = (int)ceil(f1), s2 = (int)floor(f2);
    s2 = min(s2, ss - 1);
    s1 = min(s1, s2);
    r.s1 = s1;
    r.s2 = s2;
    r.first = s1 - f1 > 1e-3;
    r.a_first = (float)((s1 - f1) / cell);
    r.a_mid = (float)(1.0 / cell);
    r.last = f2 - s2 > 1e-3;
    r.a_last = (float)(fmin(fmin(f2 - s2, 1.), cell) / cell);
    return r;
}

// buf = sum over the x entries of S[si] * alpha, for both components
__device__ __forceinline__ float2 area_row(const float* S, const AreaSpan& x)
{
    float2 b = make_float2(0.f, 0.f);
    if (x.first) {
        const float2 v = *reinterpret_cast<const float2*>(S + 2 * (x.s1 - 1));
        b.x = b.x + v.x * x.a_first;
        b.y = b.y + v.y * x.a_first;
    }
    for (int sx = x.s1; sx < x.s2; ++sx) {
        const float2 v = *reinterpret_cast<const float2*>(S + 2 * sx);
        b.x = b.x + v.x * x.a_mid;
        b.y = b.y + v.y * x.a_mid;
    }
    if (x.last) {
        const float2 v = *reinterpret_cast<const float2*>(S + 2 * x.s2);
        b.x = b.x + v.x * x.a_last;
        b.y = b.y + v.y * x.a_last;
    }
    return b;
}

__global__ __launch_bounds__(256) void fb_flow_area_kernel(FbFlowAreaArgs a)
{
    const int dx = blockIdx.x * 256 + threadIdx.x;
    const int dy = blockIdx.y;
    if (dx >= a.w) return;
    float2 r;
    if (a.mode == kAreaCopy) {
        r = *reinterpret_cast<const float2*>(a.src + (size_t)dy * a.spitch + 2 * dx);
    } else if (a.mode == kAreaFast) {
        const float* S = a.src + (size_t)dy * a.isy * a.spitch + (size_t)2 * dx * a.isx;
        const int area = a.isx * a.isy;
        float sx_ = 0.f, sy_ = 0.f;
        // k enumerates (sy, sx) row-major, as the reference's ofs[] table
        int k = 0;
        for (; k <= area - 4; k += 4) {
            float2 v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int kk = k + t, yy = kk / a.isx, xx = kk - yy * a.isx;
                v[t] = *reinterpret_cast<const float2*>(S + (size_t)yy * a.spitch + 2 * xx);
            }
            sx_ += ((v[0].x + v[1].x) + v[2].x) + v[3].x;
            sy_ += ((v[0].y + v[1].y) + v[2].y) + v[3].y;
        }
        for (; k < area; ++k) {
            const int yy = k / a.isx, xx = k - yy * a.isx;
            const float2 v = *reinterpret_cast<const float2*>(S + (size_t)yy * a.spitch + 2 * xx);
            sx_ += v.x;
            sy_ += v.y;
        }
        const float sc = 1.f / area;
        r = make_float2(sx_ * sc, sy_ * sc);
    } else {
        const AreaSpan x = area_span(dx, a.scale_x, a.sw);
        const AreaSpan y = area_span(dy, a.scale_y, a.sh);
        // sum over the y entries in table order; the row's first entry starts it
        bool started = false;
        r = make_float2(0.f, 0.f);
        auto acc = [&](int sy, float beta) {
            const float2 b = area_row(a.src + (size_t)sy * a.spitch, x);
            if (!started) {
                r = make_float2(beta * b.x, beta * b.y);
                started = true;
            } else {
                r.x += beta * b.x;
                r.y += beta * b.y;
            }
        };
        if (y.first) acc(y.s1 - 1, y.a_first);
        for (int sy = y.s1; sy < y.s2; ++sy) acc(sy, y.a_mid);
        if (y.last) acc(y.s2, y.a_last);
    }
    if (a.apply_alpha) {
        r.x = r.x * a.alpha + 0.0f;
        r.y = r.y * a.alpha + 0.0f;
    }
    a.dst[(size_t)dy * a.dpitch + dx] = r.x;
    a.dst[a.dplane + (size_t)dy * a.dpitch + dx] = r.y;
}

// planar -> interleaved CV_32FC2 (numIters == 0 at level 0)
__global__ __launch_bounds__(256) void fb_interleave_kernel(const float* src, int w, int h, int spitch, int64_t splane,
                                                           float* dst, int dpitch)
{
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= w) return;
    const size_t o = (size_t)y * spitch + x;
    float2 v = make_float2(src[o], src[o + splane]);
    *reinterpret_cast<float2*>(dst + (size_t)y * dpitch + 2 * x) = v;
}

// ---------------------------------------------------------------------------
// one iteration: flow_out = solve(blur(M(flow_in, R0, R1)))

struct FbIterArgs {
    const float* fin;  // planes x, y
    float* fout;       // planes x, y (or interleaved when out_il)
    const float* R0;
    const float* R1;
    int w, h, pitch;   // plane pitch (floats)
    int64_t fplane, rplane;
    int seg;           // output rows per workgroup
    int out_il, out_pitch;
    double scale;      // box: 1 / (winsize^2)
    float gk[kFbMaxHalf + 1];  // Gaussian variant: kernel[0..m]
};

__device__ __forceinline__ float fb_border(int i) { return i < 2 ? 0.14f : 0.4472f; }

// 1: each batch's 2x2 solves run at the top of the next batch, beside its M
// rows' finish (whose bilinear R1 terms are selected, not branched around);
// 0: the solve right after the horizontal sums (tuning builds)
#ifndef TBDK_FB_DEFER
#define TBDK_FB_DEFER 1
#endif

// FarnebackUpdateMatrices at pixel (x, y) (optflowgf.cpp:235-309), in three
// phases so a strip can keep two rows of loads in flight: A = the pixel's flow
// and R0 (7 loads), B = the four R1 neighbours of x + flow (20 loads, their
// addresses need A), then the arithmetic.
struct FbRowA {
    float dx, dy, r0[5];
};
struct FbRowB {
    float q[5][4];  // R1 corners (x1,y1) (x1+1,y1) (x1,y1+1) (x1+1,y1+1) per channel
    float fx, fy;   // fractional parts
    bool in;        // (x1, y1) inside [0, w-1) x [0, h-1)
};

// buffer loads: one VGPR byte offset per pixel, the plane / row offsets in SGPRs
struct FbRsrc {
    __amdgpu_buffer_rsrc_t fin, r0, r1;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fb_rsrc(const float* base, int64_t floats)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)(floats * 4), 0x00020000);
}
__device__ __forceinline__ float fb_bload(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

__device__ __forceinline__ void fb_load_a(const FbIterArgs& a, const FbRsrc& rs, int x, int y, FbRowA& A)
{
    const uint32_t o = (uint32_t)(y * a.pitch + x) * 4u;
    const int pl = (int)a.fplane * 4, rpl = (int)a.rplane * 4;
    A.dx = fb_bload(rs.fin, o, 0);
    A.dy = fb_bload(rs.fin, o, pl);
#pragma unroll
    for (int c = 0; c < 5; ++c) A.r0[c] = fb_bload(rs.r0, o, c * rpl);
}

__device__ __forceinline__ void fb_load_b(const FbIterArgs& a, const FbRsrc& rs, int x, int y, const FbRowA& A,
                                          FbRowB& B)
{
    const float fx = (float)x + A.dx, fy = (float)y + A.dy;
    const float ffx = floorf(fx), ffy = floorf(fy);
    // cvFloor (x86: INT_MIN for NaN / out of range); the fraction fx - x1 is
    // only used in range, where it equals fx - floor(fx)
    const int x1 = (ffx >= -2147483648.f && ffx < 2147483648.f) ? (int)ffx : INT_MIN;
    const int y1 = (ffy >= -2147483648.f && ffy < 2147483648.f) ? (int)ffy : INT_MIN;
    B.fx = fx - ffx;
    B.fy = fy - ffy;
    B.in = (unsigned)x1 < (unsigned)(a.w - 1) && (unsigned)y1 < (unsigned)(a.h - 1);
    // out-of-range lanes load a clamped (unused) neighbourhood: no divergent branch
    const int xc = clampi(x1, 0, a.w - 2 < 0 ? 0 : a.w - 2), yc = clampi(y1, 0, a.h - 2 < 0 ? 0 : a.h - 2);
    const uint32_t o = (uint32_t)(yc * a.pitch + xc) * 4u;
    const uint32_t dx1 = a.w > 1 ? 4u : 0u;
    const int dy1 = a.h > 1 ? a.pitch * 4 : 0, rpl = (int)a.rplane * 4;
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        B.q[c][0] = fb_bload(rs.r1, o, c * rpl);
        B.q[c][1] = fb_bload(rs.r1, o + dx1, c * rpl);
        B.q[c][2] = fb_bload(rs.r1, o, c * rpl + dy1);
        B.q[c][3] = fb_bload(rs.r1, o + dx1, c * rpl + dy1);
    }
}

__device__ __forceinline__ void fb_finish(const FbIterArgs& a, int x, int y, const FbRowA& A, const FbRowB& B,
                                          float M[5])
{
    const float dx = A.dx, dy = A.dy;
    const float R00 = A.r0[0], R01 = A.r0[1], R02 = A.r0[2], R03 = A.r0[3], R04 = A.r0[4];
    float r2, r3, r4, r5, r6;
#if TBDK_FB_DEFER
    // the R1 terms evaluated for every pixel and selected by B.in (same
    // values as the branch), so the finish of interior rows is one basic
    // block the deferred solve can interleave with
    {
        const float fx = B.fx, fy = B.fy;
        const float a00 = (1.f - fx) * (1.f - fy), a01 = fx * (1.f - fy), a10 = (1.f - fx) * fy, a11 = fx * fy;
        float r[5];
#pragma unroll
        for (int c = 0; c < 5; ++c) r[c] = a00 * B.q[c][0] + a01 * B.q[c][1] + a10 * B.q[c][2] + a11 * B.q[c][3];
        r2 = B.in ? r[0] : 0.f;
        r3 = B.in ? r[1] : 0.f;
        r4 = B.in ? (R02 + r[2]) * 0.5f : R02;
        r5 = B.in ? (R03 + r[3]) * 0.5f : R03;
        r6 = B.in ? (R04 + r[4]) * 0.25f : R04 * 0.5f;
    }
#else
    if (B.in) {
        const float fx = B.fx, fy = B.fy;
        const float a00 = (1.f - fx) * (1.f - fy), a01 = fx * (1.f - fy), a10 = (1.f - fx) * fy, a11 = fx * fy;
        float r[5];
#pragma unroll
        for (int c = 0; c < 5; ++c) r[c] = a00 * B.q[c][0] + a01 * B.q[c][1] + a10 * B.q[c][2] + a11 * B.q[c][3];
        r2 = r[0];
        r3 = r[1];
        r4 = (R02 + r[2]) * 0.5f;
        r5 = (R03 + r[3]) * 0.5f;
        r6 = (R04 + r[4]) * 0.25f;
    } else {
        r2 = r3 = 0.f;
        r4 = R02;
        r5 = R03;
        r6 = R04 * 0.5f;
    }
#endif
    r2 = (R00 - r2) * 0.5f;
    r3 = (R01 - r3) * 0.5f;
    r2 += r4 * dy + r6 * dx;
    r3 += r6 * dy + r5 * dx;
    if ((unsigned)(x - 5) >= (unsigned)(a.w - 10) || (unsigned)(y - 5) >= (unsigned)(a.h - 10)) {
        const float scale = (x < 5 ? fb_border(x) : 1.f) * (x >= a.w - 5 ? fb_border(a.w - x - 1) : 1.f) *
                            (y < 5 ? fb_border(y) : 1.f) * (y >= a.h - 5 ? fb_border(a.h - y - 1) : 1.f);
        r2 *= scale;
        r3 *= scale;
        r4 *= scale;
        r5 *= scale;
        r6 *= scale;
    }
    M[0] = r4 * r4 + r6 * r6;
    M[1] = (r4 + r5) * r6;
    M[2] = r5 * r5 + r6 * r6;
    M[3] = r4 * r2 + r6 * r3;
    M[4] = r6 * r2 + r5 * r3;
}

// LDS slot of strip lane l: one pad double every 4, so the horizontal runs
// (thread q reads lanes 4q..4q+3+2m) hit distinct banks
//
// TBDK_FB_W64 (round 6): the horizontal windows read as 8-byte pairs
// (ds_read_b64: twice the bytes per LDS cycle of ds_read_b32); the windows
// start at even columns, so the row is unpadded, and rows (channel, batch
// row) are kFbStrip + 2 floats apart — an odd number of 8-byte banks — so the
// 32 lanes of a read group, 16 distinct windows of one row or the tail of one
// row and the head of the next, hit distinct banks (tools/r06_fb_lds.sh)
#ifndef TBDK_FB_W64
#define TBDK_FB_W64 1
#endif
#if TBDK_FB_W64
__device__ __forceinline__ int fb_slot(int l) { return l; }
constexpr int kFbSlots = kFbStrip + 2;
#else
__device__ __forceinline__ int fb_slot(int l) { return l + (l >> 2); }
constexpr int kFbSlots = kFbStrip + kFbStrip / 4;
#endif
// the window values row[l0 .. l0 + NW) (l0 and NW even under TBDK_FB_W64)
template <int NW>
__device__ __forceinline__ void fb_window(const float* row, int l0, float (&win)[NW])
{
#if TBDK_FB_W64
    static_assert(NW % 2 == 0, "8-byte pairs");
#pragma unroll
    for (int i = 0; i < NW; i += 2) {
        // volatile: one ds_read_b64 per pair (the load merger otherwise pairs
        // them into ds_read2_b64, which moves 128 B per LDS cycle, as b32 does)
        typedef const volatile __attribute__((address_space(3))) uint64_t lds_u64;
        const uint64_t p = *(lds_u64*)(row + min(l0 + i, kFbStrip - 2));
        win[i] = __uint_as_float((uint32_t)p);
        win[i + 1] = __uint_as_float((uint32_t)(p >> 32));
    }
#else
#pragma unroll
    for (int i = 0; i < NW; ++i) win[i] = row[fb_slot(min(l0 + i, kFbStrip - 1))];
#endif
}

// horizontal window + 2x2 solve of one batch row: thread task -> (row r, TK
// consecutive output columns starting at strip offset o0).  Box sums restart at
// every strip offset divisible by 4 (image columns divisible by 4) and slide
// from there, whatever TK is, so the sums do not depend on the task split.
#ifndef TBDK_FB_TK
#define TBDK_FB_TK 2  // output columns per horizontal task (2: twice the threads in the solve phase)
#endif
constexpr int kFbTK = TBDK_FB_TK;
// 1 (tuning builds): 4-column horizontal tasks in half-waves, outputs handed
// to the other half by v_permlane32_swap (requires kFbTK == 2 and the deferred solve)
#ifndef TBDK_FB_HX
#define TBDK_FB_HX 0
#endif
static_assert(!TBDK_FB_HX || kFbTK == 2, "TBDK_FB_HX takes 2-column solves");
static_assert(kFbTK == 2 || kFbTK == 4, "tasks of 2 or 4 columns");
template <int M, bool GAUSS, int TK = kFbTK>
__device__ __forceinline__ void fb_hsums(const FbIterArgs& a, const float (*vb)[5][kFbSlots], int r, int o0,
                                         float (&out)[5][TK])
{
    const int g0 = o0 & ~3, sk = o0 - g0;  // the box sums' group start, slides to o0 (0 or 2)
#pragma unroll
    for (int ch = 0; ch < 5; ++ch) {
        const float* row = vb[r][ch];
        if (GAUSS) {
            // optflowgf.cpp:548-553: sum = v[x]*k0; sum += k[i]*(v[x-i] + v[x+i])
            constexpr int NW = TK + 2 * M;
            float win[NW];
            fb_window<NW>(row, o0, win);
#pragma unroll
            for (int k = 0; k < TK; ++k) {
                float s = win[k + M] * a.gk[0];
#pragma unroll
                for (int i = 1; i <= M; ++i) s += a.gk[i] * (win[k + M - i] + win[k + M + i]);
                out[ch][k] = s;
            }
        } else {
            // window of group start g0 summed from the left, then slid:
            // out(c) = (out(c-1) + v[c+2m]) - v[c-1]
            constexpr int NW = 4 + 2 * M;
            float win[NW];
            fb_window<NW>(row, g0, win);
            float sacc = win[0];
#pragma unroll
            for (int i = 1; i <= 2 * M; ++i) sacc += win[i];
            float v[4];
            v[0] = sacc;
#pragma unroll
            for (int k = 1; k < 4; ++k) v[k] = (v[k - 1] + win[k + 2 * M]) - win[k - 1];
#pragma unroll
            for (int k = 0; k < TK; ++k) out[ch][k] = TK == 4 ? v[k] : (sk ? v[2 + k] : v[k]);
        }
    }
}

// the 2x2 solve (optflowgf.cpp:190-200) of a horizontal task's TK outputs and
// their stores; `ok` false: nothing stored
template <int M, bool GAUSS>
__device__ __forceinline__ void fb_solve(const FbIterArgs& a, const float (&out)[5][kFbTK], int o0, int y, int ox0,
                                         bool ok)
{
    constexpr int TK = kFbTK;
    constexpr int OW = fb_ow(M);
    float rx[TK], ry[TK];
#pragma unroll
    for (int k = 0; k < TK; ++k) {
        double g11, g12, g22, h1, h2;
        if (GAUSS) {
            g11 = out[0][k];
            g12 = out[1][k];
            g22 = out[2][k];
            h1 = out[3][k];
            h2 = out[4][k];
        } else {
            g11 = out[0][k] * a.scale;
            g12 = out[1][k] * a.scale;
            g22 = out[2][k] * a.scale;
            h1 = out[3][k] * a.scale;
            h2 = out[4][k] * a.scale;
        }
        const double idet = 1. / (g11 * g22 - g12 * g12 + 1e-3);
        rx[k] = (float)((g11 * h2 - g12 * h1) * idet);
        ry[k] = (float)((g22 * h1 - g12 * h2) * idet);
    }
#pragma unroll
    for (int k = 0; k < TK; ++k) {
        const int o = o0 + k, x = ox0 + o;
        if (!ok || o >= OW || x >= a.w) break;
        if (a.out_il) {
            *reinterpret_cast<float2*>(a.fout + (size_t)y * a.out_pitch + 2 * x) = make_float2(rx[k], ry[k]);
        } else {
            const size_t off = (size_t)y * a.pitch + x;
            a.fout[off] = rx[k];
            a.fout[off + a.fplane] = ry[k];
        }
    }
}

template <int M, bool GAUSS>
__device__ __forceinline__ void fb_horizontal(const FbIterArgs& a, const float (*vb)[5][kFbSlots], int r, int o0,
                                              int y, int ox0)
{
    float out[5][kFbTK];
    fb_hsums<M, GAUSS>(a, vb, r, o0, out);
    fb_solve<M, GAUSS>(a, out, o0, y, ox0, true);
}

// workgroup barrier that waits only for LDS traffic
__device__ __forceinline__ void fb_lds_barrier()
{
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
}

#ifndef TBDK_FB_RB
#define TBDK_FB_RB 4
#endif
constexpr int kFbRB = TBDK_FB_RB;  // output rows per batch of fb_iter (4 or 8)
constexpr int kFbThreads = 256; // two threads per strip column

// M of NR rows t0 + half, t0 + half + 2, ... (relative to the segment's first
// M row) of column x into the LDS ring: every row's loads are issued before
// any row waits (A loads, then the dependent R1 gathers)
// the three phases of M for NR rows t0 + half + 2i of column x, split so a
// batch's loads can be in flight while the previous batch is summed
template <int NR>
__device__ __forceinline__ void fb_rows_a(const FbIterArgs& a, const FbRsrc& rs, int x, int ybase, int t0, int half,
                                          FbRowA (&A)[NR])
{
#pragma unroll
    for (int i = 0; i < NR; ++i) fb_load_a(a, rs, x, clampi(ybase + t0 + half + 2 * i, 0, a.h - 1), A[i]);
}
template <int NR>
__device__ __forceinline__ void fb_rows_b(const FbIterArgs& a, const FbRsrc& rs, int x, int ybase, int t0, int half,
                                          const FbRowA (&A)[NR], FbRowB (&B)[NR])
{
#pragma unroll
    for (int i = 0; i < NR; ++i) fb_load_b(a, rs, x, clampi(ybase + t0 + half + 2 * i, 0, a.h - 1), A[i], B[i]);
}
template <int NR>
__device__ __forceinline__ void fb_rows_finish(const FbIterArgs& a, float* mr, int rr, int x, int col, int ybase,
                                               int t0, int half, const FbRowA (&A)[NR], const FbRowB (&B)[NR])
{
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        float Mv[5];
        const int t = t0 + half + 2 * i;
        fb_finish(a, x, clampi(ybase + t, 0, a.h - 1), A[i], B[i], Mv);
        float* dst = mr + (t % rr) * kFbStrip + col;
#pragma unroll
        for (int ch = 0; ch < 5; ++ch) dst[ch * rr * kFbStrip] = Mv[ch];
    }
}
template <int NR>
__device__ __forceinline__ void fb_rows(const FbIterArgs& a, const FbRsrc& rs, float* mr, int rr, int x, int col,
                                        int ybase, int t0, int half)
{
    FbRowA A[NR];
    FbRowB B[NR];
    fb_rows_a<NR>(a, rs, x, ybase, t0, half, A);
    fb_rows_b<NR>(a, rs, x, ybase, t0, half, A, B);
    fb_rows_finish<NR>(a, mr, rr, x, col, ybase, t0, half, A, B);
}

// One workgroup = one 128-column strip (m halo columns per side) over the
// output rows [y0, y0 + seg).  M of the strip's rows lives in an LDS ring of
// kFbRB + 2m rows; each batch computes kFbRB new rows (two threads per column,
// all their loads in flight together), then the vertical windows (box: exact-
// order float sum; Gaussian: the reference's float weighted sum) of kFbRB
// centre rows, then the horizontal windows and the solve.  Every value is a
// fixed-order function of the pixel's neighbourhood, independent of the
// strip/segment split.
template <int M, bool GAUSS>
__global__ __launch_bounds__(kFbThreads, (kFbRB == 8 ? (M <= 6 && !GAUSS ? 2 : 1)
                                                       : (M <= 6 ? (GAUSS ? 2 : 3) : (GAUSS ? 1 : 2)))) void fb_iter_kernel(FbIterArgs a)
{
    constexpr int K = 2 * M + 1;
    constexpr int OW = fb_ow(M);
    [[maybe_unused]] constexpr int NQ = (OW + kFbTK - 1) / kFbTK;  // horizontal tasks per row
    constexpr int RR = kFbRB + 2 * M;     // M ring rows
    constexpr int VC = 4;                 // centres per thread in the vertical pass
    __shared__ float mr[5 * RR * kFbStrip];
    __shared__ __attribute__((aligned(16))) float vb[kFbRB][5][kFbSlots];

    const int tid = threadIdx.x;
    const int col = tid & (kFbStrip - 1), half = tid >> 7;
    const int ox0 = blockIdx.x * OW;
    const int x = clampi(ox0 - M + col, 0, a.w - 1);
    const int y0 = blockIdx.y * a.seg;
    const int nrows = min(a.h, y0 + a.seg) - y0;
    const int ybase = y0 - M;  // M row t (relative) is image row ybase + t (clamped)
    const int sl = fb_slot(col);

    const int64_t plane_end = (int64_t)a.h * a.pitch;
    const FbRsrc rs{fb_rsrc(a.fin, a.fplane + plane_end), fb_rsrc(a.R0, 4 * a.rplane + plane_end),
                    fb_rsrc(a.R1, 4 * a.rplane + plane_end)};
    // warm-up rows 0 .. 2m-1: batch-sized chunks, then the remainder
    for (int t = 0; t + kFbRB <= 2 * M; t += kFbRB) fb_rows<kFbRB / 2>(a, rs, mr, RR, x, col, ybase, t, half);
    if constexpr ((2 * M) % kFbRB != 0)
        fb_rows<((2 * M) % kFbRB) / 2>(a, rs, mr, RR, x, col, ybase, 2 * M - (2 * M) % kFbRB, half);
    // batch pipeline: the M rows of batch s0 + kFbRB are loaded (A during the
    // vertical pass, the dependent R1 gathers B during the horizontal pass of
    // batch s0) before they are finished at the top of the next iteration
    constexpr int NR = kFbRB / 2;
    FbRowA A[NR];
    FbRowB B[NR];
    fb_rows_a<NR>(a, rs, x, ybase, 2 * M, half, A);
    fb_rows_b<NR>(a, rs, x, ybase, 2 * M, half, A, B);
#if TBDK_FB_DEFER
    // the solve of batch s0's horizontal task runs at the top of the next
    // iteration, in one basic block with the next M rows' finish (independent
    // work the scheduler interleaves with the double-precision chain)
    static_assert(kFbRB * ((OW + kFbTK - 1) / kFbTK) <= kFbThreads, "one horizontal task per thread and batch (TBDK_FB_RB=8 builds: TBDK_FB_DEFER=0)");
    float pend[5][kFbTK];
    int pend_o0 = 0, pend_y = 0;
    bool pend_ok = false;
#endif
    for (int s0 = 0; s0 < nrows; s0 += kFbRB) {
        fb_rows_finish<NR>(a, mr, RR, x, col, ybase, 2 * M + s0, half, A, B);
#if TBDK_FB_DEFER
        fb_solve<M, GAUSS>(a, pend, pend_o0, pend_y, ox0, pend_ok);
#endif
        const bool more = s0 + kFbRB < nrows;
        if (more) fb_rows_a<NR>(a, rs, x, ybase, 2 * M + s0 + kFbRB, half, A);
        fb_lds_barrier();
        // vertical windows of centres s0 + cb + j: relative rows c .. c+2m
        // (batch of 8: each half takes 4 centres; batch of 4: the halves split
        // the channels, 0-2 and 3-4)
        const int cb = kFbRB == 8 ? half * VC : 0;
#pragma unroll
        for (int ch = 0; ch < 5; ++ch) {
            if (kFbRB == 4 && (ch < 3) != (half == 0)) continue;
            const float* m = mr + ch * RR * kFbStrip + col;
            float win[VC + 2 * M];
            float prev = 0.f;
#pragma unroll
            for (int i = 0; i < VC + 2 * M; ++i) win[i] = m[((s0 + cb + i) % RR) * kFbStrip];
#pragma unroll
            for (int j = 0; j < VC; ++j) {
                float v;
                if (GAUSS) {
                    // optflowgf.cpp:509-515: s0 = M(c)*k0; s0 += (M(c+i) + M(c-i))*k[i]
                    v = win[j + M] * a.gk[0];
#pragma unroll
                    for (int i = 1; i <= M; ++i) v += (win[j + M + i] + win[j + M - i]) * a.gk[i];
                } else {
                    // rows c-m .. c+m: summed from the top at the batch's first
                    // centre (image row divisible by 4), then slid
                    if (j == 0) {
                        v = win[0];
#pragma unroll
                        for (int i = 1; i < K; ++i) v += win[i];
                    } else {
                        v = (prev + win[j + 2 * M]) - win[j - 1];
                    }
                    prev = v;
                }
                vb[cb + j][ch][sl] = v;
            }
        }
        if (more) fb_rows_b<NR>(a, rs, x, ybase, 2 * M + s0 + kFbRB, half, A, B);
        fb_lds_barrier();
        const int nb = min(kFbRB, nrows - s0);
#if TBDK_FB_DEFER && TBDK_FB_HX
        {
            // tasks of 4 columns in lanes 0-31 of each wave (half the LDS reads of
            // two 2-column tasks); v_permlane32_swap hands outputs 2-3 to lanes
            // 32-63, so every lane still solves 2 (bit-identical sums: the box
            // sums restart at the same columns)
            constexpr int NQ4 = (OW + 3) / 4;
            const int lane = tid & 63, task = (tid >> 6) * 32 + (lane & 31);
            const bool in = task < nb * NQ4;
            const int r = in ? task / NQ4 : 0, q = in ? task - r * NQ4 : 0;
            float o4[5][4];
            if (lane < 32) fb_hsums<M, GAUSS, 4>(a, vb, r, 4 * q, o4);
#pragma unroll
            for (int ch = 0; ch < 5; ++ch) {
                const auto p2 = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, o4[ch][0]),
                                                                 __builtin_bit_cast(unsigned, o4[ch][2]), false, false);
                const auto p3 = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, o4[ch][1]),
                                                                 __builtin_bit_cast(unsigned, o4[ch][3]), false, false);
                pend[ch][0] = lane < 32 ? o4[ch][0] : __builtin_bit_cast(float, p2[0]);
                pend[ch][1] = lane < 32 ? o4[ch][1] : __builtin_bit_cast(float, p3[0]);
            }
            pend_o0 = 4 * q + (lane < 32 ? 0 : 2);
            pend_ok = in && ox0 + pend_o0 < a.w;
            pend_y = y0 + s0 + r;
        }
#elif TBDK_FB_DEFER
        {
            const bool in = tid < nb * NQ;
            const int r = in ? tid / NQ : 0, q = in ? tid - r * NQ : 0;
            pend_ok = in && ox0 + kFbTK * q < a.w;
            pend_o0 = kFbTK * q;
            pend_y = y0 + s0 + r;
            fb_hsums<M, GAUSS>(a, vb, r, pend_o0, pend);
        }
#else
        for (int task = tid; task < nb * NQ; task += kFbThreads) {
            const int r = task / NQ, q = task - r * NQ;
            if (ox0 + kFbTK * q < a.w) fb_horizontal<M, GAUSS>(a, vb, r, kFbTK * q, y0 + s0 + r, ox0);
        }
#endif
        // the next batch's M rows overwrite ring rows the vertical pass read,
        // and its vertical pass vb rows this horizontal pass reads: both are
        // ordered by the two barriers above (this pass ends before the next
        // batch's first barrier)
    }
#if TBDK_FB_DEFER
    fb_solve<M, GAUSS>(a, pend, pend_o0, pend_y, ox0, pend_ok);
#endif
}

template <int M>
hipError_t launch_fb_iter_m(const FbIterArgs& a, bool gauss, dim3 grid, hipStream_t s)
{
    if (gauss) hipLaunchKernelGGL((fb_iter_kernel<M, true>), grid, dim3(kFbThreads), 0, s, a);
    else hipLaunchKernelGGL((fb_iter_kernel<M, false>), grid, dim3(kFbThreads), 0, s, a);
    return hipGetLastError();
}

// resident fb_iter workgroups per CU (occupancy of the instance for m, gauss)
template <int M>
int fb_iter_occ_m(bool gauss)
{
    int n = 0;
    hipError_t e = gauss ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fb_iter_kernel<M, true>, kFbThreads, 0)
                         : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fb_iter_kernel<M, false>, kFbThreads, 0);
    return e == hipSuccess && n > 0 ? n : 1;
}

int fb_iter_occupancy(int m, bool gauss)
{
    switch (m) {
    case 0: return fb_iter_occ_m<0>(gauss);
    case 1: return fb_iter_occ_m<1>(gauss);
    case 2: return fb_iter_occ_m<2>(gauss);
    case 3: return fb_iter_occ_m<3>(gauss);
    case 4: return fb_iter_occ_m<4>(gauss);
    case 5: return fb_iter_occ_m<5>(gauss);
    case 6: return fb_iter_occ_m<6>(gauss);
    case 7: return fb_iter_occ_m<7>(gauss);
    case 8: return fb_iter_occ_m<8>(gauss);
    case 9: return fb_iter_occ_m<9>(gauss);
    case 10: return fb_iter_occ_m<10>(gauss);
    default: return 1;
    }
}

hipError_t launch_fb_iter(const FbIterArgs& a, int m, bool gauss, hipStream_t s)
{
    const int ow = fb_ow(m);
    const int nstrips = (a.w + ow - 1) / ow;
    const int nseg = (a.h + a.seg - 1) / a.seg;
    const dim3 grid(nstrips, nseg);
    switch (m) {
    case 0: return launch_fb_iter_m<0>(a, gauss, grid, s);
    case 1: return launch_fb_iter_m<1>(a, gauss, grid, s);
    case 2: return launch_fb_iter_m<2>(a, gauss, grid, s);
    case 3: return launch_fb_iter_m<3>(a, gauss, grid, s);
    case 4: return launch_fb_iter_m<4>(a, gauss, grid, s);
    case 5: return launch_fb_iter_m<5>(a, gauss, grid, s);
    case 6: return launch_fb_iter_m<6>(a, gauss, grid, s);
    case 7: return launch_fb_iter_m<7>(a, gauss, grid, s);
    case 8: return launch_fb_iter_m<8>(a, gauss, grid, s);
    case 9: return launch_fb_iter_m<9>(a, gauss, grid, s);
    case 10: return launch_fb_iter_m<10>(a, gauss, grid, s);
    default: return hipErrorInvalidValue;
    }
}

// ---------------------------------------------------------------------------
// host helpers: the reference's kernels (computed on the host, as it does)

int cv_round(double v) { return (int)lrint(v); }

// getGaussianKernel(n, sigma, CV_32F) (imgproc/src/smooth.dispatch.cpp:70-122)
void gaussian_kernel(int n, double sigma, float* cf)
{
    static const float tab[4][7] = {{1.f},
                                    {0.25f, 0.5f, 0.25f},
                                    {0.0625f, 0.25f, 0.375f, 0.25f, 0.0625f},
                                    {0.03125f, 0.109375f, 0.21875f, 0.28125f, 0.21875f, 0.109375f, 0.03125f}};
    const float* fixed = (n % 2 == 1 && n <= 7 && sigma <= 0) ? tab[n >> 1] : nullptr;
    const double sigmaX = sigma > 0 ? sigma : ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
    const double scale2X = -0.5 / (sigmaX * sigmaX);
    double sum = 0;
    for (int i = 0; i < n; i++) {
        const double x = i - (n - 1) * 0.5;
        const double t = fixed ? (double)fixed[i] : std::exp(scale2X * x * x);
        cf[i] = (float)t;
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; i++) cf[i] = (float)(cf[i] * sum);
}

// FarnebackPrepareGaussian (optflowgf.cpp:60-114) incl. invert(G, DECOMP_CHOLESKY)
// (hal::Cholesky64f, core/src/matrix_decomp.cpp:95-170)
void prepare_gaussian(int n, double sigma, float* g, float* xg, float* xxg, double* ig)
{
    if (sigma < FLT_EPSILON) sigma = n * 0.3;
    float gb[2 * kFbMaxPolyN + 1], xgb[2 * kFbMaxPolyN + 1], xxgb[2 * kFbMaxPolyN + 1];
    float* G_ = gb + n;
    float* XG = xgb + n;
    float* XXG = xxgb + n;
    double s = 0.;
    for (int x = -n; x <= n; x++) {
        G_[x] = (float)std::exp(-x * x / (2 * sigma * sigma));
        s += G_[x];
    }
    s = 1. / s;
    for (int x = -n; x <= n; x++) {
        G_[x] = (float)(G_[x] * s);
        XG[x] = (float)(x * G_[x]);
        XXG[x] = (float)(x * x * G_[x]);
    }
    double G[36] = {0};
    for (int y = -n; y <= n; y++)
        for (int x = -n; x <= n; x++) {
            G[0] += G_[y] * G_[x];
            G[7] += G_[y] * G_[x] * x * x;
            G[21] += G_[y] * G_[x] * x * x * x * x;
            G[35] += G_[y] * G_[x] * x * x * y * y;
        }
    G[14] = G[3] = G[4] = G[18] = G[24] = G[7];
    G[28] = G[21];
    G[22] = G[27] = G[35];
    double* A = G;
    double b[36] = {0};
    for (int i = 0; i < 6; i++) b[i * 6 + i] = 1;
    int i, j, k;
    for (i = 0; i < 6; i++) {
        for (j = 0; j < i; j++) {
            s = A[i * 6 + j];
            for (k = 0; k < j; k++) s -= A[i * 6 + k] * A[j * 6 + k];
            A[i * 6 + j] = s * A[j * 6 + j];
        }
        s = A[i * 6 + i];
        for (k = 0; k < j; k++) {
            const double t = A[i * 6 + k];
            s -= t * t;
        }
        A[i * 6 + i] = 1. / std::sqrt(s);
    }
    for (i = 0; i < 6; i++)
        for (j = 0; j < 6; j++) {
            s = b[i * 6 + j];
            for (k = 0; k < i; k++) s -= A[i * 6 + k] * b[k * 6 + j];
            b[i * 6 + j] = s * A[i * 6 + i];
        }
    for (i = 5; i >= 0; i--)
        for (j = 0; j < 6; j++) {
            s = b[i * 6 + j];
            for (k = 5; k > i; k--) s -= A[k * 6 + i] * b[k * 6 + j];
            b[i * 6 + j] = s * A[i * 6 + i];
        }
    ig[0] = b[1 * 6 + 1];
    ig[1] = b[0 * 6 + 3];
    ig[2] = b[3 * 6 + 3];
    ig[3] = b[5 * 6 + 5];
    for (int x = 0; x <= n; x++) {
        g[x] = G_[x];
        xg[x] = XG[x];
        xxg[x] = XXG[x];
    }
}

struct LevelImagePlan {
    int mode, nc, ks;
    double scale_x, scale_y;
    float k[kFbMaxKs];
};

// resize()'s path choice for (W,H) -> (w,h) (resize.cpp:3483-3550)
int plan_level_image(int W, int H, int w, int h, int ks, double sigma, LevelImagePlan* p)
{
    if (ks < 1 || ks > kFbMaxKs || !(ks & 1)) return TBDK_EINVAL;
    p->ks = ks;
    gaussian_kernel(ks, sigma, p->k);
    p->scale_x = 1. / ((double)w / W);
    p->scale_y = 1. / ((double)h / H);
    if (w == W && h == H) {
        p->mode = kModeNone;
        p->nc = W;
        return TBDK_OK;
    }
    const int isx = cv_round(p->scale_x), isy = cv_round(p->scale_y);
    const bool fast = std::fabs(p->scale_x - isx) < DBL_EPSILON && std::fabs(p->scale_y - isy) < DBL_EPSILON;
    if (fast && isx == 2 && isy == 2) {
        p->mode = kModeArea2;
        p->nc = W;
    } else {
        p->mode = kModeLinear;
        p->nc = 2 * w;
    }
    return TBDK_OK;
}

hipError_t launch_level_image(const LevelImagePlan& p, const uint8_t* img, int W, int H, int pitch, float* T,
                              int tpitch, float* I, int w, int h, int ipitch, hipStream_t s)
{
    FbRowArgs ra;
    ra.img = img;
    ra.W = W;
    ra.H = H;
    ra.pitch = pitch;
    ra.T = T;
    ra.tpitch = tpitch;
    ra.nc = p.nc;
    ra.mode = p.mode;
    ra.scale_x = p.scale_x;
    ra.ks = p.ks;
    std::memcpy(ra.k, p.k, sizeof(float) * p.ks);
    // LDS for the wide-kernel path: one block's column span plus the border
    const size_t span = p.mode == kModeLinear ? (size_t)std::ceil(128.0 * p.scale_x) + 4 : 256;
    const size_t smem = p.ks > 5 ? (span + 2 * (p.ks >> 1) + 16 + 15) & ~(size_t)15 : 0;
    hipLaunchKernelGGL(fb_rowpass_kernel, dim3((p.nc + 255) / 256, H), dim3(256), smem, s, ra);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    FbColArgs ca;
    ca.T = T;
    ca.tpitch = tpitch;
    ca.H = H;
    ca.W = W;
    ca.I = I;
    ca.w = w;
    ca.h = h;
    ca.ipitch = ipitch;
    ca.mode = p.mode;
    ca.scale_x = p.scale_x;
    ca.scale_y = p.scale_y;
    ca.ks = p.ks;
    std::memcpy(ca.k, p.k, sizeof(float) * p.ks);
    hipLaunchKernelGGL(fb_colpass_kernel, dim3((w + 255) / 256, h), dim3(256), 0, s, ca);
    return hipGetLastError();
}

hipError_t launch_polyexp(const float* I, int w, int h, int ipitch, float* R, int rpitch, int64_t rplane, int n,
                          double sigma, hipStream_t s)
{
    FbPolyArgs a;
    a.I = I;
    a.w = w;
    a.h = h;
    a.ipitch = ipitch;
    a.R = R;
    a.rpitch = rpitch;
    a.rplane = rplane;
    a.n = n;
    double ig[4];
    prepare_gaussian(n, sigma, a.g, a.xg, a.xxg, ig);
    a.ig11 = ig[0];
    a.ig03 = ig[1];
    a.ig33 = ig[2];
    a.ig55 = ig[3];
    hipLaunchKernelGGL(fb_polyexp_kernel, dim3((w + 255) / 256, h), dim3(256), 0, s, a);
    return hipGetLastError();
}

inline int plane_pitch(int w) { return align_up(w, 64); }
inline int64_t plane_stride(int pp, int h) { return (int64_t)pp * h; }

// rows per fb_iter workgroup (a multiple of the batch) for `wgs` workgroups in
// total.  Longer segments pay the 2m warm-up rows of M less often, fewer
// workgroups hide less latency: the caller asks for whole rounds of resident
// workgroups, at least 3 per CU (4K, win 13: box 768 = one round of 3 per CU
// beat 512 / 1024 / 1536 by 4-13 %; Gaussian 1024 = two rounds of 2 per CU
// beat 512 / 768 / 1536 by 1-13 %).  Small levels get one batch per workgroup
// so their serial chain of round trips stays short.
int iter_seg(int w, int h, int m, int wgs)
{
    const int ow = fb_ow(m);
    const int nstrips = (w + ow - 1) / ow;
    const int target = wgs;
    const int nseg = (target + nstrips - 1) / nstrips;
    int seg = (h + nseg - 1) / nseg;
    seg = (seg + kFbRB - 1) / kFbRB * kFbRB;
    return seg < kFbRB ? kFbRB : seg;
}

int fb_reserve(tbdk_ctx* ctx, int64_t px, int64_t tcap)
{
    FbScratch* f = ctx->fb;
    if (!f) {
        f = new (std::nothrow) FbScratch();
        if (!f) return TBDK_ENOMEM;
        ctx->fb = f;
    }
    if (px > f->cap_px) {
        (void)hipFree(f->R0);
        f->R0 = f->R1 = f->F[0] = f->F[1] = f->I = nullptr;
        f->cap_px = 0;
        float* base = nullptr;
        // R0 (5) + R1 (5) + F0 (2) + F1 (2) + I (1) planes in one allocation
        if (hipMalloc(&base, sizeof(float) * (size_t)px * 15) != hipSuccess) return TBDK_ENOMEM;
        f->R0 = base;
        f->R1 = base + px * 5;
        f->F[0] = base + px * 10;
        f->F[1] = base + px * 12;
        f->I = base + px * 14;
        f->cap_px = px;
    }
    if (tcap > f->cap_T) {
        (void)hipFree(f->T);
        f->T = nullptr;
        f->cap_T = 0;
        if (hipMalloc(&f->T, sizeof(float) * (size_t)tcap) != hipSuccess) return TBDK_ENOMEM;
        f->cap_T = tcap;
    }
    return TBDK_OK;
}

struct FbLevel {
    int w, h, ks;
    double sigma;
};

// the prep stream, its events and the per-level R planes (rfloats in all)
int fb_reserve_ahead(FbScratch* f, int64_t rfloats, int nlev)
{
    if (!f->prep && hipStreamCreateWithFlags(&f->prep, hipStreamNonBlocking) != hipSuccess) return TBDK_EHIP;
    if (!f->fork && hipEventCreateWithFlags(&f->fork, hipEventDisableTiming) != hipSuccess) return TBDK_EHIP;
    for (int k = 0; k < nlev; ++k)
        if (!f->lev_ev[k] && hipEventCreateWithFlags(&f->lev_ev[k], hipEventDisableTiming) != hipSuccess)
            return TBDK_EHIP;
    if (rfloats > f->cap_Rl) {
        (void)hipFree(f->Rl);
        f->Rl = nullptr;
        f->cap_Rl = 0;
        if (hipMalloc(&f->Rl, sizeof(float) * (size_t)rfloats) != hipSuccess) return TBDK_ENOMEM;
        f->cap_Rl = rfloats;
    }
    return TBDK_OK;
}

int fb_check(const tbdk_farneback_params* p)
{
    if (!p) return TBDK_EINVAL;
    if (!(p->pyr_scale < 1)) return TBDK_EINVAL;  // CV_Assert(pyrScale_ < 1) (optflowgf.cpp:1113-1114)
    if (p->fast_pyramids) return TBDK_EINVAL;      // CUDA-only pyrDown pyramids: not provided
    if (p->win_size < 1 || p->win_size / 2 > kFbMaxHalf) return TBDK_EINVAL;
    if (p->num_iters < 0) return TBDK_EINVAL;
    if (p->poly_n < 1 || p->poly_n > kFbMaxPolyN) return TBDK_EINVAL;
    if (p->flags & ~(TBDK_OPTFLOW_FARNEBACK_GAUSSIAN | TBDK_OPTFLOW_USE_INITIAL_FLOW)) return TBDK_EINVAL;
    return TBDK_OK;
}

}  // namespace

// Called by tbdk_ctx_create: the prep stream exists before the caller's later
// streams (HIP maps streams onto a few hardware queues in creation order; a prep
// stream created after a TBD loop's streams measured 259 instead of 288 pairs/s)
void fb_create_streams(tbdk_ctx* ctx)
{
    if (!ctx->fb) ctx->fb = new (std::nothrow) FbScratch();
    FbScratch* f = ctx->fb;
    if (f && !f->prep && hipStreamCreateWithFlags(&f->prep, hipStreamNonBlocking) != hipSuccess) f->prep = nullptr;
}

void fb_release(tbdk_ctx* ctx)
{
    if (!ctx || !ctx->fb) return;
    (void)hipFree(ctx->fb->R0);
    (void)hipFree(ctx->fb->T);
    if (ctx->fb->Rl) (void)hipFree(ctx->fb->Rl);
    if (ctx->fb->prep) (void)hipStreamDestroy(ctx->fb->prep);
    if (ctx->fb->fork) (void)hipEventDestroy(ctx->fb->fork);
    if (ctx->fb->done) (void)hipEventDestroy(ctx->fb->done);
    for (hipEvent_t ev : ctx->fb->lev_ev)
        if (ev) (void)hipEventDestroy(ev);
    delete ctx->fb;
    ctx->fb = nullptr;
}

}  // namespace tbdk

using namespace tbdk;

extern "C" {

int tbdk_farneback_default_params(tbdk_farneback_params* p)
{
    if (!p) return TBDK_EINVAL;
    // cv::cuda::FarnebackOpticalFlow::create defaults (cudaoptflow.hpp:242-250)
    p->num_levels = 5;
    p->pyr_scale = 0.5;
    p->fast_pyramids = 0;
    p->win_size = 13;
    p->num_iters = 10;
    p->poly_n = 5;
    p->poly_sigma = 1.1;
    p->flags = 0;
    return TBDK_OK;
}

int tbdk_farneback_levels(int width, int height, const tbdk_farneback_params* p, int* nlevels, int32_t* sizes)
{
    if (fb_check(p) != TBDK_OK || width <= 0 || height <= 0 || !nlevels) return TBDK_EINVAL;
    // FarnebackOpticalFlowImpl::calc level count (optflowgf.cpp:1125-1132)
    const int min_size = 32;
    int k;
    double scale = 1;
    for (k = 0; k < p->num_levels; k++) {
        scale *= p->pyr_scale;
        if (width * scale < min_size || height * scale < min_size) break;
    }
    *nlevels = k + 1;
    if (sizes) {
        for (int l = 0; l <= k; ++l) {
            double sc = 1;
            for (int i = 0; i < l; i++) sc *= p->pyr_scale;
            sizes[2 * l] = cv_round(width * sc);
            sizes[2 * l + 1] = cv_round(height * sc);
        }
    }
    return TBDK_OK;
}

int tbdk_farneback(tbdk_ctx* ctx, const uint8_t* prev, const uint8_t* next, int width, int height, int pitch,
                   float* flow, int flow_pitch, const tbdk_farneback_params* p, void* stream)
{
    if (!ctx || !prev || !next || !flow || width <= 0 || height <= 0 || pitch < width) return TBDK_EINVAL;
    if (flow_pitch < 8 * width || flow_pitch % 8 != 0) return TBDK_EINVAL;
    int rc = fb_check(p);
    if (rc != TBDK_OK) return rc;
    int nl = 0;
    int32_t sizes[2 * 64];
    if (p->num_levels > 63) return TBDK_EINVAL;
    tbdk_farneback_levels(width, height, p, &nl, sizes);
    const int levels = nl - 1;
    // per-level smoothing (optflowgf.cpp:1136-1144) and scratch sizes
    FbLevel lv[64];
    int64_t tcap = 0;
    LevelImagePlan plan;
    for (int k = 0; k <= levels; ++k) {
        double scale = 1;
        for (int i = 0; i < k; i++) scale *= p->pyr_scale;
        const double sigma = (1. / scale - 1) * 0.5;
        int smooth_sz = cv_round(sigma * 5) | 1;
        smooth_sz = smooth_sz < 3 ? 3 : smooth_sz;
        lv[k] = FbLevel{sizes[2 * k], sizes[2 * k + 1], smooth_sz, sigma};
        if (lv[k].w <= 0 || lv[k].h <= 0) return TBDK_EINVAL;
        rc = plan_level_image(width, height, lv[k].w, lv[k].h, smooth_sz, sigma, &plan);
        if (rc != TBDK_OK) return rc;
        const int64_t t = (int64_t)height * plane_pitch(plan.nc);
        tcap = t > tcap ? t : tcap;
    }
    const int64_t px = plane_stride(plane_pitch(width), height);
    DeviceGuard g(ctx->device);
    rc = fb_reserve(ctx, px, tcap);
    if (rc != TBDK_OK) return rc;
    FbScratch* f = ctx->fb;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // every buffer of the scratch (R0 / R1 / Rl, T, I, the flow ping-pong) is
    // still in use by the previous call until its stream reaches `done`
    if (f->done && f->last_stream != s) {
        const hipError_t w = hipStreamWaitEvent(s, f->done, 0);
        if (w != hipSuccess) return map_status(w);
    }
    const bool gauss = (p->flags & TBDK_OPTFLOW_FARNEBACK_GAUSSIAN) != 0;
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0)
        cus = 256;
    const int m = p->win_size / 2;
    const int round_wgs = cus * fb_iter_occupancy(m, gauss);  // one round of resident fb_iter workgroups
    const int iter_wgs = round_wgs * ((3 * cus + round_wgs - 1) / round_wgs);
    hipError_t e = hipSuccess;
    // level images and polynomial expansion of both frames (the flow does not
    // enter them): with prep-ahead every level's R0 / R1 is its own region,
    // computed on the prep stream coarse to fine while the coarser levels iterate
    const bool ahead = ctx->opt_fb_prep_ahead && levels > 0;
    int64_t roff[64];
    int64_t rtot = 0;
    for (int k = 0; k <= levels; ++k) {
        roff[k] = rtot;
        rtot += 10 * plane_stride(plane_pitch(lv[k].w), lv[k].h);
    }
    if (ahead) {
        if ((rc = fb_reserve_ahead(f, rtot, levels + 1)) != TBDK_OK) return rc;
        e = hipEventRecord(f->fork, s);  // the previous call's readers of Rl, T, I are done (any stream: see done)
        if (e == hipSuccess) e = hipStreamWaitEvent(f->prep, f->fork, 0);
    }
    auto prep_level = [&](int k, hipStream_t ps, float* R0, float* R1) {
        const int w = lv[k].w, h = lv[k].h, pp = plane_pitch(w);
        const int64_t plane = plane_stride(pp, h);
        LevelImagePlan pl;
        plan_level_image(width, height, w, h, lv[k].ks, lv[k].sigma, &pl);
        const int tpitch = plane_pitch(pl.nc);
        hipError_t r = hipSuccess;
        for (int i = 0; i < 2 && r == hipSuccess; ++i) {
            int rec = timing_begin(ctx, "fb_pyr", ps);
            r = launch_level_image(pl, i ? next : prev, width, height, pitch, f->T, tpitch, f->I, w, h, pp, ps);
            timing_end(ctx, rec, ps);
            if (r != hipSuccess) break;
            rec = timing_begin(ctx, "fb_polyexp", ps);
            r = launch_polyexp(f->I, w, h, pp, i ? R1 : R0, pp, plane, p->poly_n, p->poly_sigma, ps);
            timing_end(ctx, rec, ps);
        }
        return r;
    };
    for (int k = levels; ahead && k >= 0 && e == hipSuccess; --k) {
        const int64_t plane = plane_stride(plane_pitch(lv[k].w), lv[k].h);
        e = prep_level(k, f->prep, f->Rl + roff[k], f->Rl + roff[k] + 5 * plane);
        if (e == hipSuccess) e = hipEventRecord(f->lev_ev[k], f->prep);
    }
    int cur = 0;  // ping-pong index of the current flow
    int pw = 0, ph = 0, ppitch = 0;
    for (int k = levels; k >= 0 && e == hipSuccess; --k) {
        const int w = lv[k].w, h = lv[k].h, pp = plane_pitch(w);
        const int64_t plane = plane_stride(pp, h);
        float* R0 = ahead ? f->Rl + roff[k] : f->R0;
        float* R1 = ahead ? R0 + 5 * plane : f->R1;
        e = ahead ? hipStreamWaitEvent(s, f->lev_ev[k], 0) : prep_level(k, s, R0, R1);
        if (e != hipSuccess) break;
        // initial flow of the level
        int rec = timing_begin(ctx, "fb_flow_init", s);
        if (k == levels && (p->flags & TBDK_OPTFLOW_USE_INITIAL_FLOW)) {
            double scale = 1;
            for (int i = 0; i < k; i++) scale *= p->pyr_scale;
            FbFlowAreaArgs u;
            u.src = flow;
            u.sw = width;
            u.sh = height;
            u.spitch = flow_pitch / 4;
            u.dst = f->F[cur];
            u.w = w;
            u.h = h;
            u.dpitch = pp;
            u.dplane = plane;
            u.scale_x = 1. / ((double)w / width);
            u.scale_y = 1. / ((double)h / height);
            u.isx = cv_round(u.scale_x);
            u.isy = cv_round(u.scale_y);
            u.mode = (w == width && h == height) ? kAreaCopy
                     : (std::fabs(u.scale_x - u.isx) < DBL_EPSILON && std::fabs(u.scale_y - u.isy) < DBL_EPSILON)
                         ? kAreaFast
                         : kAreaTable;
            u.alpha = (float)scale;
            u.apply_alpha = !(std::fabs(scale - 1) < DBL_EPSILON);
            hipLaunchKernelGGL(fb_flow_area_kernel, dim3((w + 255) / 256, h), dim3(256), 0, s, u);
            e = hipGetLastError();
        } else if (k == levels) {
            e = hipMemsetAsync(f->F[cur], 0, sizeof(float) * (size_t)plane * 2, s);
        } else {
            FbFlowUpArgs u;
            u.src = f->F[cur];
            u.sw = pw;
            u.sh = ph;
            u.spitch = ppitch;
            u.splane = plane_stride(ppitch, ph);
            u.dst = f->F[cur ^ 1];
            u.w = w;
            u.h = h;
            u.dpitch = pp;
            u.dplane = plane;
            u.scale_x = 1. / ((double)w / pw);
            u.scale_y = 1. / ((double)h / ph);
            u.alpha = (float)(1. / p->pyr_scale);
            hipLaunchKernelGGL(fb_flow_up_kernel, dim3((w + 255) / 256, h), dim3(256), 0, s, u);
            e = hipGetLastError();
            cur ^= 1;
        }
        timing_end(ctx, rec, s);
        if (e != hipSuccess) break;
        // iterations
        FbIterArgs a;
        a.R0 = R0;
        a.R1 = R1;
        a.w = w;
        a.h = h;
        a.pitch = pp;
        a.fplane = plane;
        a.rplane = plane;
        a.seg = iter_seg(w, h, m, iter_wgs);
        a.scale = 1. / (p->win_size * p->win_size);
        // FarnebackUpdateFlow_GaussianBlur kernel (optflowgf.cpp:416-435)
        {
            double sg = m * 0.3, sum = 1;
            a.gk[0] = (float)sum;
            for (int i = 1; i <= m; i++) {
                const float t = (float)std::exp(-i * i / (2 * sg * sg));
                a.gk[i] = t;
                sum += t * 2;
            }
            sum = 1. / sum;
            for (int i = 0; i <= m; i++) a.gk[i] = (float)(a.gk[i] * sum);
        }
        for (int it = 0; it < p->num_iters && e == hipSuccess; ++it) {
            const bool last = k == 0 && it == p->num_iters - 1;
            a.fin = f->F[cur];
            a.fout = last ? flow : f->F[cur ^ 1];
            a.out_il = last;
            a.out_pitch = flow_pitch / 4;
            rec = timing_begin(ctx, "fb_iter", s);
            e = launch_fb_iter(a, m, gauss, s);
            timing_end(ctx, rec, s);
            if (!last) cur ^= 1;
        }
        if (e == hipSuccess && k == 0 && p->num_iters == 0) {
            hipLaunchKernelGGL(fb_interleave_kernel, dim3((w + 255) / 256, h), dim3(256), 0, s, f->F[cur], w, h, pp,
                               plane, flow, flow_pitch / 4);
            e = hipGetLastError();
        }
        pw = w;
        ph = h;
        ppitch = pp;
    }
    // the call's completion on s (its prep-stream work is joined into s by the
    // level events before the last iterations)
    if (e == hipSuccess && !f->done) e = hipEventCreateWithFlags(&f->done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(f->done, s);
    f->last_stream = s;
    return map_status(e);
}

int tbdk_fb_level_image(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, int dst_width,
                        int dst_height, int smooth_size, double sigma, float* dst, int dst_pitch, void* stream)
{
    if (!ctx || !img || !dst || width <= 0 || height <= 0 || pitch < width || dst_width <= 0 || dst_height <= 0 ||
        dst_pitch < 4 * dst_width || dst_pitch % 4 != 0)
        return TBDK_EINVAL;
    LevelImagePlan plan;
    int rc = plan_level_image(width, height, dst_width, dst_height, smooth_size, sigma, &plan);
    if (rc != TBDK_OK) return rc;
    const int tpitch = plane_pitch(plan.nc);
    DeviceGuard g(ctx->device);
    rc = fb_reserve(ctx, ctx->fb ? ctx->fb->cap_px : 0, (int64_t)height * tpitch);
    if (rc != TBDK_OK) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    FbScratch* f = ctx->fb;  // T: ordered after the last tbdk_farneback call, as that call orders itself
    if (f->done && f->last_stream != s) {
        const hipError_t w = hipStreamWaitEvent(s, f->done, 0);
        if (w != hipSuccess) return map_status(w);
    }
    return map_status(launch_level_image(plan, img, width, height, pitch, f->T, tpitch, dst, dst_width,
                                         dst_height, dst_pitch / 4, s));
}

int tbdk_fb_poly_exp(tbdk_ctx* ctx, const float* src, int width, int height, int src_pitch, int poly_n,
                     double poly_sigma, float* dst, int dst_pitch, void* stream)
{
    if (!ctx || !src || !dst || width <= 0 || height <= 0 || src_pitch < 4 * width || src_pitch % 4 != 0 ||
        dst_pitch < 4 * width || dst_pitch % 4 != 0 || poly_n < 1 || poly_n > kFbMaxPolyN)
        return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    return map_status(launch_polyexp(src, width, height, src_pitch / 4, dst, dst_pitch / 4,
                                     (int64_t)(dst_pitch / 4) * height, poly_n, poly_sigma, s));
}

}  // extern "C"
