// klt_pyr.hip — image-pyramid kernels for gfx950.
//
// Semantics: cv::buildOpticalFlowPyramid (video/src/lkpyramid.cpp:697-793) with
// pyrDown_<FixPtCast<uchar,8>> (imgproc/src/pyramids.cpp:722-857): integer 5x5
// [1 4 6 4 1]^2, (s + 128) >> 8, BORDER_REFLECT_101 on the isolated source
// level, every level stored with a reflect-101 frame of `pad` pixels.
// The border of each level is produced by the same kernel that produces its
// interior (a border pixel is the pyrDown value at its reflected coordinate),
// so one launch writes one complete padded level.
#include "tbdk_internal.hpp"

namespace tbdk {

__device__ __forceinline__ int reflect101(int p, int len)
{
    // cv::borderInterpolate(BORDER_REFLECT_101), looped for tiny levels
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// Level 0: copy the frame into the padded buffer (copyMakeBorder REFLECT_101,
// lkpyramid.cpp:738).  One thread writes 4 consecutive bytes of a padded row.
__global__ void pad_copy_kernel(const uint8_t* __restrict__ src, int spitch, int w, int h,
                                uint8_t* __restrict__ dst, int dpitch, int pad, int wp4)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y;
    if (t >= wp4) return;
    const int sy = reflect101(py - pad, h);
    const uint8_t* srow = src + (size_t)sy * spitch;
    const int x0 = t * 4 - pad;
    uint32_t v;
    if (x0 >= 0 && x0 + 3 < w) {
        v = (uint32_t)srow[x0] | ((uint32_t)srow[x0 + 1] << 8) | ((uint32_t)srow[x0 + 2] << 16) |
            ((uint32_t)srow[x0 + 3] << 24);
    } else {
        v = 0;
        for (int k = 0; k < 4; ++k) v |= (uint32_t)srow[reflect101(x0 + k, w)] << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(dst + (size_t)py * dpitch + t * 4) = v;
}

// pyrDown of a padded level into a padded level.  Reads of the source at
// 2x-2 .. 2x+2 stay inside the source's reflect-101 frame (pad >= 2), which
// equals borderInterpolate on the isolated source (pyramids.cpp:795-800).
__global__ void pyr_down_padded_kernel(const uint8_t* __restrict__ src, int spitch, int spad,
                                       uint8_t* __restrict__ dst, int dpitch, int dpad, int dw, int dh,
                                       int wp4)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y;
    if (t >= wp4) return;
    const int ry = reflect101(py - dpad, dh);
    const uint8_t* s0 = src + (size_t)(2 * ry - 2 + spad) * spitch + spad;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int rx = reflect101(t * 4 + k - dpad, dw);
        const uint8_t* s = s0 + 2 * rx;
        int r[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint8_t* q = s + (size_t)j * spitch;
            r[j] = q[0] * 6 + (q[-1] + q[1]) * 4 + q[-2] + q[2];
        }
        const int sum = r[2] * 6 + (r[1] + r[3]) * 4 + r[0] + r[4];
        v |= (uint32_t)((sum + 128) >> 8) << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(dst + (size_t)py * dpitch + t * 4) = v;
}

// Plain (unpadded) single-level pyrDown: cv::cuda::pyrDown replacement.
__global__ void pyr_down_plain_kernel(const uint8_t* __restrict__ src, int sw, int sh, int spitch,
                                      uint8_t* __restrict__ dst, int dpitch, int dw)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= dw) return;
    int cx[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) cx[i] = reflect101(2 * x + i - 2, sw);
    int r[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const uint8_t* q = src + (size_t)reflect101(2 * y + j - 2, sh) * spitch;
        r[j] = q[cx[2]] * 6 + (q[cx[1]] + q[cx[3]]) * 4 + q[cx[0]] + q[cx[4]];
    }
    const int sum = r[2] * 6 + (r[1] + r[3]) * 4 + r[0] + r[4];
    dst[(size_t)y * dpitch + x] = (uint8_t)((sum + 128) >> 8);
}

// calcSharrDeriv (lkpyramid.cpp:55-144) of every level into its int16x2 plane.
// Rows/columns outside the level come from the level's reflect-101 frame, which
// is exactly the reference's row (:78-80) and column (:111-116) reflection.
struct ScharrLevels {
    const uint8_t* src[TBDK_MAX_LEVELS];
    uint8_t* dst[TBDK_MAX_LEVELS];
    int w[TBDK_MAX_LEVELS], h[TBDK_MAX_LEVELS], spitch[TBDK_MAX_LEVELS], spad[TBDK_MAX_LEVELS];
    int dpitch[TBDK_MAX_LEVELS], dpad[TBDK_MAX_LEVELS];
};

__global__ void scharr_levels_kernel(ScharrLevels a)
{
    const int lvl = blockIdx.z;
    const int y = blockIdx.y;
    const int x0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int w = a.w[lvl], h = a.h[lvl];
    if (y >= h || x0 >= w) return;
    const int sp = a.spitch[lvl];
    const uint8_t* r1 = a.src[lvl] + (size_t)(y + a.spad[lvl]) * sp + a.spad[lvl] + x0;
    const uint8_t* r0 = r1 - sp;
    const uint8_t* r2 = r1 + sp;
    int t0[6], t1[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int c = k - 1;
        t0[k] = (r0[c] + r2[c]) * 3 + r1[c] * 10;
        t1[k] = r2[c] - r0[c];
    }
    int32_t out[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int ix = t0[k + 2] - t0[k];
        const int iy = (t1[k + 2] + t1[k]) * 3 + t1[k + 1] * 10;
        out[k] = (int32_t)(((uint32_t)ix & 0xffffu) | ((uint32_t)iy << 16));
    }
    int32_t* d = reinterpret_cast<int32_t*>(a.dst[lvl] + (size_t)(y + a.dpad[lvl]) * a.dpitch[lvl]) + a.dpad[lvl] + x0;
    const int n = w - x0 < 4 ? w - x0 : 4;
    for (int k = 0; k < n; ++k) d[k] = out[k];
}

// ---- fused build: the padded copy of a source level and the next one or two
// levels below it in ONE launch (no level is re-read from HBM, one launch
// instead of three).  A workgroup owns a band of R rows x TW columns of the
// deepest level; it stages the source region those need (with halo) in LDS,
// computes the intermediate level's region (with its own halo) in LDS, then
// the deepest level, and writes its part of every level plus that part's
// reflect-101 mirrors in the padding.  LDS regions are indexed by VIRTUAL
// coordinates (possibly outside the level): an entry holds the value at the
// reflect-101 image of its coordinate, which is what pyrDown_'s
// borderInterpolate reads there (pyramids.cpp:795-800), so interior and edge
// workgroups run the same code.  Every level must be at least pad + 1 pixels
// in each direction (one reflection reaches the whole padding); the host falls
// back to the per-level kernels otherwise.
constexpr int kFuseThreads = 256;
constexpr int kFuseBand = 2;     // rows of the deepest level per workgroup
constexpr int kFuseTile = 128;   // columns of the deepest level per workgroup

struct PyrFuseArgs {
    const uint8_t* src;  // source level, in-image origin
    int spitch, sw, sh;
    uint8_t* copy;       // padded copy of the source (level 0 of a pyramid) or null
    int cpitch, cpad;
    uint8_t* d[2];       // padded buffers of the levels below (d[1] unused with one level)
    int dpitch[2], dpad[2], dw[2], dh[2];
    int ntx;             // column tiles of the deepest level
};

// LDS tile shapes of a workgroup, levels fused below the source: NL = 1 or 2.
// Level d[0]'s tile starts at virtual column X1 = 2 * cx0 - 4 (NL 2; its
// deepest-level taps reach 2 * cx0 - 2 .. 2 * cx0 + 2 * TW) or cx0 (NL 1); the
// source tile at 2 * X1 - 4.  Every tile's row length and column origin are
// multiples of 4, so LDS rows are read and written as dwords.
template <int NL>
struct FuseShape {
    static constexpr int R = kFuseBand, TW = kFuseTile;
    static constexpr int L1R = NL == 2 ? 2 * R + 3 : R;      // level d[0] tile rows
    static constexpr int L1C = NL == 2 ? 2 * TW + 8 : TW;     // ... columns
    static constexpr int SR = 2 * L1R + 3;                    // source tile rows
    static constexpr int SC = 2 * L1C + 8;                    // ... columns
    static constexpr int oS = 0;                                           // u8 [SR][SC]
    static constexpr int oV = (oS + SR * SC + 15) & ~15;                   // int16 [L1R][SC]
    static constexpr int oT1 = (oV + 2 * L1R * SC + 15) & ~15;             // u8 [L1R][L1C]
    static constexpr int oV2 = (oT1 + L1R * L1C + 15) & ~15;               // int16 [R][L1C]
    static constexpr int oT2 = (oV2 + 2 * R * L1C + 15) & ~15;             // u8 [R][TW]
    static constexpr int bytes = NL == 2 ? oT2 + R * TW : oV2;
};

__device__ __forceinline__ int pyr5(int a, int b, int c, int d, int e) { return c * 6 + (b + d) * 4 + a + e; }

// value v of in-image pixel (y, x) of a padded level (w, h >= pad + 1) into
// every position of the padded buffer that reflects to it: itself, its mirror
// across the first row / column (1 <= y <= pad) and across the last
// (h-1-pad <= y <= h-2)
__device__ __forceinline__ void put_mirrors(uint8_t* buf, int pitch, int pad, int w, int h, int y, int x, uint8_t v)
{
    int ry[3], rx[3], ny = 0, nx = 0;
    ry[ny++] = y;
    if (y >= 1 && y <= pad) ry[ny++] = -y;
    if (y >= h - 1 - pad && y <= h - 2) ry[ny++] = 2 * (h - 1) - y;
    rx[nx++] = x;
    if (x >= 1 && x <= pad) rx[nx++] = -x;
    if (x >= w - 1 - pad && x <= w - 2) rx[nx++] = 2 * (w - 1) - x;
    for (int i = 0; i < ny; ++i)
        for (int j = 0; j < nx; ++j) buf[(size_t)(ry[i] + pad) * pitch + rx[j] + pad] = v;
}

// in-image rows [y0, y0 + NR) x cols [x0, x0 + 4 * G4) of a level (clipped to
// the level) from an LDS tile whose (row 0, col tc0) is pixel (y0, x0): dword
// LDS reads and dword stores; the mirror copies of pixels near a column edge
// byte by byte, of rows near a row edge as dwords
template <int NR, int G4, int TCOLS>
__device__ __forceinline__ void write_level_region(uint8_t* buf, int pitch, int pad, int w, int h, int y0, int x0,
                                                   const uint8_t* tile, int tc0, int tid)
{
    for (int i = tid; i < NR * G4; i += kFuseThreads) {
        const int r = i / G4, y = y0 + r, x = x0 + 4 * (i - r * G4);
        if (y >= h || x >= w) continue;
        const uint32_t v = *reinterpret_cast<const uint32_t*>(tile + r * TCOLS + tc0 + 4 * (i - r * G4));
        const bool edge_x = x <= pad || x + 3 >= w - 1 - pad;
        if (!edge_x) {  // x0 is a multiple of 4 and pitch / pad keep rows dword-aligned
            *reinterpret_cast<uint32_t*>(buf + (size_t)(y + pad) * pitch + x + pad) = v;
            if (y >= 1 && y <= pad) *reinterpret_cast<uint32_t*>(buf + (size_t)(pad - y) * pitch + x + pad) = v;
            if (y >= h - 1 - pad && y <= h - 2)
                *reinterpret_cast<uint32_t*>(buf + (size_t)(2 * (h - 1) - y + pad) * pitch + x + pad) = v;
        } else {
            for (int k = 0; k < 4 && x + k < w; ++k) put_mirrors(buf, pitch, pad, w, h, y, x + k, (uint8_t)(v >> (8 * k)));
        }
    }
}

// vertical 5-tap sums of an u8 LDS tile [*][COLS], four columns per item: out
// row r (level row v = vo + r, reflected into [0, lh)) = taps over tile rows
// 2 * reflect(v) - 2 - vt .. + 4; rows outside [lo, hi] are never read and not
// computed
template <int ROWS, int COLS>
__device__ __forceinline__ void vpass(const uint8_t* in, int vt, int16_t* out, int vo, int lh, int lo, int hi, int tid)
{
    constexpr int C4 = COLS / 4;
    for (int i = tid; i < ROWS * C4; i += kFuseThreads) {
        const int r = i / C4, c = 4 * (i - r * C4);
        if (vo + r < lo || vo + r > hi) continue;
        const uint8_t* p = in + (2 * reflect101(vo + r, lh) - 2 - vt) * COLS + c;
        uint32_t q[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) q[k] = *reinterpret_cast<const uint32_t*>(p + k * COLS);
        int s[4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
            s[b] = pyr5((q[0] >> (8 * b)) & 255, (q[1] >> (8 * b)) & 255, (q[2] >> (8 * b)) & 255,
                        (q[3] >> (8 * b)) & 255, (q[4] >> (8 * b)) & 255);
        uint32_t* o = reinterpret_cast<uint32_t*>(out + r * COLS + c);
        o[0] = (uint32_t)(s[0] & 0xFFFF) | ((uint32_t)s[1] << 16);
        o[1] = (uint32_t)(s[2] & 0xFFFF) | ((uint32_t)s[3] << 16);
    }
}

// horizontal 5-tap pass + rounding, two output columns per item: out(r, c) for
// level col v = vo + c (reflected into [0, lw)) from vertical sums [*][ICOLS]
// whose column 0 is virtual col vt; columns outside [lo, hi] and rows outside
// [rlo, rhi] are never read and not computed
template <int ROWS, int OCOLS, int ICOLS>
__device__ __forceinline__ void hpass(const int16_t* in, int vt, uint8_t* out, int vo, int lw, int lo, int hi, int rlo,
                                      int rhi, int tid)
{
    constexpr int C2 = OCOLS / 2;
    for (int i = tid; i < ROWS * C2; i += kFuseThreads) {
        const int r = i / C2, c = 2 * (i - r * C2);
        if (r < rlo || r > rhi) continue;
        const int v0 = vo + c, v1 = v0 + 1;
        const bool ok0 = v0 >= lo && v0 <= hi, ok1 = v1 >= lo && v1 <= hi;
        if (!ok0 && !ok1) continue;
        const int r0 = reflect101(v0, lw), r1 = reflect101(v1, lw);
        const int16_t* row = in + r * ICOLS;
        int o0, o1;
        if (r1 == r0 + 1) {  // no reflection between them: one run of 7 sums (even start, dword-aligned)
            const int16_t* p = row + 2 * r0 - 2 - vt;
            const uint32_t* pw = reinterpret_cast<const uint32_t*>(p);
            const uint32_t w0 = pw[0], w1 = pw[1], w2 = pw[2], w3 = pw[3];
            const int t0 = (int16_t)w0, t1 = (int16_t)(w0 >> 16), t2 = (int16_t)w1, t3 = (int16_t)(w1 >> 16);
            const int t4 = (int16_t)w2, t5 = (int16_t)(w2 >> 16), t6 = (int16_t)w3;
            o0 = (pyr5(t0, t1, t2, t3, t4) + 128) >> 8;
            o1 = (pyr5(t2, t3, t4, t5, t6) + 128) >> 8;
        } else {
            const int16_t* p0 = row + 2 * r0 - 2 - vt;
            const int16_t* p1 = row + 2 * r1 - 2 - vt;
            o0 = ok0 ? (pyr5(p0[0], p0[1], p0[2], p0[3], p0[4]) + 128) >> 8 : 0;
            o1 = ok1 ? (pyr5(p1[0], p1[1], p1[2], p1[3], p1[4]) + 128) >> 8 : 0;
        }
        *reinterpret_cast<uint16_t*>(out + r * OCOLS + c) = (uint16_t)(o0 | (o1 << 8));
    }
}

template <int NL>
__global__ __launch_bounds__(kFuseThreads) void pyr_build_kernel(PyrFuseArgs a)
{
    using F = FuseShape<NL>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* S = smem + F::oS;
    int16_t* V = reinterpret_cast<int16_t*>(smem + F::oV);
    uint8_t* T1 = smem + F::oT1;
    const int tid = threadIdx.x;
    const int b = xcd_swizzle(blockIdx.x, gridDim.x);  // neighbouring bands on one XCD share its L2
    const int by = b / a.ntx, bx = b - by * a.ntx;
    // deepest level: rows [ry0, ry0 + R), cols [cx0, cx0 + TW); virtual tile origins above it
    const int ry0 = by * F::R, cx0 = bx * F::TW;
    const int l1y0 = NL == 2 ? 2 * ry0 - 2 : ry0, l1x0 = NL == 2 ? 2 * cx0 - 4 : cx0;
    const int sy0 = 2 * l1y0 - 2, sx0 = 2 * l1x0 - 4;
    // ---- stage the source region (reflect-101 at the source's edges)
    const bool vec = ((reinterpret_cast<uintptr_t>(a.src) | (uintptr_t)a.spitch) & 3) == 0;
    // every load of the thread is issued before the first LDS store (a
    // load-store loop waits out one memory round trip per item)
    constexpr int SC4 = F::SC / 4;
    constexpr int NIT = (F::SR * SC4 + kFuseThreads - 1) / kFuseThreads;
    uint32_t sv[NIT];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
        const int i = tid + k * kFuseThreads;
        if (i >= F::SR * SC4) break;
        const int r = i / SC4, c = 4 * (i - r * SC4);
        const uint8_t* row = a.src + (size_t)reflect101(sy0 + r, a.sh) * a.spitch;
        const int vx = sx0 + c;
        if (vec && vx >= 0 && vx + 3 < a.sw) {
            sv[k] = *reinterpret_cast<const uint32_t*>(row + vx);
        } else {
            uint32_t v = 0;
            for (int q = 0; q < 4; ++q) v |= (uint32_t)row[reflect101(vx + q, a.sw)] << (8 * q);
            sv[k] = v;
        }
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
        const int i = tid + k * kFuseThreads;
        if (i >= F::SR * SC4) break;
        const int r = i / SC4, c = 4 * (i - r * SC4);
        *reinterpret_cast<uint32_t*>(S + r * F::SC + c) = sv[k];
    }
    __syncthreads();
#if defined(TBDK_PYR_PROBE) && TBDK_PYR_PROBE == 1
    if (S[tid] == 7 && tid == 1000) a.copy[0] = 1;
    return;
#endif
    // ---- level d[0]'s tile.  Entries that are read: with a deeper level,
    // virtual rows / cols [-2, 2 * (deepest size - 1) + 2] (its in-image taps);
    // without, the in-image ones (they are written out)
    const int ylo = NL == 2 ? -2 : 0, xlo = ylo;
    const int yhi = NL == 2 ? 2 * a.dh[1] : a.dh[0] - 1, xhi = NL == 2 ? 2 * a.dw[1] : a.dw[0] - 1;
    vpass<F::L1R, F::SC>(S, sy0, V, l1y0, a.dh[0], ylo, yhi, tid);
    __syncthreads();
    hpass<F::L1R, F::L1C, F::SC>(V, sx0, T1, l1x0, a.dw[0], xlo, xhi, ylo - l1y0, yhi - l1y0, tid);
    __syncthreads();
#if defined(TBDK_PYR_PROBE) && TBDK_PYR_PROBE == 2
    if (T1[tid] == 7 && tid == 1000) a.copy[0] = 1;
    return;
#endif
    // ---- writes: the source copy, level d[0]; then the deepest level
    constexpr int f = NL == 2 ? 4 : 2;  // source rows / cols per deepest-level row / col
    if (a.copy)
        write_level_region<f * F::R, f * F::TW / 4, F::SC>(a.copy, a.cpitch, a.cpad, a.sw, a.sh, f * ry0, f * cx0,
                                                          S + (f * ry0 - sy0) * F::SC, f * cx0 - sx0, tid);
    constexpr int f1 = NL == 2 ? 2 : 1;
    write_level_region<f1 * F::R, f1 * F::TW / 4, F::L1C>(a.d[0], a.dpitch[0], a.dpad[0], a.dw[0], a.dh[0], f1 * ry0,
                                                         f1 * cx0, T1 + (f1 * ry0 - l1y0) * F::L1C, f1 * cx0 - l1x0,
                                                         tid);
    if constexpr (NL == 2) {
        int16_t* V2 = reinterpret_cast<int16_t*>(smem + F::oV2);
        uint8_t* T2 = smem + F::oT2;
        const int hD = a.dh[1], wD = a.dw[1];
        vpass<F::R, F::L1C>(T1, l1y0, V2, ry0, hD, 0, hD - 1, tid);
        __syncthreads();
        hpass<F::R, F::TW, F::L1C>(V2, l1x0, T2, cx0, wD, 0, wD - 1, 0, hD - 1 - ry0, tid);
        __syncthreads();
        write_level_region<F::R, F::TW / 4, F::TW>(a.d[1], a.dpitch[1], a.dpad[1], wD, hD, ry0, cx0, T2, 0, tid);
    }
}

// levels [first, first + nl] of pyr: from the in-image source (first == 0: the
// frame, whose padded copy is level 0) to nl (1 or 2) levels below it
static hipError_t launch_pyr_fuse(const uint8_t* src, int spitch, const tbdk_pyr& pyr, int first, int nl,
                                  bool copy, hipStream_t s)
{
    PyrFuseArgs a;
    const tbdk_level& S = pyr.lv[first];
    a.src = src;
    a.spitch = spitch;
    a.sw = S.width;
    a.sh = S.height;
    a.copy = copy ? S.data : nullptr;
    a.cpitch = S.pitch;
    a.cpad = S.pad;
    for (int k = 0; k < 2; ++k) {
        const tbdk_level& D = pyr.lv[first + 1 + (k < nl ? k : 0)];
        a.d[k] = D.data;
        a.dpitch[k] = D.pitch;
        a.dpad[k] = D.pad;
        a.dw[k] = D.width;
        a.dh[k] = D.height;
    }
    const tbdk_level& Dd = pyr.lv[first + nl];
    a.ntx = (Dd.width + kFuseTile - 1) / kFuseTile;
    const int nty = (Dd.height + kFuseBand - 1) / kFuseBand;
    const dim3 grid(a.ntx * nty), block(kFuseThreads);
    if (nl == 2) hipLaunchKernelGGL(pyr_build_kernel<2>, grid, block, FuseShape<2>::bytes, s, a);
    else hipLaunchKernelGGL(pyr_build_kernel<1>, grid, block, FuseShape<1>::bytes, s, a);
    return hipGetLastError();
}

// every level of a u8 pyramid from the frame: fused launches where the levels
// allow it (>= pad + 1 pixels each way), the per-level kernels otherwise
hipError_t launch_pyr_levels(const uint8_t* img, int pitch, const tbdk_pyr& pyr, bool fuse, hipStream_t s)
{
    auto fusable = [&](int l) {
        return fuse && pyr.lv[l].width > pyr.lv[l].pad && pyr.lv[l].height > pyr.lv[l].pad;
    };
    int done = 0;  // levels [0, done] built
    hipError_t e = hipSuccess;
    if (pyr.nlevels == 1 || !fusable(0) || !fusable(1)) {
        e = launch_pad_copy(img, pitch, pyr.lv[0], s);
    } else {
        const int nl = pyr.nlevels >= 3 && fusable(2) ? 2 : 1;
        e = launch_pyr_fuse(img, pitch, pyr, 0, nl, true, s);
        done = nl;
    }
    while (e == hipSuccess && done + 1 < pyr.nlevels) {
        if (fusable(done + 1)) {
            const int nl = done + 2 < pyr.nlevels && fusable(done + 2) ? 2 : 1;
            const tbdk_level& S = pyr.lv[done];
            e = launch_pyr_fuse(S.data + (size_t)S.pad * S.pitch + S.pad, S.pitch, pyr, done, nl, false, s);
            done += nl;
        } else {
            e = launch_pyr_down_padded(pyr.lv[done], pyr.lv[done + 1], s);
            done += 1;
        }
    }
    return e;
}

hipError_t launch_scharr_levels(const tbdk_pyr& pyr, hipStream_t s)
{
    ScharrLevels a;
    int maxw = 0, maxh = 0;
    for (int l = 0; l < pyr.nlevels; ++l) {
        a.src[l] = pyr.lv[l].data;
        a.dst[l] = pyr.dv[l].data;
        a.w[l] = pyr.lv[l].width;
        a.h[l] = pyr.lv[l].height;
        a.spitch[l] = pyr.lv[l].pitch;
        a.spad[l] = pyr.lv[l].pad;
        a.dpitch[l] = pyr.dv[l].pitch;
        a.dpad[l] = pyr.dv[l].pad;
        maxw = a.w[l] > maxw ? a.w[l] : maxw;
        maxh = a.h[l] > maxh ? a.h[l] : maxh;
    }
    dim3 block(256), grid(((maxw + 3) / 4 + 255) / 256, maxh, pyr.nlevels);
    hipLaunchKernelGGL(scharr_levels_kernel, grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_pad_copy(const uint8_t* src, int spitch, const tbdk_level& d, hipStream_t s)
{
    const int wp = d.width + 2 * d.pad, hp = d.height + 2 * d.pad;
    const int wp4 = (wp + 3) / 4;
    dim3 block(256), grid((wp4 + 255) / 256, hp);
    hipLaunchKernelGGL(pad_copy_kernel, grid, block, 0, s, src, spitch, d.width, d.height, d.data, d.pitch,
                       d.pad, wp4);
    return hipGetLastError();
}

hipError_t launch_pyr_down_padded(const tbdk_level& sl, const tbdk_level& dl, hipStream_t s)
{
    const int wp = dl.width + 2 * dl.pad, hp = dl.height + 2 * dl.pad;
    const int wp4 = (wp + 3) / 4;
    dim3 block(256), grid((wp4 + 255) / 256, hp);
    hipLaunchKernelGGL(pyr_down_padded_kernel, grid, block, 0, s, sl.data, sl.pitch, sl.pad, dl.data, dl.pitch,
                       dl.pad, dl.width, dl.height, wp4);
    return hipGetLastError();
}

hipError_t launch_pyr_down_plain(const uint8_t* src, int w, int h, int spitch, uint8_t* dst, int dpitch,
                                 hipStream_t s)
{
    const int dw = (w + 1) / 2, dh = (h + 1) / 2;
    dim3 block(256), grid((dw + 255) / 256, dh);
    hipLaunchKernelGGL(pyr_down_plain_kernel, grid, block, 0, s, src, w, h, spitch, dst, dpitch, dw);
    return hipGetLastError();
}

}  // namespace tbdk
