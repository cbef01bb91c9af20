// klt_lk_strip.hip — sparse pyramidal LK, register-strip variant for gfx950.
//
// Same algorithm and bit-identical results as klt_lk.hip (CPU calcOpticalFlowPyrLK
// numerics, LKTrackerInvoker video/src/lkpyramid.cpp:178-695, exact integer
// sums), organised for the CDNA4 wave instead of the reference's 16x16 block:
//   * one wave64 per point, 4 points per 256-thread workgroup, all levels in
//     one launch;
//   * lane = one window column x, G = 64 / WW column groups, each lane owns a
//     vertical strip of R = ceil(WH / G) patch rows (win 21: 3 x 21 lanes x 7 rows);
//   * the I patch and the interpolated Scharr derivatives stay in VGPRs for all
//     Newton iterations (no LDS at all); derivatives come from the pyramid's
//     precomputed int16x2 planes (withDerivatives layout, lkpyramid.cpp:765-780);
//   * each J row pair is one aligned dwordx2 load + v_alignbyte per lane; the
//     lane's R+1 rows feed R bilinear samples (row reuse in registers);
//   * b / G reductions: DPP within 16-lane rows on 16-bit halves (exact), then
//     four v_readlane into SGPRs -> wave-uniform scalars.
#include "tbdk_internal.hpp"

namespace tbdk {

namespace {

constexpr int W_BITS = 14, W_BITS1 = 14;

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

struct __attribute__((aligned(4))) u32x2 {
    uint32_t lo, hi;
};

// 4 bytes starting at byte address p (any alignment) from two aligned dwords
__device__ __forceinline__ uint32_t load_u8x4(const uint8_t* p)
{
    const uint32_t off = (uint32_t)reinterpret_cast<uintptr_t>(p) & 3u;
    const u32x2 v = *reinterpret_cast<const u32x2*>(p - off);  // keeps the global address space
    return __builtin_amdgcn_alignbyte(v.hi, v.lo, off);
}

template <int CTRL>
__device__ __forceinline__ int dpp(int v)
{
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

// sum over each 16-lane row, result in every lane of the row
__device__ __forceinline__ int row_sum16(int v)
{
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);  // row_half_mirror
    v += dpp<0x140>(v);  // row_mirror
    return v;
}

__device__ __forceinline__ int sum_rows(int v)
{
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}

// exact wave-wide sum of int32 lane values (|v| < 2^31) as int64, uniform
__device__ __forceinline__ long long wave_sum_exact(int v)
{
    const int lo = v & 0xFFFF;  // v = hi * 65536 + lo, lo in [0, 65535]
    const int hi = v >> 16;
    const int slo = sum_rows(row_sum16(lo));
    const int shi = sum_rows(row_sum16(hi));
    return (long long)shi * 65536 + (long long)slo;
}

// wave-wide sum when the total provably fits int32
__device__ __forceinline__ int wave_sum_small(int v) { return sum_rows(row_sum16(v)); }

__device__ __forceinline__ void bilinear_weights(float fa, float fb, int& w00, int& w01, int& w10, int& w11)
{
    w00 = __float2int_rn((1.f - fa) * (1.f - fb) * (1 << W_BITS));
    w01 = __float2int_rn(fa * (1.f - fb) * (1 << W_BITS));
    w10 = __float2int_rn((1.f - fa) * fb * (1 << W_BITS));
    w11 = (1 << W_BITS) - w00 - w01 - w10;
}

}  // namespace

template <int WW, int WH>
__global__ __launch_bounds__(256) void lk_strip_kernel(LkArgs a)
{
    constexpr int G = 64 / WW;              // column groups per wave
    constexpr int R = (WH + G - 1) / G;     // patch rows per lane
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;  // wave-uniform

    const int grp = lane / WW;
    const int x = lane - grp * WW;
    const bool lane_on = grp < G;
    const int row0 = lane_on ? grp * R : 0;
    // number of valid rows of this lane's strip
    const int nrows = lane_on ? (WH - row0 < R ? WH - row0 : R) : 0;

    const float FLT_SCALE = 1.f / (1 << 20);
    const float halfx = (WW - 1) * 0.5f, halfy = (WH - 1) * 0.5f;
    const float p0x = a.prev_pts[2 * i], p0y = a.prev_pts[2 * i + 1];
    float outx = 0.f, outy = 0.f;
    if (a.flags & TBDK_OPTFLOW_USE_INITIAL_FLOW) {
        outx = a.next_pts[2 * i];
        outy = a.next_pts[2 * i + 1];
    }
    int status = 1, nit = 0;
    float errv = 0.f;

    for (int level = a.max_level; level >= 0; --level) {
        const LkLevel L = a.lv[level];
        const float sc = (float)(1. / (1 << level));
        float prevx = p0x * sc, prevy = p0y * sc;
        float nextx, nexty;
        if (level == a.max_level) {
            if (a.flags & TBDK_OPTFLOW_USE_INITIAL_FLOW) {
                nextx = outx * sc;
                nexty = outy * sc;
            } else {
                nextx = prevx;
                nexty = prevy;
            }
        } else {
            nextx = outx * 2.f;
            nexty = outy * 2.f;
        }
        outx = nextx;
        outy = nexty;

        prevx -= halfx;
        prevy -= halfy;
        const int ipx = (int)floorf(prevx), ipy = (int)floorf(prevy);
        if (ipx < -WW || ipx >= L.w || ipy < -WH || ipy >= L.h) {
            if (level == 0) {
                status = 0;
                errv = 0.f;
            }
            continue;
        }
        int iw00, iw01, iw10, iw11;
        bilinear_weights(prevx - ipx, prevy - ipy, iw00, iw01, iw10, iw11);

        // ---- strip of I (2 columns) and of the derivative plane (2 columns), R+1 rows
        int ival[R], gx[R], gy[R];
        int a11 = 0, a12 = 0, a22 = 0;
        {
            const uint8_t* ib = L.I + (size_t)(ipy + row0 + L.ipad) * L.ipitch + (ipx + x + L.ipad);
            const uint8_t* db = L.D + (size_t)(ipy + row0 + L.dpad) * L.dpitch + (size_t)(ipx + x + L.dpad) * 4;
            uint32_t ir[R + 1];
            u32x2 dr[R + 1];
#pragma unroll
            for (int r = 0; r <= R; ++r) {
                ir[r] = load_u8x4(ib + (size_t)r * L.ipitch);
                dr[r] = *reinterpret_cast<const u32x2*>(db + (size_t)r * L.dpitch);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int i00 = ir[r] & 255, i01 = (ir[r] >> 8) & 255;
                const int i10 = ir[r + 1] & 255, i11 = (ir[r + 1] >> 8) & 255;
                const int iv = descale(i00 * iw00 + i01 * iw01 + i10 * iw10 + i11 * iw11, W_BITS1 - 5);
                const int d00 = (int)dr[r].lo, d01 = (int)dr[r].hi, d10 = (int)dr[r + 1].lo, d11 = (int)dr[r + 1].hi;
                const int ix = descale((int16_t)d00 * iw00 + (int16_t)d01 * iw01 + (int16_t)d10 * iw10 +
                                           (int16_t)d11 * iw11, W_BITS1);
                const int iy = descale((d00 >> 16) * iw00 + (d01 >> 16) * iw01 + (d10 >> 16) * iw10 +
                                           (d11 >> 16) * iw11, W_BITS1);
                const bool on = r < nrows;
                ival[r] = iv;
                gx[r] = on ? ix : 0;
                gy[r] = on ? iy : 0;
                a11 += gx[r] * gx[r];
                a12 += gx[r] * gy[r];
                a22 += gy[r] * gy[r];
            }
        }
        const float A11 = (float)wave_sum_exact(a11) * FLT_SCALE;
        const float A12 = (float)wave_sum_exact(a12) * FLT_SCALE;
        const float A22 = (float)wave_sum_exact(a22) * FLT_SCALE;

        float D = A11 * A22 - A12 * A12;
        const float minEig =
            (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * WW * WH);
        if (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS) errv = minEig;
        if (minEig < a.min_eig || D < 1.19209290e-07F /*FLT_EPSILON*/) {
            if (level == 0) status = 0;
            continue;
        }
        D = 1.f / D;

        nextx -= halfx;
        nexty -= halfy;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < a.max_count; ++j) {
            const int inx = (int)floorf(nextx), iny = (int)floorf(nexty);
            if (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h) {
                if (level == 0) status = 0;
                break;
            }
            nit++;
            bilinear_weights(nextx - inx, nexty - iny, iw00, iw01, iw10, iw11);
            const uint8_t* jb = L.J + (size_t)(iny + row0 + L.jpad) * L.jpitch + (inx + x + L.jpad);
            uint32_t jr[R + 1];
#pragma unroll
            for (int r = 0; r <= R; ++r) jr[r] = load_u8x4(jb + (size_t)r * L.jpitch);
            int b1 = 0, b2 = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int j00 = jr[r] & 255, j01 = (jr[r] >> 8) & 255;
                const int j10 = jr[r + 1] & 255, j11 = (jr[r + 1] >> 8) & 255;
                const int diff =
                    descale(j00 * iw00 + j01 * iw01 + j10 * iw10 + j11 * iw11, W_BITS1 - 5) - ival[r];
                b1 += diff * gx[r];
                b2 += diff * gy[r];
            }
            const float fb1 = (float)wave_sum_exact(b1) * FLT_SCALE;
            const float fb2 = (float)wave_sum_exact(b2) * FLT_SCALE;
            const float ddx = (A12 * fb2 - A22 * fb1) * D;
            const float ddy = (A12 * fb1 - A11 * fb2) * D;
            nextx += ddx;
            nexty += ddy;
            outx = nextx + halfx;
            outy = nexty + halfy;
            if ((double)ddx * ddx + (double)ddy * ddy <= a.eps2) break;
            if (j > 0 && (double)fabsf(ddx + pdx) < 0.01 && (double)fabsf(ddy + pdy) < 0.01) {
                outx -= ddx * 0.5f;
                outy -= ddy * 0.5f;
                break;
            }
            pdx = ddx;
            pdy = ddy;
        }

        if (level == 0 && status && a.err && (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS) == 0) {
            const float npx = outx - halfx, npy = outy - halfy;
            const int inx = (int)floorf(npx), iny = (int)floorf(npy);
            if (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h) {
                status = 0;
            } else {
                bilinear_weights(npx - inx, npy - iny, iw00, iw01, iw10, iw11);
                const uint8_t* jb = L.J + (size_t)(iny + row0 + L.jpad) * L.jpitch + (inx + x + L.jpad);
                uint32_t jr[R + 1];
#pragma unroll
                for (int r = 0; r <= R; ++r) jr[r] = load_u8x4(jb + (size_t)r * L.jpitch);
                int e = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int j00 = jr[r] & 255, j01 = (jr[r] >> 8) & 255;
                    const int j10 = jr[r + 1] & 255, j11 = (jr[r + 1] >> 8) & 255;
                    const int diff =
                        descale(j00 * iw00 + j01 * iw01 + j10 * iw10 + j11 * iw11, W_BITS1 - 5) - ival[r];
                    e += r < nrows ? (diff < 0 ? -diff : diff) : 0;
                }
                const float errval = (float)wave_sum_small(e);
                errv = errval * 1.f / (float)(32 * WW * WH);
            }
        }
    }

    if (lane == 0) {
        a.next_pts[2 * i] = outx;
        a.next_pts[2 * i + 1] = outy;
        a.status[i] = (uint8_t)status;
        if (a.err) a.err[i] = errv;
        if (a.iters) a.iters[i] = nit;
    }
}

#define TBDK_STRIP_WINDOWS(X) X(7) X(9) X(11) X(13) X(15) X(17) X(19) X(21) X(23) X(25) X(27) X(29) X(31)

bool lk_strip_supported(int win_w, int win_h)
{
    if (win_w != win_h) return false;
    switch (win_w) {
#define TBDK_CASE(W) case W:
        TBDK_STRIP_WINDOWS(TBDK_CASE)
#undef TBDK_CASE
        return true;
    default:
        return false;
    }
}

hipError_t launch_lk_strip(const LkArgs& a, hipStream_t s)
{
    const dim3 grid((a.n + 3) / 4), block(256);
    switch (a.win_w) {
#define TBDK_CASE(W)                                                             \
    case W:                                                                      \
        hipLaunchKernelGGL((lk_strip_kernel<W, W>), grid, block, 0, s, a);       \
        break;
        TBDK_STRIP_WINDOWS(TBDK_CASE)
#undef TBDK_CASE
    default:
        return hipErrorNotSupported;
    }
    return hipGetLastError();
}

}  // namespace tbdk
