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
//     Newton iterations (no LDS); derivatives come from the pyramid's
//     precomputed int16x2 planes (withDerivatives layout, lkpyramid.cpp:765-780);
//   * buffer loads with 32-bit lane offsets and the row offset in an SGPR
//     (soffset); one aligned dwordx2 per row, v_perm_b32 picks the two pixels
//     as an int16 pair, v_dot2_i32_i16 does the 14-bit fixed-point bilinear
//     (same int16 x int16 products as the reference's _mm_madd_epi16, :288-303);
//   * the J strip is re-loaded only when the integer window origin moves (near
//     convergence the Newton steps are sub-pixel, so most iterations are pure VALU);
//   * G / b sums: DPP over 8-lane groups in int32 (cannot overflow), eight
//     v_readlane into SGPRs, int64 scalar sum -> exact, wave-uniform.
#include "lk_device.hpp"

namespace tbdk {

namespace {

using namespace lkdev;

template <int CTRL>
__device__ __forceinline__ int dpp(int v)
{
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

// exact wave-wide sums of N int32 lane values: DPP inside GROUP-lane groups in
// int32, then an int64 scalar sum of the 64/GROUP group totals.  The caller
// picks GROUP so that GROUP * (max |lane partial|) < 2^31 (lane partial of a
// strip of R rows: R * 8160 * 4081 for b, R * 4081^2 for G).  Result is
// uniform (SGPR).
template <int GROUP, int N>
__device__ __forceinline__ void wave_sum_exact(int (&v)[N], long long (&out)[N])
{
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] += dpp<0xB1>(v[k]);  // quad_perm [1,0,3,2]
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] += dpp<0x4E>(v[k]);  // quad_perm [2,3,0,1]
    if constexpr (GROUP >= 8) {
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] += dpp<0x141>(v[k]);  // row_half_mirror
    }
    if constexpr (GROUP >= 16) {
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] += dpp<0x140>(v[k]);  // row_mirror
    }
#pragma unroll
    for (int k = 0; k < N; ++k) {
        long long s = 0;
#pragma unroll
        for (int g = 0; g < 64 / GROUP; ++g) s += (long long)__builtin_amdgcn_readlane(v[k], GROUP * g);
        out[k] = s;
    }
}

}  // namespace

template <int WW, int WH>
__global__ __launch_bounds__(256) void lk_strip_kernel(LkArgs a)
{
    constexpr int G = 64 / WW;           // column groups per wave
    constexpr int R = (WH + G - 1) / G;  // patch rows per lane
    constexpr int GRP = R <= 4 ? 16 : (R <= 8 ? 8 : 4);  // exact-reduction group (see wave_sum_exact)
    const int lane = threadIdx.x & 63;
    const int i = seg_point(a, xcd_swizzle(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
    if (i < 0) return;  // wave-uniform

    const int grp = lane / WW;
    const int x = lane - grp * WW;
    const bool lane_on = grp < G;
    const int row0 = lane_on ? grp * R : 0;
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
        uint32_t w0, w1;
        bilinear_weights(prevx - ipx, prevy - ipy, w0, w1);

        const int hp = L.h + 2 * L.ipad;
        const __amdgpu_buffer_rsrc_t rI = make_rsrc(L.I, L.ipitch * hp + 256);
        const __amdgpu_buffer_rsrc_t rD = make_rsrc(L.D, L.dpitch * (L.h + 2 * L.dpad) + 256);
        const __amdgpu_buffer_rsrc_t rJ = make_rsrc(L.J, L.jpitch * (L.h + 2 * L.jpad) + 256);

        // ---- I strip (2 columns) and derivative strip (2 columns), R+1 rows
        int ival[R], gx[R], gy[R];
        {
            const uint32_t ioff = (uint32_t)((ipy + row0 + L.ipad) * L.ipitch + ipx + x + L.ipad);
            const uint32_t doff = (uint32_t)((ipy + row0 + L.dpad) * L.dpitch + (ipx + x + L.dpad) * 4);
            uint32_t ip[R + 1], dxp[R + 1], dyp[R + 1];
#pragma unroll
            for (int r = 0; r <= R; ++r) {
                ip[r] = load_pair_u8_ua(rI, ioff, r * L.ipitch);
                const uint32_t d0 = __builtin_amdgcn_raw_buffer_load_b32(rD, doff, r * L.dpitch, 0);
                const uint32_t d1 = __builtin_amdgcn_raw_buffer_load_b32(rD, doff + 4, r * L.dpitch, 0);
                dxp[r] = __builtin_amdgcn_perm(d1, d0, 0x05040100u);  // (Ix(x), Ix(x+1))
                dyp[r] = __builtin_amdgcn_perm(d1, d0, 0x07060302u);  // (Iy(x), Iy(x+1))
            }
            int acc[3] = {0, 0, 0};
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const bool on = r < nrows;
                ival[r] = bilin(ip[r], ip[r + 1], w0, w1, W_BITS1 - 5);
                const int ix = bilin(dxp[r], dxp[r + 1], w0, w1, W_BITS1);
                const int iy = bilin(dyp[r], dyp[r + 1], w0, w1, W_BITS1);
                gx[r] = on ? ix : 0;
                gy[r] = on ? iy : 0;
                acc[0] += gx[r] * gx[r];
                acc[1] += gx[r] * gy[r];
                acc[2] += gy[r] * gy[r];
            }
            long long s[3];
            wave_sum_exact<GRP, 3>(acc, s);
            // A = float(exact sum) * 2^-20   (lkpyramid.cpp:438-440)
            const float A11 = (float)s[0] * FLT_SCALE;
            const float A12 = (float)s[1] * FLT_SCALE;
            const float A22 = (float)s[2] * FLT_SCALE;

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
            int pinx = 0x7fffffff, piny = 0;
            uint32_t jp[R + 1];
#pragma unroll
            for (int r = 0; r <= R; ++r) jp[r] = 0;
            for (int j = 0; j < a.max_count; ++j) {
                const int inx = (int)floorf(nextx), iny = (int)floorf(nexty);
                if (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h) {
                    if (level == 0) status = 0;
                    break;
                }
                nit++;
                if (inx != pinx || iny != piny) {  // uniform: reload the J strip
                    const uint32_t joff = (uint32_t)((iny + row0 + L.jpad) * L.jpitch + inx + x + L.jpad);
#pragma unroll
                    for (int r = 0; r <= R; ++r) jp[r] = load_pair_u8_ua(rJ, joff, r * L.jpitch);
                    pinx = inx;
                    piny = iny;
                }
                bilinear_weights(nextx - inx, nexty - iny, w0, w1);
                int b[2] = {0, 0};
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int diff = bilin(jp[r], jp[r + 1], w0, w1, W_BITS1 - 5) - ival[r];
                    b[0] += diff * gx[r];
                    b[1] += diff * gy[r];
                }
                long long sb[2];
                wave_sum_exact<GRP, 2>(b, sb);
                const float fb1 = (float)sb[0] * FLT_SCALE;
                const float fb2 = (float)sb[1] * FLT_SCALE;
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
        }

        if (level == 0 && status && a.err && (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS) == 0) {
            const float npx = outx - halfx, npy = outy - halfy;
            const int inx = (int)floorf(npx), iny = (int)floorf(npy);
            if (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h) {
                status = 0;
            } else {
                bilinear_weights(npx - inx, npy - iny, w0, w1);
                const uint32_t joff = (uint32_t)((iny + row0 + L.jpad) * L.jpitch + inx + x + L.jpad);
                uint32_t jp[R + 1];
#pragma unroll
                for (int r = 0; r <= R; ++r) jp[r] = load_pair_u8_ua(rJ, joff, r * L.jpitch);
                int e[1] = {0};
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int diff = bilin(jp[r], jp[r + 1], w0, w1, W_BITS1 - 5) - ival[r];
                    e[0] += r < nrows ? (diff < 0 ? -diff : diff) : 0;
                }
                long long se[1];
                wave_sum_exact<GRP, 1>(e, se);
                const float errval = (float)se[0];
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
#define TBDK_CASE(W)                                                       \
    case W:                                                                \
        hipLaunchKernelGGL((lk_strip_kernel<W, W>), grid, block, 0, s, a); \
        break;
        TBDK_STRIP_WINDOWS(TBDK_CASE)
#undef TBDK_CASE
    default:
        return hipErrorNotSupported;
    }
    return hipGetLastError();
}

}  // namespace tbdk
