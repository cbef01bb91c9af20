// klt_lk.hip — sparse pyramidal Lucas-Kanade for gfx950, one wave64 per point,
// every pyramid level in one launch.
//
// Numerics follow the CPU cv::calcOpticalFlowPyrLK (LKTrackerInvoker,
// video/src/lkpyramid.cpp:178-695), not the CUDA texture path:
//   * 14-bit fixed-point bilinear weights iw = cvRound(w * 2^14)       (:227-234)
//   * I patch scaled by 32, Scharr derivatives in int16                (:268-420)
//   * Scharr (calcSharrDeriv :55-144) is recomputed on the fly from the
//     LDS-staged (win+3)^2 u8 window; outside the level it is 0, as the
//     BORDER_CONSTANT frame of the reference derivative image (:1357)
//   * minEig gate, eps^2 and oscillation-halving rules                 (:442-652)
//   * L1 error / 32 at level 0                                          (:654-693)
// The G-matrix and b-vector sums are formed EXACTLY (integer products, int32
// lane partials, reduced in double which is exact below 2^53) and rounded to
// float once; the reference sums the same integer terms in float in SSE2-lane
// order.  The two differ only by the reference's float rounding (see the
// oracle's ORC_ACCUM_EXACT / ORC_ACCUM_SSE2 modes and DESIGN.md §Numerics).
// Built with -ffp-contract=off: every remaining float/double expression is
// evaluated exactly as written in the reference.
#include "tbdk_internal.hpp"

namespace tbdk {

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

__device__ __forceinline__ int round_even(float v) { return __float2int_rn(v); }

size_t lk_smem_bytes(int win_w, int win_h)
{
    const int SW = win_w + 3, SH = win_h + 3;
    size_t b = align_up(SW * SH, 16);
    b += align_up((win_w + 1) * (win_h + 1) * 4, 16);
    b += align_up(win_w * win_h * 2, 16);
    b += align_up(win_w * win_h * 4, 16);
    return b;
}

__global__ __launch_bounds__(64) void lk_sparse_kernel(LkArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int i = seg_point(a, xcd_swizzle(blockIdx.x, gridDim.x));
    if (i < 0) return;
    const int lane = threadIdx.x;
    const int winW = a.win_w, winH = a.win_h, area = winW * winH;
    const int SW = winW + 3, SH = winH + 3, DW = winW + 1;
    uint8_t* sI = smem;
    int32_t* sD = reinterpret_cast<int32_t*>(smem + align_up(SW * SH, 16));
    int16_t* sP = reinterpret_cast<int16_t*>(reinterpret_cast<uint8_t*>(sD) + align_up(DW * (winH + 1) * 4, 16));
    int32_t* sG = reinterpret_cast<int32_t*>(reinterpret_cast<uint8_t*>(sP) + align_up(area * 2, 16));

    const int W_BITS = 14, W_BITS1 = 14;
    const float FLT_SCALE = 1.f / (1 << 20);
    const float halfx = (winW - 1) * 0.5f, halfy = (winH - 1) * 0.5f;
    const float p0x = a.prev_pts[2 * i], p0y = a.prev_pts[2 * i + 1];
    float outx = 0.f, outy = 0.f;
    if (a.flags & TBDK_OPTFLOW_USE_INITIAL_FLOW) {
        outx = a.next_pts[2 * i];
        outy = a.next_pts[2 * i + 1];
    }
    int status = 1, nit = 0;
    float errv = 0.f;

    // lane -> patch pixel mapping (p = lane + 64k)
    const int qx = 64 % winW, qy = 64 / winW;
    const int lx0 = lane % winW, ly0 = lane / winW;
    const int dq = 64 % DW, dqy = 64 / DW;
    const int dx0 = lane % DW, dy0 = lane / DW;
    const int sq = 64 % SW, sqy = 64 / SW;
    const int sx0 = lane % SW, sy0 = lane / SW;

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
        if (ipx < -winW || ipx >= L.w || ipy < -winH || ipy >= L.h) {
            if (level == 0) {
                status = 0;
                errv = 0.f;
            }
            continue;
        }
        float fa = prevx - ipx, fb = prevy - ipy;
        int iw00 = round_even((1.f - fa) * (1.f - fb) * (1 << W_BITS));
        int iw01 = round_even(fa * (1.f - fb) * (1 << W_BITS));
        int iw10 = round_even((1.f - fa) * fb * (1 << W_BITS));
        int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

        // ---- stage the (win+3)^2 u8 window of I starting at (ipx-1, ipy-1)
        {
            const uint8_t* base = L.I + (size_t)(ipy - 1 + L.ipad) * L.ipitch + (ipx - 1 + L.ipad);
            int sx = sx0, sy = sy0;
            for (int p = lane; p < SW * SH; p += 64) {
                sI[p] = base[(size_t)sy * L.ipitch + sx];
                sx += sq;
                sy += sqy;
                if (sx >= SW) {
                    sx -= SW;
                    sy += 1;
                }
            }
        }
        __syncthreads();
        // ---- Scharr derivatives on the (win+1)^2 grid; 0 outside the level
        {
            int dx = dx0, dy = dy0;
            for (int p = lane; p < DW * (winH + 1); p += 64) {
                const int X = ipx + dx, Y = ipy + dy;
                int32_t packed = 0;
                if (X >= 0 && X < L.w && Y >= 0 && Y < L.h) {
                    const uint8_t* r0 = sI + dy * SW + dx;  // row Y-1, col X-1
                    const uint8_t* r1 = r0 + SW;
                    const uint8_t* r2 = r1 + SW;
                    const int t0l = (r0[0] + r2[0]) * 3 + r1[0] * 10;
                    const int t0r = (r0[2] + r2[2]) * 3 + r1[2] * 10;
                    const int t1l = r2[0] - r0[0], t1c = r2[1] - r0[1], t1r = r2[2] - r0[2];
                    const int ix = t0r - t0l;
                    const int iy = (t1r + t1l) * 3 + t1c * 10;
                    packed = (int32_t)(((uint32_t)ix & 0xffffu) | ((uint32_t)iy << 16));
                }
                sD[p] = packed;
                dx += dq;
                dy += dqy;
                if (dx >= DW) {
                    dx -= DW;
                    dy += 1;
                }
            }
        }
        __syncthreads();
        // ---- I patch (x32), interpolated derivatives, G partial sums
        int a11 = 0, a12 = 0, a22 = 0;
        {
            int px = lx0, py = ly0;
            for (int p = lane; p < area; p += 64) {
                const uint8_t* s = sI + (py + 1) * SW + (px + 1);
                const int ival = descale(s[0] * iw00 + s[1] * iw01 + s[SW] * iw10 + s[SW + 1] * iw11, W_BITS1 - 5);
                const int32_t* d = sD + py * DW + px;
                const int32_t d00 = d[0], d01 = d[1], d10 = d[DW], d11 = d[DW + 1];
                const int ix = descale((int16_t)d00 * iw00 + (int16_t)d01 * iw01 + (int16_t)d10 * iw10 +
                                           (int16_t)d11 * iw11, W_BITS1);
                const int iy = descale((d00 >> 16) * iw00 + (d01 >> 16) * iw01 + (d10 >> 16) * iw10 +
                                           (d11 >> 16) * iw11, W_BITS1);
                sP[p] = (int16_t)ival;
                sG[p] = (int32_t)(((uint32_t)ix & 0xffffu) | ((uint32_t)iy << 16));
                a11 += ix * ix;
                a12 += ix * iy;
                a22 += iy * iy;
                px += qx;
                py += qy;
                if (px >= winW) {
                    px -= winW;
                    py += 1;
                }
            }
        }
        const float A11 = (float)wave_sum((double)a11) * FLT_SCALE;
        const float A12 = (float)wave_sum((double)a12) * FLT_SCALE;
        const float A22 = (float)wave_sum((double)a22) * FLT_SCALE;

        float D = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                             (float)(2 * winW * winH);
        if (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS) errv = minEig;
        if (minEig < a.min_eig || D < 1.19209290e-07F /*FLT_EPSILON*/) {
            if (level == 0) status = 0;
            __syncthreads();
            continue;
        }
        D = 1.f / D;

        nextx -= halfx;
        nexty -= halfy;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < a.max_count; ++j) {
            const int inx = (int)floorf(nextx), iny = (int)floorf(nexty);
            if (inx < -winW || inx >= L.w || iny < -winH || iny >= L.h) {
                if (level == 0) status = 0;
                break;
            }
            nit++;
            fa = nextx - inx;
            fb = nexty - iny;
            iw00 = round_even((1.f - fa) * (1.f - fb) * (1 << W_BITS));
            iw01 = round_even(fa * (1.f - fb) * (1 << W_BITS));
            iw10 = round_even((1.f - fa) * fb * (1 << W_BITS));
            iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
            const uint8_t* jb = L.J + (size_t)(iny + L.jpad) * L.jpitch + (inx + L.jpad);
            int b1 = 0, b2 = 0;
            int px = lx0, py = ly0;
            for (int p = lane; p < area; p += 64) {
                const uint8_t* q = jb + (size_t)py * L.jpitch + px;
                const int jv = descale(q[0] * iw00 + q[1] * iw01 + q[L.jpitch] * iw10 + q[L.jpitch + 1] * iw11,
                                       W_BITS1 - 5);
                const int diff = jv - sP[p];
                const int32_t g = sG[p];
                b1 += diff * (int16_t)g;
                b2 += diff * (g >> 16);
                px += qx;
                py += qy;
                if (px >= winW) {
                    px -= winW;
                    py += 1;
                }
            }
            const float fb1 = (float)wave_sum((double)b1) * FLT_SCALE;
            const float fb2 = (float)wave_sum((double)b2) * FLT_SCALE;
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
            if (inx < -winW || inx >= L.w || iny < -winH || iny >= L.h) {
                status = 0;
            } else {
                const float aa = npx - inx, bb = npy - iny;
                iw00 = round_even((1.f - aa) * (1.f - bb) * (1 << W_BITS));
                iw01 = round_even(aa * (1.f - bb) * (1 << W_BITS));
                iw10 = round_even((1.f - aa) * bb * (1 << W_BITS));
                iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
                const uint8_t* jb = L.J + (size_t)(iny + L.jpad) * L.jpitch + (inx + L.jpad);
                int e = 0;
                int px = lx0, py = ly0;
                for (int p = lane; p < area; p += 64) {
                    const uint8_t* q = jb + (size_t)py * L.jpitch + px;
                    const int jv = descale(q[0] * iw00 + q[1] * iw01 + q[L.jpitch] * iw10 + q[L.jpitch + 1] * iw11,
                                           W_BITS1 - 5);
                    const int diff = jv - sP[p];
                    e += diff < 0 ? -diff : diff;
                    px += qx;
                    py += qy;
                    if (px >= winW) {
                        px -= winW;
                        py += 1;
                    }
                }
                const float errval = (float)wave_sum((double)e);
                errv = errval * 1.f / (float)(32 * winW * winH);
            }
        }
        __syncthreads();  // LDS is rewritten by the next level
    }

    if (lane == 0) {
        a.next_pts[2 * i] = outx;
        a.next_pts[2 * i + 1] = outy;
        a.status[i] = (uint8_t)status;
        if (a.err) a.err[i] = errv;
        if (a.iters) a.iters[i] = nit;
    }
}

hipError_t launch_lk_sparse(const LkArgs& a, hipStream_t s)
{
    const size_t smem = lk_smem_bytes(a.win_w, a.win_h);
    hipLaunchKernelGGL(lk_sparse_kernel, dim3(a.n), dim3(64), smem, s, a);
    return hipGetLastError();
}

}  // namespace tbdk
