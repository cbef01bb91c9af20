// klt_cn.hip — PyrLK on multi-channel (interleaved cn = 2..4) u8 frames:
// the pyramid levels, their CV_16SC(2cn) Scharr planes and the sparse
// tracker, for gfx950.
//
// The CPU path handles any channel count the same way (video/src/lkpyramid.cpp):
//   * pyrDown_ of an interleaved image filters each channel on its own
//     (imgproc/src/pyramids.cpp:746-790: the border tables hold pixel*cn + c)
//   * calcSharrDeriv (:55-144) runs over rows of cols*cn elements whose
//     horizontal neighbours are cn elements apart; per pixel the plane holds
//     (Ix_c, Iy_c) for c = 0..cn-1
//   * LKTrackerInvoker (:178-695) walks the window as winW*cn elements per row
//     (bilinear neighbours cn elements / 2cn derivative values apart), G and b
//     summed over all of them, minEig normalised by 2*winW*winH, the level-0
//     error by 32*winW*cn*winH.
// As for one channel, the G and b sums are formed exactly (int64 lane partials,
// an exact double wave reduction) and rounded to float once: bit-exact with the
// oracle's ORC_ACCUM_EXACT mode (oracle/klt_oracle.c, cn-generic).
// This is not the TBD path (the sample tracks 8-bit gray frames); the kernels
// are straightforward: one thread per element for the pyramid and the planes,
// one wave per point with the window in LDS for the tracker.
#include <atomic>

#include "tbdk_internal.hpp"

namespace tbdk {

namespace {

__device__ __forceinline__ int crefl(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ int cdescale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

__device__ __forceinline__ double cwave_sum(double v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

}  // namespace

// level 0: the frame into the padded level, reflect-101 frame of `pad` pixels
__global__ __launch_bounds__(256) void pyr_cn_copy_kernel(const uint8_t* __restrict__ img, int pitch, tbdk_level L,
                                                          int cn)
{
    const int ex = blockIdx.x * 256 + threadIdx.x;  // element of the padded row
    const int yp = blockIdx.y;
    const int wp = L.width + 2 * L.pad;
    if (ex >= wp * cn) return;
    const int xp = ex / cn, c = ex - xp * cn;
    const int x = crefl(xp - L.pad, L.width), y = crefl(yp - L.pad, L.height);
    L.data[(size_t)yp * L.pitch + ex] = img[(size_t)y * pitch + (size_t)x * cn + c];
}

// level l+1 from level l: pyrDown_ (5x5 [1 4 6 4 1]^2, (s + 128) >> 8) of the
// isolated level, evaluated at every element of the padded destination (the
// frame at its reflect-101 interior position)
__global__ __launch_bounds__(256) void pyr_cn_down_kernel(tbdk_level S, tbdk_level D, int cn)
{
    const int ex = blockIdx.x * 256 + threadIdx.x;
    const int yp = blockIdx.y;
    const int wp = D.width + 2 * D.pad;
    if (ex >= wp * cn) return;
    const int xp = ex / cn, c = ex - xp * cn;
    const int x = crefl(xp - D.pad, D.width), y = crefl(yp - D.pad, D.height);
    const uint8_t* src = S.data + (size_t)S.pad * S.pitch + (size_t)S.pad * cn + c;
    int cols[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) cols[i] = crefl(2 * x + i - 2, S.width) * cn;
    int r[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const uint8_t* s = src + (size_t)crefl(2 * y + j - 2, S.height) * S.pitch;
        r[j] = s[cols[2]] * 6 + (s[cols[1]] + s[cols[3]]) * 4 + s[cols[0]] + s[cols[4]];
    }
    const int v = r[2] * 6 + (r[1] + r[3]) * 4 + r[0] + r[4];
    D.data[(size_t)yp * D.pitch + ex] = (uint8_t)((v + 128) >> 8);
}

// calcSharrDeriv over the interior (the zero frame is written at creation)
__global__ __launch_bounds__(256) void scharr_cn_kernel(tbdk_level L, tbdk_level Dv, int cn)
{
    const int ex = blockIdx.x * 256 + threadIdx.x;  // element x*cn + c of an interior row
    const int y = blockIdx.y;
    const int wn = L.width * cn;
    if (ex >= wn) return;
    const int x = ex / cn, c = ex - x * cn;
    const int h = L.height, w = L.width;
    const uint8_t* base = L.data + (size_t)L.pad * L.pitch + (size_t)L.pad * cn + c;
    const uint8_t* s0 = base + (size_t)(y > 0 ? y - 1 : (h > 1 ? 1 : 0)) * L.pitch;
    const uint8_t* s1 = base + (size_t)y * L.pitch;
    const uint8_t* s2 = base + (size_t)(y < h - 1 ? y + 1 : (h > 1 ? h - 2 : 0)) * L.pitch;
    // the row buffers' borders copy column 1 / w-2 (lkpyramid.cpp:111-116)
    const int xl = (x > 0 ? x - 1 : (w > 1 ? 1 : 0)) * cn, xr = (x < w - 1 ? x + 1 : (w > 1 ? w - 2 : 0)) * cn;
    const int xc = x * cn;
    const int t0l = (int16_t)((s0[xl] + s2[xl]) * 3 + s1[xl] * 10), t0r = (int16_t)((s0[xr] + s2[xr]) * 3 + s1[xr] * 10);
    const int t1l = (int16_t)(s2[xl] - s0[xl]), t1c = (int16_t)(s2[xc] - s0[xc]), t1r = (int16_t)(s2[xr] - s0[xr]);
    int16_t* d = reinterpret_cast<int16_t*>(Dv.data + (size_t)(y + Dv.pad) * Dv.pitch) + (size_t)(Dv.pad * cn + ex) * 2;
    d[0] = (int16_t)(t0r - t0l);
    d[1] = (int16_t)((t1r + t1l) * 3 + t1c * 10);
}

// one wave per point, every level; LDS: the window's I (x32) and interpolated
// (Ix, Iy), winW*winH*cn elements each
__global__ __launch_bounds__(64) void lk_cn_kernel(LkArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int i = seg_point(a, xcd_swizzle(blockIdx.x, gridDim.x));
    if (i < 0) return;
    const int lane = threadIdx.x;
    const int cn = a.cn, cn2 = 2 * cn;
    const int winW = a.win_w, winH = a.win_h, wcn = winW * cn, area = wcn * winH;
    int16_t* sP = reinterpret_cast<int16_t*>(smem);
    int32_t* sG = reinterpret_cast<int32_t*>(smem + align_up(area * 2, 16));

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
        int iw00 = __float2int_rn((1.f - fa) * (1.f - fb) * (1 << W_BITS));
        int iw01 = __float2int_rn(fa * (1.f - fb) * (1 << W_BITS));
        int iw10 = __float2int_rn((1.f - fa) * fb * (1 << W_BITS));
        int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

        // ---- I patch (x32), interpolated derivatives, G partial sums (exact)
        int64_t a11 = 0, a12 = 0, a22 = 0;
        {
            const uint8_t* ib = L.I + (size_t)(ipy + L.ipad) * L.ipitch + (size_t)(ipx + L.ipad) * cn;
            const int dstep = L.dpitch / 2;
            const int16_t* db = reinterpret_cast<const int16_t*>(L.D + (size_t)(ipy + L.dpad) * L.dpitch) +
                                (size_t)(ipx + L.dpad) * cn2;
            for (int p = lane; p < area; p += 64) {
                const int y = p / wcn, x = p - y * wcn;
                const uint8_t* s = ib + (size_t)y * L.ipitch + x;
                const int ival = cdescale(s[0] * iw00 + s[cn] * iw01 + s[L.ipitch] * iw10 + s[L.ipitch + cn] * iw11,
                                          W_BITS1 - 5);
                const int16_t* d = db + (size_t)y * dstep + 2 * x;
                const int ix = cdescale(d[0] * iw00 + d[cn2] * iw01 + d[dstep] * iw10 + d[dstep + cn2] * iw11, W_BITS1);
                const int iy = cdescale(d[1] * iw00 + d[cn2 + 1] * iw01 + d[dstep + 1] * iw10 + d[dstep + cn2 + 1] * iw11,
                                        W_BITS1);
                sP[p] = (int16_t)ival;
                sG[p] = (int32_t)(((uint32_t)(int16_t)ix & 0xffffu) | ((uint32_t)iy << 16));
                a11 += (int64_t)(int16_t)ix * (int16_t)ix;
                a12 += (int64_t)(int16_t)ix * (int16_t)iy;
                a22 += (int64_t)(int16_t)iy * (int16_t)iy;
            }
        }
        const float A11 = (float)cwave_sum((double)a11) * FLT_SCALE;
        const float A12 = (float)cwave_sum((double)a12) * FLT_SCALE;
        const float A22 = (float)cwave_sum((double)a22) * FLT_SCALE;
        __syncthreads();  // sP / sG complete

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
            iw00 = __float2int_rn((1.f - fa) * (1.f - fb) * (1 << W_BITS));
            iw01 = __float2int_rn(fa * (1.f - fb) * (1 << W_BITS));
            iw10 = __float2int_rn((1.f - fa) * fb * (1 << W_BITS));
            iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
            const uint8_t* jb = L.J + (size_t)(iny + L.jpad) * L.jpitch + (size_t)(inx + L.jpad) * cn;
            int64_t b1 = 0, b2 = 0;
            for (int p = lane; p < area; p += 64) {
                const int y = p / wcn, x = p - y * wcn;
                const uint8_t* q = jb + (size_t)y * L.jpitch + x;
                const int jv = cdescale(q[0] * iw00 + q[cn] * iw01 + q[L.jpitch] * iw10 + q[L.jpitch + cn] * iw11,
                                        W_BITS1 - 5);
                const int diff = jv - sP[p];
                const int32_t g = sG[p];
                b1 += (int64_t)diff * (int16_t)g;
                b2 += (int64_t)diff * (g >> 16);
            }
            const float fb1 = (float)cwave_sum((double)b1) * FLT_SCALE;
            const float fb2 = (float)cwave_sum((double)b2) * FLT_SCALE;
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
                iw00 = __float2int_rn((1.f - aa) * (1.f - bb) * (1 << W_BITS));
                iw01 = __float2int_rn(aa * (1.f - bb) * (1 << W_BITS));
                iw10 = __float2int_rn((1.f - aa) * bb * (1 << W_BITS));
                iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
                const uint8_t* jb = L.J + (size_t)(iny + L.jpad) * L.jpitch + (size_t)(inx + L.jpad) * cn;
                int64_t e = 0;
                for (int p = lane; p < area; p += 64) {
                    const int y = p / wcn, x = p - y * wcn;
                    const uint8_t* q = jb + (size_t)y * L.jpitch + x;
                    const int jv = cdescale(q[0] * iw00 + q[cn] * iw01 + q[L.jpitch] * iw10 + q[L.jpitch + cn] * iw11,
                                            W_BITS1 - 5);
                    const int diff = jv - sP[p];
                    e += diff < 0 ? -diff : diff;
                }
                // the reference adds |diff| in float in window order: equal to the
                // exact integer sum while that stays below 2^24
                const float errval = (float)cwave_sum((double)e);
                errv = errval * 1.f / (float)(32 * winW * cn * winH);
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

size_t lk_cn_smem_bytes(int win_w, int win_h, int cn)
{
    const size_t area = (size_t)win_w * win_h * cn;
    return align_up((int)(area * 2), 16) + area * 4;
}

hipError_t launch_pyr_cn(const uint8_t* img, int pitch, const tbdk_pyr& pyr, hipStream_t s)
{
    const int cn = pyr.cn;
    for (int l = 0; l < pyr.nlevels; ++l) {
        const tbdk_level& L = pyr.lv[l];
        const dim3 grid(((L.width + 2 * L.pad) * cn + 255) / 256, L.height + 2 * L.pad);
        if (l == 0) hipLaunchKernelGGL(pyr_cn_copy_kernel, grid, dim3(256), 0, s, img, pitch, L, cn);
        else hipLaunchKernelGGL(pyr_cn_down_kernel, grid, dim3(256), 0, s, pyr.lv[l - 1], L, cn);
        if (pyr.dv[l].data)
            hipLaunchKernelGGL(scharr_cn_kernel, dim3((L.width * cn + 255) / 256, L.height), dim3(256), 0, s, L,
                               pyr.dv[l], cn);
    }
    return hipGetLastError();
}

hipError_t launch_lk_cn(const LkArgs& a, hipStream_t s)
{
    const size_t smem = lk_cn_smem_bytes(a.win_w, a.win_h, a.cn);
    // > 64 KiB of LDS (large windows x 4 channels) must be opted into, once per device
    static std::atomic<unsigned long long> opted{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (smem > 64 * 1024 && !(opted.load(std::memory_order_acquire) & bit)) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lk_cn_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
        if (e != hipSuccess) return e;
        opted.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL(lk_cn_kernel, dim3(a.n), dim3(64), smem, s, a);
    return hipGetLastError();
}

}  // namespace tbdk
