// klt_cn_f32.hip — multi-channel 16-bit / float frames on the fp32 pixel path
// (cv::cuda::SparsePyrLKOpticalFlow on CV_16UC3/C4 and CV_32FC3/C4,
// cudaoptflow/src/pyrlk.cpp:189-205), for gfx950.
//
// Numerics: the fp32 pixel path of klt_f16.hip (levels pyrDown_<FltCast<float,8>>
// in its scalar order, calcSharrDeriv's formula, fma bilinear chains, per window
// column the rows accumulated by fma in row order, the columns then summed in
// order) with the CPU path's channel handling (video/src/lkpyramid.cpp:55-144,
// 178-695): a window row is winW * cn elements, column e = pixel e / cn, channel
// e % cn; G and b sum over all elements; minEig normalised by 2 * winW * winH,
// the error by 32 * winW * cn * winH.  The definition is oracle/klt16_oracle.c
// (orc16_lk on fp32 levels with cn channels), matched bit for bit.
//
// Layout: one wave per point (these depths are rare and the windows are cn
// times wider than the gray path's): the window's I, Ix, Iy values of a level in
// LDS (3 x winH x winW*cn floats), lanes over its elements; the column sums in
// LDS, added in column order by one lane per value.  Pyramids: interleaved fp32
// levels with a reflect-101 frame of pad pixels, fp32 (Ix, Iy) pairs per element
// with a zero frame (the fp32 layout of tbdk_pyr_create_f32, cn values per pixel).
#include <atomic>

#include "lk_device.hpp"

namespace tbdk {

namespace {

__device__ __forceinline__ int reflect101c(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ float bil4(float w00, float w01, float w10, float w11, float v00, float v01, float v10,
                                      float v11, float c)
{
    float t = __builtin_fmaf(w00, v00, c);
    t = __builtin_fmaf(w01, v01, t);
    t = __builtin_fmaf(w10, v10, t);
    return __builtin_fmaf(w11, v11, t);
}

}  // namespace

// level 0: one element of a padded row per thread, converted exactly from a u8
// (kind 0), u16 (1) or fp32 (2) frame of cn interleaved channels
__global__ void pyr_cn_f32_copy_kernel(const uint8_t* __restrict__ src, int spitch, int kind, int cn, tbdk_level d)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y;
    if (e >= (d.width + 2 * d.pad) * cn) return;
    const int px = e / cn, c = e - px * cn;
    const uint8_t* srow = src + (size_t)reflect101c(py - d.pad, d.height) * spitch;
    const int se = reflect101c(px - d.pad, d.width) * cn + c;
    const float v = kind == 2 ? reinterpret_cast<const float*>(srow)[se]
                              : kind == 1 ? (float)reinterpret_cast<const uint16_t*>(srow)[se] : (float)srow[se];
    reinterpret_cast<float*>(d.data + (size_t)py * d.pitch)[e] = v;
}

// pyrDown of a padded fp32 cn level into a padded level (the source's frame is
// its reflect-101, pad >= 2), one element per thread
__global__ void pyr_cn_f32_down_kernel(tbdk_level s, tbdk_level d, int cn)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y;
    if (e >= (d.width + 2 * d.pad) * cn) return;
    const int px = e / cn, c = e - px * cn;
    const int rx = reflect101c(px - d.pad, d.width), ry = reflect101c(py - d.pad, d.height);
    const float* s0 = reinterpret_cast<const float*>(s.data + (size_t)(2 * ry - 2 + s.pad) * s.pitch) +
                      (size_t)(s.pad + 2 * rx) * cn + c;
    float r[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float* q = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(s0) + (size_t)j * s.pitch);
        r[j] = q[0] * 6.f + (q[-cn] + q[cn]) * 4.f + q[-2 * cn] + q[2 * cn];
    }
    reinterpret_cast<float*>(d.data + (size_t)py * d.pitch)[e] =
        (r[2] * 6.f + (r[1] + r[3]) * 4.f + r[0] + r[4]) * (1.f / 256.f);
}

// calcSharrDeriv's formula per element, neighbours cn elements apart (the
// level's reflect-101 frame), stored as fp32 (Ix, Iy) pairs
__global__ void scharr_cn_f32_kernel(tbdk_level L, tbdk_level D, int cn)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (e >= L.width * cn) return;
    const float* r1 = reinterpret_cast<const float*>(L.data + (size_t)(y + L.pad) * L.pitch) + (size_t)L.pad * cn + e;
    const float* r0 = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(r1) - L.pitch);
    const float* r2 = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(r1) + L.pitch);
    float t0[3], t1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int o = (k - 1) * cn;
        t0[k] = (r0[o] + r2[o]) * 3.f + r1[o] * 10.f;
        t1[k] = r2[o] - r0[o];
    }
    float2* d = reinterpret_cast<float2*>(D.data + (size_t)(y + D.pad) * D.pitch) + (size_t)D.pad * cn + e;
    *d = make_float2(t0[2] - t0[0], (t1[2] + t1[0]) * 3.f + t1[1] * 10.f);
}

hipError_t launch_pyr_build_f32_cn(const uint8_t* img, int pitch, int kind, const tbdk_pyr& pyr, hipStream_t s)
{
    const int cn = pyr.cn;
    for (int l = 0; l < pyr.nlevels; ++l) {
        const tbdk_level& L = pyr.lv[l];
        const dim3 grid(((L.width + 2 * L.pad) * cn + 255) / 256, L.height + 2 * L.pad);
        if (l == 0) hipLaunchKernelGGL(pyr_cn_f32_copy_kernel, grid, dim3(256), 0, s, img, pitch, kind, cn, L);
        else hipLaunchKernelGGL(pyr_cn_f32_down_kernel, grid, dim3(256), 0, s, pyr.lv[l - 1], L, cn);
        if (pyr.dv[l].data)
            hipLaunchKernelGGL(scharr_cn_f32_kernel, dim3((L.width * cn + 255) / 256, L.height), dim3(256), 0, s, L,
                               pyr.dv[l], cn);
    }
    return hipGetLastError();
}

// one wave per point; dynamic LDS: I, Ix, Iy of the window (winH x winW*cn each),
// then three column-partial rows of winW*cn and three totals
__global__ __launch_bounds__(64) void lk_cn_f32_kernel(LkArgs a)
{
    extern __shared__ float smem[];
    const int i = seg_point(a, blockIdx.x);
    if (i < 0) return;  // the whole wave
    const int lane = threadIdx.x;
    const int cn = a.cn, WW = a.win_w, WH = a.win_h, WE = WW * cn, AREA = WE * WH;
    float* const iv = smem;
    float* const gx = iv + AREA;
    float* const gy = gx + AREA;
    float* const col = gy + AREA;  // [3][WE]
    float* const tot = col + 3 * WE;
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
    // totals of nv column-partial rows, each added in column order by one lane
    auto ordered_sums = [&](int nv) {
        __syncthreads();
        if (lane < nv) {
            const float* q = col + lane * WE;
            float t = q[0];
            for (int e = 1; e < WE; ++e) t += q[e];
            tot[lane] = t;
        }
        __syncthreads();
    };

    for (int level = a.max_level; level >= 0; --level) {
        const LkLevel L = a.lv[level];
        const float sc = (float)(1. / (1 << level));
        float prevx = p0x * sc, prevy = p0y * sc, nextx, nexty;
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
        float a_ = prevx - ipx, b_ = prevy - ipy;
        float w00 = (1.f - a_) * (1.f - b_), w01 = a_ * (1.f - b_), w10 = (1.f - a_) * b_, w11 = a_ * b_;
        // the window's I, Ix, Iy (padded level: reflect-101 frame; derivative planes: zero frame)
        for (int k = lane; k < AREA; k += 64) {
            const int r = k / WE, e = k - r * WE;
            const int x = e / cn, c = e - x * cn;
            const float* p = reinterpret_cast<const float*>(L.I + (size_t)(ipy + r + L.ipad) * L.ipitch) +
                             (size_t)(ipx + x + L.ipad) * cn + c;
            const float* pn = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(p) + L.ipitch);
            iv[k] = bil4(w00, w01, w10, w11, p[0], p[cn], pn[0], pn[cn], 0.f);
            const float2* d = reinterpret_cast<const float2*>(L.D + (size_t)(ipy + r + L.dpad) * L.dpitch) +
                              (size_t)(ipx + x + L.dpad) * cn + c;
            const float2* dn = reinterpret_cast<const float2*>(reinterpret_cast<const uint8_t*>(d) + L.dpitch);
            const float2 d00 = d[0], d01 = d[cn], d10 = dn[0], d11 = dn[cn];
            gx[k] = bil4(w00, w01, w10, w11, d00.x, d01.x, d10.x, d11.x, 0.f);
            gy[k] = bil4(w00, w01, w10, w11, d00.y, d01.y, d10.y, d11.y, 0.f);
        }
        __syncthreads();
        for (int e = lane; e < WE; e += 64) {
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            for (int r = 0; r < WH; ++r) {
                const float x_ = gx[r * WE + e], y_ = gy[r * WE + e];
                s0 = __builtin_fmaf(x_, x_, s0);
                s1 = __builtin_fmaf(x_, y_, s1);
                s2 = __builtin_fmaf(y_, y_, s2);
            }
            col[e] = s0;
            col[WE + e] = s1;
            col[2 * WE + e] = s2;
        }
        ordered_sums(3);
        const float A11 = tot[0] * FLT_SCALE, A12 = tot[1] * FLT_SCALE, A22 = tot[2] * FLT_SCALE;
        float D = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * WW * WH);
        if (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS) errv = minEig;
        if (minEig < a.min_eig || D < 1.19209290e-07F) {
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
            ++nit;
            a_ = nextx - inx;
            b_ = nexty - iny;
            w00 = (1.f - a_) * (1.f - b_);
            w01 = a_ * (1.f - b_);
            w10 = (1.f - a_) * b_;
            w11 = a_ * b_;
            for (int e = lane; e < WE; e += 64) {
                const int x = e / cn, c = e - x * cn;
                const float* q = reinterpret_cast<const float*>(L.J + (size_t)(iny + L.jpad) * L.jpitch) +
                                 (size_t)(inx + x + L.jpad) * cn + c;
                float bx = 0.f, by = 0.f;
                for (int r = 0; r < WH; ++r) {
                    const float* qn = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(q) + L.jpitch);
                    const float d = bil4(w00, w01, w10, w11, q[0], q[cn], qn[0], qn[cn], -iv[r * WE + e]);
                    bx = __builtin_fmaf(d, gx[r * WE + e], bx);
                    by = __builtin_fmaf(d, gy[r * WE + e], by);
                    q = qn;
                }
                col[e] = bx;
                col[WE + e] = by;
            }
            ordered_sums(2);
            const float b1 = tot[0] * (32.f * FLT_SCALE), b2 = tot[1] * (32.f * FLT_SCALE);
            const float ddx = (A12 * b2 - A22 * b1) * D;
            const float ddy = (A12 * b1 - A11 * b2) * D;
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
        if (level == 0 && a.err && (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS) == 0 && status) {
            const float npx = outx - halfx, npy = outy - halfy;
            const int inx = (int)floorf(npx), iny = (int)floorf(npy);
            if (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h) {
                status = 0;
            } else {
                a_ = npx - inx;
                b_ = npy - iny;
                w00 = (1.f - a_) * (1.f - b_);
                w01 = a_ * (1.f - b_);
                w10 = (1.f - a_) * b_;
                w11 = a_ * b_;
                for (int e = lane; e < WE; e += 64) {
                    const int x = e / cn, c = e - x * cn;
                    const float* q = reinterpret_cast<const float*>(L.J + (size_t)(iny + L.jpad) * L.jpitch) +
                                     (size_t)(inx + x + L.jpad) * cn + c;
                    float ev = 0.f;
                    for (int r = 0; r < WH; ++r) {
                        const float* qn = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(q) + L.jpitch);
                        ev += fabsf(bil4(w00, w01, w10, w11, q[0], q[cn], qn[0], qn[cn], -iv[r * WE + e]));
                        q = qn;
                    }
                    col[e] = ev;
                }
                ordered_sums(1);
                // lkpyramid.cpp:690: errval / (32 * winSize.width * cn * winSize.height)
                errv = (tot[0] * 32.f) * (1.f / (float)(32 * WW * cn * WH));
            }
        }
        __syncthreads();  // the window arrays are rewritten by the next level
    }
    if (lane == 0) {
        a.next_pts[2 * i] = outx;
        a.next_pts[2 * i + 1] = outy;
        a.status[i] = (uint8_t)status;
        if (a.err) a.err[i] = errv;
        if (a.iters) a.iters[i] = nit;
    }
}

size_t lk_cn_f32_smem_bytes(int win_w, int win_h, int cn)
{
    const size_t we = (size_t)win_w * cn;
    return (3 * we * win_h + 3 * we + 4) * sizeof(float);
}

hipError_t launch_lk_cn_f32(const LkArgs& a, hipStream_t s)
{
    const size_t smem = lk_cn_f32_smem_bytes(a.win_w, a.win_h, a.cn);
    static std::atomic<unsigned long long> opted{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (smem > 64 * 1024 && !(opted.load(std::memory_order_acquire) & bit)) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lk_cn_f32_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        opted.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL(lk_cn_f32_kernel, dim3(a.n), dim3(64), smem, s, a);
    return hipGetLastError();
}

}  // namespace tbdk
