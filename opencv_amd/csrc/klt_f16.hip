// klt_f16.hip — the fp16 pixel path of sparse PyrLK (BASELINE
// configs[4]) for gfx950.
//
// The reference has no fp16 (or fp32) CPU PyrLK: calcSharrDeriv and
// LKTrackerInvoker take 8-bit levels only (video/src/lkpyramid.cpp:57,
// 1272-1276); cv::cuda::SparsePyrLKOpticalFlow accepts CV_32F images through
// texture fetches (cudaoptflow/src/pyrlk.cpp:197-205, cuda/pyrlk.cu:67-85).
// This path keeps the CPU algorithm of LKTrackerInvoker (lkpyramid.cpp:178-695:
// window origin, bounds gates, minEig / det gate, eps^2 stop, oscillation
// halving, L1 error) and replaces its fixed-point steps by fp32 on fp16 pixels:
//   * levels: fp16, pyrDown_<FltCast<float,8>> in its scalar expression order
//     (imgproc/src/pyramids.cpp:775-777, 856: s2*6 + (s1+s3)*4 + s0 + s4, then
//     x 1/256), rounded to fp16 (round to nearest even);
//   * derivatives: calcSharrDeriv's formula (lkpyramid.cpp:86-131) in fp32,
//     stored as fp16 (Ix, Iy) pairs with a zero frame;
//   * bilinear weights (1-a)(1-b), a(1-b), (1-a)b, ab in fp32; every window
//     value an fma chain over the four fp16 taps; per window column the rows
//     accumulated by fma in row order, the columns then summed left to right.
// The restated order is oracle/klt16_oracle.c, which matches this bit for bit.
// The fp32 pixel path (16U / 32F frames, the other depths
// cv::cuda::SparsePyrLKOpticalFlow takes, cudaoptflow/src/pyrlk.cpp:189-205) is
// the same code on fp32 storage (template F32): levels and derivative pairs are
// kept in fp32 instead of being rounded to fp16.
// Layout and work split follow klt_lk_multi.hip: lane = window column, P = 64 / WW
// points per wave (lane 0 idle), all levels in one launch; the per-point column
// sums go through LDS and are added by one lane per value in column order.
#include "lk_device.hpp"

namespace tbdk {

namespace {

using namespace lkdev;

typedef _Float16 half_t;

__device__ __forceinline__ float h_lo(uint32_t v) { return (float)__builtin_bit_cast(half_t, (uint16_t)(v & 0xFFFFu)); }
__device__ __forceinline__ float h_hi(uint32_t v) { return (float)__builtin_bit_cast(half_t, (uint16_t)(v >> 16)); }
__device__ __forceinline__ float h_at(const uint16_t* p) { return (float)__builtin_bit_cast(half_t, *p); }
__device__ __forceinline__ uint16_t to_h(float f) { return __builtin_bit_cast(uint16_t, (half_t)f); }

__device__ __forceinline__ int reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ void weights16(float a, float b, float& w00, float& w01, float& w10, float& w11)
{
    w00 = (1.f - a) * (1.f - b);
    w01 = a * (1.f - b);
    w10 = (1.f - a) * b;
    w11 = a * b;
}

__device__ __forceinline__ bool any_lane(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// storage of a pixel path: fp16 (2 B per value) or fp32 (4 B per value); a
// "pair" is two consecutive values (I(x), I(x+1)) or a pixel's (Ix, Iy)
template <bool F32>
struct Pix {
    typedef uint32_t pair_t;
    static constexpr int B = 2;
    __device__ static pair_t ld(__amdgpu_buffer_rsrc_t r, uint32_t off, int soff)
    {
        return __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0);
    }
    __device__ static float lo(pair_t p) { return h_lo(p); }
    __device__ static float hi(pair_t p) { return h_hi(p); }
    __device__ static float at(const uint8_t* p) { return h_at(reinterpret_cast<const uint16_t*>(p)); }
};
template <>
struct Pix<true> {
    struct pair_t {
        uint32_t x, y;
    };
    static constexpr int B = 4;
    __device__ static pair_t ld(__amdgpu_buffer_rsrc_t r, uint32_t off, int soff)
    {
        return pair_t{__builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0),
                      __builtin_amdgcn_raw_buffer_load_b32(r, off + 4, soff, 0)};
    }
    __device__ static float lo(pair_t p) { return __builtin_bit_cast(float, p.x); }
    __device__ static float hi(pair_t p) { return __builtin_bit_cast(float, p.y); }
    __device__ static float at(const uint8_t* p) { return *reinterpret_cast<const float*>(p); }
};

// bilinear value of a pair on rows r (p0) and r+1 (p1), started from c:
// fma(w11, p1.hi, fma(w10, p1.lo, fma(w01, p0.hi, fma(w00, p0.lo, c))))
template <bool F32>
__device__ __forceinline__ float bilp(typename Pix<F32>::pair_t p0, typename Pix<F32>::pair_t p1, float w00,
                                      float w01, float w10, float w11, float c)
{
    typedef Pix<F32> P;
    float t = __builtin_fmaf(w00, P::lo(p0), c);
    t = __builtin_fmaf(w01, P::hi(p0), t);
    t = __builtin_fmaf(w10, P::lo(p1), t);
    return __builtin_fmaf(w11, P::hi(p1), t);
}

}  // namespace

// ---- pyramid -----------------------------------------------------------------

// Level 0 of an fp16 pyramid: copy (u8 -> fp16 exactly, or fp16) into the
// padded level with a reflect-101 frame.  One thread writes 4 halves.
__global__ void pad_copy_f16_kernel(const uint8_t* __restrict__ src, int spitch, int src_f16, int w, int h,
                                    uint8_t* __restrict__ dst, int dpitch, int pad, int wp4)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y;
    if (t >= wp4) return;
    const int sy = reflect101(py - pad, h);
    const uint8_t* srow = src + (size_t)sy * spitch;
    uint16_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int sx = reflect101(t * 4 + k - pad, w);
        v[k] = src_f16 ? reinterpret_cast<const uint16_t*>(srow)[sx] : to_h((float)srow[sx]);
    }
    uint2 o;
    o.x = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
    o.y = (uint32_t)v[2] | ((uint32_t)v[3] << 16);
    *reinterpret_cast<uint2*>(dst + (size_t)py * dpitch + (size_t)t * 8) = o;
}

// pyrDown of a padded fp16 level into a padded fp16 level (4 outputs per thread)
__global__ void pyr_down_f16_kernel(const uint8_t* __restrict__ src, int spitch, int spad, uint8_t* __restrict__ dst,
                                    int dpitch, int dpad, int dw, int dh, int wp4)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y;
    if (t >= wp4) return;
    const int ry = reflect101(py - dpad, dh);
    const uint16_t* s0 = reinterpret_cast<const uint16_t*>(src + (size_t)(2 * ry - 2 + spad) * spitch) + spad;
    uint16_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int rx = reflect101(t * 4 + k - dpad, dw);
        float r[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint16_t* q = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(s0) +
                                                                  (size_t)j * spitch) + 2 * rx;
            r[j] = h_at(q) * 6.f + (h_at(q - 1) + h_at(q + 1)) * 4.f + h_at(q - 2) + h_at(q + 2);
        }
        v[k] = to_h((r[2] * 6.f + (r[1] + r[3]) * 4.f + r[0] + r[4]) * (1.f / 256.f));
    }
    uint2 o;
    o.x = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
    o.y = (uint32_t)v[2] | ((uint32_t)v[3] << 16);
    *reinterpret_cast<uint2*>(dst + (size_t)py * dpitch + (size_t)t * 8) = o;
}

struct Scharr16Levels {
    const uint8_t* src[TBDK_MAX_LEVELS];
    uint8_t* dst[TBDK_MAX_LEVELS];
    int w[TBDK_MAX_LEVELS], h[TBDK_MAX_LEVELS], spitch[TBDK_MAX_LEVELS], spad[TBDK_MAX_LEVELS];
    int dpitch[TBDK_MAX_LEVELS], dpad[TBDK_MAX_LEVELS];
};

// calcSharrDeriv's formula in fp32 on every fp16 level, stored as fp16 (Ix, Iy)
__global__ void scharr_f16_levels_kernel(Scharr16Levels a)
{
    const int lvl = blockIdx.z;
    const int y = blockIdx.y;
    const int x0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int w = a.w[lvl], h = a.h[lvl];
    if (y >= h || x0 >= w) return;
    const int sp = a.spitch[lvl];
    const uint16_t* r1 = reinterpret_cast<const uint16_t*>(a.src[lvl] + (size_t)(y + a.spad[lvl]) * sp) +
                         a.spad[lvl] + x0;
    const uint16_t* r0 = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(r1) - sp);
    const uint16_t* r2 = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(r1) + sp);
    float t0[6], t1[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int c = k - 1;
        t0[k] = (h_at(r0 + c) + h_at(r2 + c)) * 3.f + h_at(r1 + c) * 10.f;
        t1[k] = h_at(r2 + c) - h_at(r0 + c);
    }
    uint32_t* d = reinterpret_cast<uint32_t*>(a.dst[lvl] + (size_t)(y + a.dpad[lvl]) * a.dpitch[lvl]) + a.dpad[lvl] + x0;
    const int n = w - x0 < 4 ? w - x0 : 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float ix = t0[k + 2] - t0[k];
        const float iy = (t1[k + 2] + t1[k]) * 3.f + t1[k + 1] * 10.f;
        if (k < n) d[k] = (uint32_t)to_h(ix) | ((uint32_t)to_h(iy) << 16);
    }
}

// ---- fp32 pyramid (the fp32 pixel path) ----------------------------------------

// level 0: a u8 / u16 / fp32 frame (src_kind 0 / 1 / 2) converted exactly into the
// padded fp32 level, reflect-101 frame; 4 values per thread
__global__ void pad_copy_f32_kernel(const uint8_t* __restrict__ src, int spitch, int src_kind, int w, int h,
                                    uint8_t* __restrict__ dst, int dpitch, int pad, int wp4)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y;
    if (t >= wp4) return;
    const uint8_t* srow = src + (size_t)reflect101(py - pad, h) * spitch;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int sx = reflect101(t * 4 + k - pad, w);
        v[k] = src_kind == 2 ? reinterpret_cast<const float*>(srow)[sx]
                             : src_kind == 1 ? (float)reinterpret_cast<const uint16_t*>(srow)[sx] : (float)srow[sx];
    }
    *reinterpret_cast<float4*>(dst + (size_t)py * dpitch + (size_t)t * 16) = make_float4(v[0], v[1], v[2], v[3]);
}

__global__ void pyr_down_f32_kernel(const uint8_t* __restrict__ src, int spitch, int spad, uint8_t* __restrict__ dst,
                                    int dpitch, int dpad, int dw, int dh, int wp4)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y;
    if (t >= wp4) return;
    const int ry = reflect101(py - dpad, dh);
    const float* s0 = reinterpret_cast<const float*>(src + (size_t)(2 * ry - 2 + spad) * spitch) + spad;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int rx = reflect101(t * 4 + k - dpad, dw);
        float r[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const float* q = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(s0) +
                                                            (size_t)j * spitch) + 2 * rx;
            r[j] = q[0] * 6.f + (q[-1] + q[1]) * 4.f + q[-2] + q[2];
        }
        v[k] = (r[2] * 6.f + (r[1] + r[3]) * 4.f + r[0] + r[4]) * (1.f / 256.f);
    }
    *reinterpret_cast<float4*>(dst + (size_t)py * dpitch + (size_t)t * 16) = make_float4(v[0], v[1], v[2], v[3]);
}

// calcSharrDeriv's formula in fp32 on every fp32 level, stored as fp32 (Ix, Iy)
__global__ void scharr_f32_levels_kernel(Scharr16Levels a)
{
    const int lvl = blockIdx.z;
    const int y = blockIdx.y;
    const int x0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int w = a.w[lvl], h = a.h[lvl];
    if (y >= h || x0 >= w) return;
    const int sp = a.spitch[lvl];
    const float* r1 = reinterpret_cast<const float*>(a.src[lvl] + (size_t)(y + a.spad[lvl]) * sp) + a.spad[lvl] + x0;
    const float* r0 = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(r1) - sp);
    const float* r2 = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(r1) + sp);
    float t0[6], t1[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int c = k - 1;
        t0[k] = (r0[c] + r2[c]) * 3.f + r1[c] * 10.f;
        t1[k] = r2[c] - r0[c];
    }
    float2* d = reinterpret_cast<float2*>(a.dst[lvl] + (size_t)(y + a.dpad[lvl]) * a.dpitch[lvl]) + a.dpad[lvl] + x0;
    const int n = w - x0 < 4 ? w - x0 : 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float ix = t0[k + 2] - t0[k];
        const float iy = (t1[k + 2] + t1[k]) * 3.f + t1[k + 1] * 10.f;
        if (k < n) d[k] = make_float2(ix, iy);
    }
}

hipError_t launch_pyr_build_f32(const uint8_t* img, int pitch, int src_kind, const tbdk_pyr& pyr, hipStream_t s)
{
    {
        const tbdk_level& d = pyr.lv[0];
        const int wp4 = (d.width + 2 * d.pad + 3) / 4, hp = d.height + 2 * d.pad;
        hipLaunchKernelGGL(pad_copy_f32_kernel, dim3((wp4 + 255) / 256, hp), dim3(256), 0, s, img, pitch, src_kind,
                           d.width, d.height, d.data, d.pitch, d.pad, wp4);
    }
    for (int l = 1; l < pyr.nlevels; ++l) {
        const tbdk_level &sl = pyr.lv[l - 1], &dl = pyr.lv[l];
        const int wp4 = (dl.width + 2 * dl.pad + 3) / 4, hp = dl.height + 2 * dl.pad;
        hipLaunchKernelGGL(pyr_down_f32_kernel, dim3((wp4 + 255) / 256, hp), dim3(256), 0, s, sl.data, sl.pitch,
                           sl.pad, dl.data, dl.pitch, dl.pad, dl.width, dl.height, wp4);
    }
    Scharr16Levels a;
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
    hipLaunchKernelGGL(scharr_f32_levels_kernel, dim3(((maxw + 3) / 4 + 255) / 256, maxh, pyr.nlevels), dim3(256), 0,
                       s, a);
    return hipGetLastError();
}

hipError_t launch_pyr_build_f16(const uint8_t* img, int pitch, int img_f16, const tbdk_pyr& pyr, hipStream_t s)
{
    {
        const tbdk_level& d = pyr.lv[0];
        const int wp4 = (d.width + 2 * d.pad + 3) / 4, hp = d.height + 2 * d.pad;
        hipLaunchKernelGGL(pad_copy_f16_kernel, dim3((wp4 + 255) / 256, hp), dim3(256), 0, s, img, pitch, img_f16,
                           d.width, d.height, d.data, d.pitch, d.pad, wp4);
    }
    for (int l = 1; l < pyr.nlevels; ++l) {
        const tbdk_level &sl = pyr.lv[l - 1], &dl = pyr.lv[l];
        const int wp4 = (dl.width + 2 * dl.pad + 3) / 4, hp = dl.height + 2 * dl.pad;
        hipLaunchKernelGGL(pyr_down_f16_kernel, dim3((wp4 + 255) / 256, hp), dim3(256), 0, s, sl.data, sl.pitch,
                           sl.pad, dl.data, dl.pitch, dl.pad, dl.width, dl.height, wp4);
    }
    Scharr16Levels a;
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
    hipLaunchKernelGGL(scharr_f16_levels_kernel, dim3(((maxw + 3) / 4 + 255) / 256, maxh, pyr.nlevels), dim3(256), 0,
                       s, a);
    return hipGetLastError();
}

// ---- sparse LK on fp16 levels ------------------------------------------------

// fp16 instances up to the 21x21 window: at most 128 VGPRs, so 4 waves per
// SIMD (the compiler's own choice was 129, i.e. 3); the fp32 instances keep
// the compiler's allocation (capping them spills)
#ifndef TBDK_LK16_MINW
#define TBDK_LK16_MINW 4
#endif
template <int WW, int WH, bool F32>
__global__ __launch_bounds__(64, (!F32 && WW <= 21) ? TBDK_LK16_MINW : 1) void lk_f16_kernel(LkArgs a)
{
    typedef Pix<F32> PX;
    typedef typename PX::pair_t pair_t;
    constexpr int VB = PX::B, DB = 2 * PX::B;  // bytes per value / per derivative pair
    constexpr int P = 64 / WW;  // points per wave
    __shared__ float red[3][64];
    const int lane = threadIdx.x;
    const int k = lane == 0 ? P : (lane - 1) / WW;  // lane 0 (and lanes past the last point) idle
    const int x = k < P ? lane - 1 - k * WW : 0;
    const int base = k < P ? 1 + k * WW : 1;         // first lane of the point
    const int wave = xcd_swizzle(blockIdx.x, gridDim.x);
    const int i = k < P ? seg_point(a, wave * P + k) : -1;
    const bool valid = i >= 0;
    if (!any_lane(valid)) return;  // wave-uniform
    const int vsel = x < 3 ? x : 2;  // value summed by this lane (lanes x = 0, 1, 2 of a point)

    // column sums of up to three per-lane values: lane base + v adds value v's
    // WW column partials left to right; every lane gets its point's totals
    auto colsum3 = [&](float p0, float p1, float p2, float& s0, float& s1, float& s2) {
        red[0][lane] = p0;
        red[1][lane] = p1;
        red[2][lane] = p2;
        __syncthreads();
        const float* q = &red[vsel][base];
        float s = q[0];
#pragma unroll
        for (int j = 1; j < WW; ++j) s += q[j];
        __syncthreads();
        s0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * base, __builtin_bit_cast(int, s)));
        s1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * (base + 1), __builtin_bit_cast(int, s)));
        s2 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * (base + 2), __builtin_bit_cast(int, s)));
    };
    auto colsum2 = [&](float p0, float p1, float& s0, float& s1) {
        red[0][lane] = p0;
        red[1][lane] = p1;
        __syncthreads();
        const float* q = &red[x < 2 ? x : 1][base];
        float s = q[0];
#pragma unroll
        for (int j = 1; j < WW; ++j) s += q[j];
        __syncthreads();
        s0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * base, __builtin_bit_cast(int, s)));
        s1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * (base + 1), __builtin_bit_cast(int, s)));
    };

    const float FLT_SCALE = 1.f / (1 << 20);
    const float halfx = (WW - 1) * 0.5f, halfy = (WH - 1) * 0.5f;
    const float p0x = valid ? a.prev_pts[2 * i] : 0.f, p0y = valid ? a.prev_pts[2 * i + 1] : 0.f;
    float outx = 0.f, outy = 0.f;
    if ((a.flags & TBDK_OPTFLOW_USE_INITIAL_FLOW) && valid) {
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
        bool act = valid;
        if (ipx < -WW || ipx >= L.w || ipy < -WH || ipy >= L.h) {
            if (level == 0) {
                status = 0;
                errv = 0.f;
            }
            act = false;
        }
        if (!any_lane(act)) continue;
        float w00, w01, w10, w11;
        weights16(prevx - ipx, prevy - ipy, w00, w01, w10, w11);

        const int hp = L.h + 2 * L.ipad;
        const __amdgpu_buffer_rsrc_t rI = make_rsrc(L.I, L.ipitch * hp + 256);
        const __amdgpu_buffer_rsrc_t rD = make_rsrc(L.D, L.dpitch * (L.h + 2 * L.dpad) + 256);
        const __amdgpu_buffer_rsrc_t rJ = make_rsrc(L.J, L.jpitch * (L.h + 2 * L.jpad) + 256);

        nextx -= halfx;
        nexty -= halfy;
        int pinx = (int)floorf(nextx), piny = (int)floorf(nexty);
        pair_t jp[WH + 1];

        float iv[WH], gx[WH], gy[WH];
        float A11, A12, A22;
        {
            const uint32_t ioff = act ? (uint32_t)((ipy + L.ipad) * L.ipitch + (ipx + x + L.ipad) * VB) : 0u;
            const uint32_t doff = act ? (uint32_t)((ipy + L.dpad) * L.dpitch + (ipx + x + L.dpad) * DB) : 0u;
            pair_t ip[WH + 1], d0[WH + 1], d1[WH + 1];
#pragma unroll
            for (int r = 0; r <= WH; ++r) {
                ip[r] = PX::ld(rI, ioff, r * L.ipitch);         // (I(x), I(x+1))
                d0[r] = PX::ld(rD, doff, r * L.dpitch);         // (Ix, Iy)(x)
                d1[r] = PX::ld(rD, doff + DB, r * L.dpitch);    // (Ix, Iy)(x+1)
            }
            float a11 = 0.f, a12 = 0.f, a22 = 0.f;
#pragma unroll
            for (int r = 0; r < WH; ++r) {
                iv[r] = bilp<F32>(ip[r], ip[r + 1], w00, w01, w10, w11, 0.f);
                float t = __builtin_fmaf(w00, PX::lo(d0[r]), 0.f);
                t = __builtin_fmaf(w01, PX::lo(d1[r]), t);
                t = __builtin_fmaf(w10, PX::lo(d0[r + 1]), t);
                gx[r] = __builtin_fmaf(w11, PX::lo(d1[r + 1]), t);
                t = __builtin_fmaf(w00, PX::hi(d0[r]), 0.f);
                t = __builtin_fmaf(w01, PX::hi(d1[r]), t);
                t = __builtin_fmaf(w10, PX::hi(d0[r + 1]), t);
                gy[r] = __builtin_fmaf(w11, PX::hi(d1[r + 1]), t);
                a11 = __builtin_fmaf(gx[r], gx[r], a11);
                a12 = __builtin_fmaf(gx[r], gy[r], a12);
                a22 = __builtin_fmaf(gy[r], gy[r], a22);
            }
            {
                const bool jin = act && !(pinx < -WW || pinx >= L.w || piny < -WH || piny >= L.h);
                const uint32_t joff = jin ? (uint32_t)((piny + L.jpad) * L.jpitch + (pinx + x + L.jpad) * VB) : 0u;
#pragma unroll
                for (int r = 0; r <= WH; ++r) jp[r] = PX::ld(rJ, joff, r * L.jpitch);
            }
            if (k >= P) a11 = a12 = a22 = 0.f;
            colsum3(a11, a12, a22, A11, A12, A22);
            A11 *= FLT_SCALE;
            A12 *= FLT_SCALE;
            A22 *= FLT_SCALE;
        }
        float D = A11 * A22 - A12 * A12;
        const float minEig =
            (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * WW * WH);
        if (act && (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS)) errv = minEig;
        if (act && (minEig < a.min_eig || D < 1.19209290e-07F /*FLT_EPSILON*/)) {
            if (level == 0) status = 0;
            act = false;
        }
        D = 1.f / D;

        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < a.max_count; ++j) {
            if (!any_lane(act)) break;
            const int inx = (int)floorf(nextx), iny = (int)floorf(nexty);
            if (act && (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h)) {
                if (level == 0) status = 0;
                act = false;
            }
            nit += act ? 1 : 0;
            const bool moved = act && (inx != pinx || iny != piny);
            if (any_lane(moved)) {
                const uint32_t joff = act ? (uint32_t)((iny + L.jpad) * L.jpitch + (inx + x + L.jpad) * VB) : 0u;
#pragma unroll
                for (int r = 0; r <= WH; ++r) jp[r] = PX::ld(rJ, joff, r * L.jpitch);
                pinx = inx;
                piny = iny;
            }
            weights16(nextx - inx, nexty - iny, w00, w01, w10, w11);
            float b1 = 0.f, b2 = 0.f;
#pragma unroll
            for (int r = 0; r < WH; ++r) {
                const float d = bilp<F32>(jp[r], jp[r + 1], w00, w01, w10, w11, -iv[r]);  // J - I at the window pixel
                b1 = __builtin_fmaf(d, gx[r], b1);
                b2 = __builtin_fmaf(d, gy[r], b2);
            }
            if (k >= P) b1 = b2 = 0.f;
            float fb1, fb2;
            colsum2(b1, b2, fb1, fb2);
            fb1 *= 32.f * FLT_SCALE;  // the CPU path's x32 patch scale, exact
            fb2 *= 32.f * FLT_SCALE;
            const float ddx = (A12 * fb2 - A22 * fb1) * D;
            const float ddy = (A12 * fb1 - A11 * fb2) * D;
            if (act) {
                nextx += ddx;
                nexty += ddy;
                outx = nextx + halfx;
                outy = nexty + halfy;
                if ((double)ddx * ddx + (double)ddy * ddy <= a.eps2) {
                    act = false;
                } else if (j > 0 && (double)fabsf(ddx + pdx) < 0.01 && (double)fabsf(ddy + pdy) < 0.01) {
                    outx -= ddx * 0.5f;
                    outy -= ddy * 0.5f;
                    act = false;
                }
                pdx = ddx;
                pdy = ddy;
            }
        }

        if (level == 0 && a.err && (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS) == 0) {
            bool want = valid && status;
            const float npx = outx - halfx, npy = outy - halfy;
            const int inx = (int)floorf(npx), iny = (int)floorf(npy);
            if (want && (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h)) {
                status = 0;
                want = false;
            }
            if (any_lane(want)) {
                weights16(npx - inx, npy - iny, w00, w01, w10, w11);
                const uint32_t joff = want ? (uint32_t)((iny + L.jpad) * L.jpitch + (inx + x + L.jpad) * VB) : 0u;
#pragma unroll
                for (int r = 0; r <= WH; ++r) jp[r] = PX::ld(rJ, joff, r * L.jpitch);
                float e = 0.f;
#pragma unroll
                for (int r = 0; r < WH; ++r) e += fabsf(bilp<F32>(jp[r], jp[r + 1], w00, w01, w10, w11, -iv[r]));
                if (k >= P) e = 0.f;
                float es, unused;
                colsum2(e, 0.f, es, unused);
                if (want) errv = (es * 32.f) * (1.f / (float)(32 * WW * WH));
            }
        }
    }

    if (valid && x == 0) {
        a.next_pts[2 * i] = outx;
        a.next_pts[2 * i + 1] = outy;
        a.status[i] = (uint8_t)status;
        if (a.err) a.err[i] = errv;
        if (a.iters) a.iters[i] = nit;
    }
}

#define TBDK_F16_WINDOWS(X) X(7) X(9) X(11) X(13) X(15) X(17) X(19) X(21) X(23) X(25) X(27) X(29) X(31)

bool lk_f16_supported(int win_w, int win_h)
{
    if (win_w != win_h) return false;
    switch (win_w) {
#define TBDK_CASE(W) case W:
        TBDK_F16_WINDOWS(TBDK_CASE)
#undef TBDK_CASE
        return true;
    default:
        return false;
    }
}

hipError_t launch_lk_f16(const LkArgs& a, bool f32, hipStream_t s)
{
    if (!lk_f16_supported(a.win_w, a.win_h)) return hipErrorNotSupported;
    const int per_wg = 64 / a.win_w;
    const dim3 grid((a.n + per_wg - 1) / per_wg), block(64);
    switch (a.win_w) {
#define TBDK_CASE(W)                                                                  \
    case W:                                                                           \
        if (f32) hipLaunchKernelGGL((lk_f16_kernel<W, W, true>), grid, block, 0, s, a); \
        else hipLaunchKernelGGL((lk_f16_kernel<W, W, false>), grid, block, 0, s, a);   \
        break;
        TBDK_F16_WINDOWS(TBDK_CASE)
#undef TBDK_CASE
    default:
        return hipErrorNotSupported;
    }
    return hipGetLastError();
}

}  // namespace tbdk
