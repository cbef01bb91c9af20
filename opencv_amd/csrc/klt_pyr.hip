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
