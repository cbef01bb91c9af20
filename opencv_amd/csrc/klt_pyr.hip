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
    const int x0 = t * 4 - dpad;
    if (x0 >= 0 && x0 + 3 < dw && ((spitch | spad) & 3) == 0) {
        // four consecutive in-level pixels: source columns 2x0-2 .. 2x0+8 of each
        // of the 5 rows (inside the source's frame) as dword loads
        const int c0 = 2 * x0 - 2 + spad, base = c0 & ~3, o = c0 - base;  // o in {0, 2}
        const uint8_t* r0 = src + (size_t)(2 * ry - 2 + spad) * spitch + base;
        int h[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(r0 + (size_t)j * spitch);
            const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
            const uint32_t a0 = __builtin_amdgcn_alignbyte(w1, w0, o), a1 = __builtin_amdgcn_alignbyte(w2, w1, o),
                           a2 = __builtin_amdgcn_alignbyte(w3, w2, o);
            int px[11];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                px[k] = (int)((a0 >> (8 * k)) & 255u);
                px[4 + k] = (int)((a1 >> (8 * k)) & 255u);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) px[8 + k] = (int)((a2 >> (8 * k)) & 255u);
            const int kj = j == 2 ? 6 : (j == 1 || j == 3) ? 4 : 1;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                h[k] += kj * (px[2 * k + 2] * 6 + (px[2 * k + 1] + px[2 * k + 3]) * 4 + px[2 * k] + px[2 * k + 4]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) v |= (uint32_t)((h[k] + 128) >> 8) << (8 * k);
        *reinterpret_cast<uint32_t*>(dst + (size_t)py * dpitch + t * 4) = v;
        return;
    }
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

// ---- fused build: the padded copy of the frame (level 0) and level 1 in ONE
// launch.  Two roles share the grid, each reading only the frame (so neither
// waits for the other): role A copies the frame into its padded buffer (4
// bytes per thread), role B computes level 1 from the frame (4 pixels per
// thread).  A padded pixel is the value at its reflect-101 coordinate, and
// pyrDown_ reads its source through borderInterpolate (pyramids.cpp:795-800),
// so a level-1 pixel is a function of the frame alone:
//   L1(y, x) = (sum_ab k_a k_b F(r0(2y + a - 2), r0(2x + b - 2)) + 128) >> 8
// with r0 the frame's reflection; pixels whose taps need none take dword loads
// of the 5 x 11 patch of four pixels.  The levels below 1 are pyrDown launches
// of the padded level above (their sources are small and L2-resident).
// (A single launch computing level 2 from the frame too was measured slower:
// the pixels near an edge need 625 reflected taps each, and their threads set
// the kernel's length.)
constexpr int kRoleThreads = 256;

struct PyrRolesArgs {
    const uint8_t* src;  // source level, in-image origin
    int spitch, sw, sh;
    int vec;             // src and spitch dword-aligned
    uint8_t* copy;       // padded copy of the source (level 0 of a pyramid), or null: no role A
    int cpitch, cpad;
    uint8_t* d1;         // the level below (padded)
    int p1, pad1, w1, h1;
    int nA;              // blocks of role A (role B: the rest)
    int wa4, wb4;        // items per padded row of roles A (4 or 16 bytes) and B (4 pixels)
    int a16;             // role A copies 16 bytes per thread (source, copy and pitches 16-byte aligned, pad % 16 == 0)
};

__device__ __forceinline__ int pyr5(int a, int b, int c, int d, int e) { return c * 6 + (b + d) * 4 + a + e; }

// level-1 pixel (y, x) (in-image) from the source, every tap reflected (the
// path of pixels near an edge)
__device__ __forceinline__ int pyr_down_at(const PyrRolesArgs& a, int y, int x)
{
    int cx[5], r[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) cx[i] = reflect101(2 * x + i - 2, a.sw);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const uint8_t* q = a.src + (size_t)reflect101(2 * y + j - 2, a.sh) * a.spitch;
        r[j] = pyr5(q[cx[0]], q[cx[1]], q[cx[2]], q[cx[3]], q[cx[4]]);
    }
    return (pyr5(r[0], r[1], r[2], r[3], r[4]) + 128) >> 8;
}

__device__ __forceinline__ int byte_of(uint32_t w, int k) { return (int)((w >> (8 * k)) & 255u); }

__global__ __launch_bounds__(kRoleThreads) void pyr_build_kernel(PyrRolesArgs a)
{
    int b = blockIdx.x;
    const int tid = threadIdx.x;
    if (b < a.nA) {  // ---- role A: the padded copy of the source
        const int item = b * kRoleThreads + tid;
        const int py = item / a.wa4, t = item - py * a.wa4;
        if (py >= a.sh + 2 * a.cpad) return;
        const uint8_t* srow = a.src + (size_t)reflect101(py - a.cpad, a.sh) * a.spitch;
        if (a.a16) {  // 16 bytes per thread: one dwordx4 load and store in the frame's interior
            const int x0 = 16 * t - a.cpad;
            uint4 v;
            if (x0 >= 0 && x0 + 15 < a.sw) {
                v = *reinterpret_cast<const uint4*>(srow + x0);
            } else {
                uint32_t q[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    q[d] = 0;
                    for (int k = 0; k < 4; ++k) q[d] |= (uint32_t)srow[reflect101(x0 + 4 * d + k, a.sw)] << (8 * k);
                }
                v = make_uint4(q[0], q[1], q[2], q[3]);
            }
            *reinterpret_cast<uint4*>(a.copy + (size_t)py * a.cpitch + 16 * t) = v;
            return;
        }
        const int x0 = 4 * t - a.cpad;
        uint32_t v;
        if (a.vec && (x0 & 3) == 0 && x0 >= 0 && x0 + 3 < a.sw) {
            v = *reinterpret_cast<const uint32_t*>(srow + x0);
        } else {
            v = 0;
            for (int k = 0; k < 4; ++k) v |= (uint32_t)srow[reflect101(x0 + k, a.sw)] << (8 * k);
        }
        *reinterpret_cast<uint32_t*>(a.copy + (size_t)py * a.cpitch + 4 * t) = v;
        return;
    }
    b -= a.nA;
    {  // ---- role B: the level below, 4 pixels per thread
        const int item = b * kRoleThreads + tid;
        const int py = item / a.wb4, t = item - py * a.wb4;
        if (py >= a.h1 + 2 * a.pad1) return;
        const int y = reflect101(py - a.pad1, a.h1);
        const int x0 = reflect101(4 * t - a.pad1, a.w1);
        uint32_t v = 0;
        // fast path: four consecutive in-image pixels whose taps need no reflection.
        // x0 even (the pads are multiples of 16) puts the taps' first byte c0 at
        // offset 2 of an aligned dword, so the four aligned dwords read per row end
        // with the dword holding byte c0 + 10 < sw: no byte past the row's last
        // in-image dword is touched (a frame ending at its allocation's last byte
        // with sw % 4 == 0 is safe; sw % 4 != 0 needs a dword pitch, a.vec).
        const bool fast = a.vec && 2 * y - 2 >= 0 && 2 * y + 2 < a.sh && 4 * t - a.pad1 == x0 && 2 * x0 - 2 >= 0 &&
                          2 * x0 + 8 < a.sw && x0 + 3 < a.w1 && (x0 & 1) == 0;
        if (fast) {
            const int c0 = 2 * x0 - 2, base = c0 & ~3, o = 2;  // c0 - base
            int h[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const uint32_t* q = reinterpret_cast<const uint32_t*>(a.src + (size_t)(2 * y + j - 2) * a.spitch + base);
                const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
                // bytes c0 .. c0 + 10 as three dwords
                const uint32_t s0 = __builtin_amdgcn_alignbyte(w1, w0, o), s1 = __builtin_amdgcn_alignbyte(w2, w1, o),
                               s2 = __builtin_amdgcn_alignbyte(w3, w2, o);
                int px[11];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    px[k] = byte_of(s0, k);
                    px[4 + k] = byte_of(s1, k);
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) px[8 + k] = byte_of(s2, k);
                const int kj = j == 2 ? 6 : (j == 1 || j == 3) ? 4 : 1;
#pragma unroll
                for (int k = 0; k < 4; ++k) h[k] += kj * pyr5(px[2 * k], px[2 * k + 1], px[2 * k + 2], px[2 * k + 3],
                                                                px[2 * k + 4]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) v |= (uint32_t)((h[k] + 128) >> 8) << (8 * k);
        } else {
#pragma nounroll
            for (int k = 0; k < 4; ++k)
                v |= (uint32_t)pyr_down_at(a, y, reflect101(4 * t + k - a.pad1, a.w1)) << (8 * k);
        }
        *reinterpret_cast<uint32_t*>(a.d1 + (size_t)py * a.p1 + 4 * t) = v;
        return;
    }
}

// levels 0 and 1 of pyr from the frame in one launch
static hipError_t launch_pyr_fuse01(const uint8_t* src, int spitch, const tbdk_pyr& pyr, hipStream_t s)
{
    PyrRolesArgs a;
    const tbdk_level& S = pyr.lv[0];
    const tbdk_level& D1 = pyr.lv[1];
    a.src = src;
    a.spitch = spitch;
    a.sw = S.width;
    a.sh = S.height;
    a.vec = ((reinterpret_cast<uintptr_t>(src) | (uintptr_t)spitch) & 3) == 0;
    a.copy = S.data;
    a.cpitch = S.pitch;
    a.cpad = S.pad;
    a.d1 = D1.data;
    a.p1 = D1.pitch;
    a.pad1 = D1.pad;
    a.w1 = D1.width;
    a.h1 = D1.height;
    auto blocks = [](long items) { return (int)((items + kRoleThreads - 1) / kRoleThreads); };
    a.a16 = ((reinterpret_cast<uintptr_t>(src) | (uintptr_t)spitch | reinterpret_cast<uintptr_t>(S.data) |
              (uintptr_t)S.pitch | (uintptr_t)S.pad) & 15) == 0 && S.pitch >= ((S.width + 2 * S.pad + 15) & ~15);
    a.wa4 = a.a16 ? (S.width + 2 * S.pad + 15) / 16 : (S.width + 2 * S.pad + 3) / 4;
    a.wb4 = (D1.width + 2 * D1.pad + 3) / 4;
    a.nA = blocks((long)a.wa4 * (S.height + 2 * S.pad));
    const int nB = blocks((long)a.wb4 * (D1.height + 2 * D1.pad));
    hipLaunchKernelGGL(pyr_build_kernel, dim3(a.nA + nB), dim3(kRoleThreads), 0, s, a);
    return hipGetLastError();
}

// every level of a u8 pyramid from the frame: levels 0 and 1 in one launch
// (fuse), or one launch per level
hipError_t launch_pyr_levels(const uint8_t* img, int pitch, const tbdk_pyr& pyr, bool fuse, hipStream_t s)
{
    hipError_t e;
    int level = 1;
    if (fuse && pyr.nlevels >= 2) {
        e = launch_pyr_fuse01(img, pitch, pyr, s);
        level = 2;
    } else {
        e = launch_pad_copy(img, pitch, pyr.lv[0], s);
    }
    for (; e == hipSuccess && level < pyr.nlevels; ++level)
        e = launch_pyr_down_padded(pyr.lv[level - 1], pyr.lv[level], s);
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
