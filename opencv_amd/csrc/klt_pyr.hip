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
    int ra, rb;          // rows per thread: role A (16-byte path, 1..kRowsA), role B (1 or 2)
    int nAr, nB;         // blocks of role A (nA - nAr alignment blocks idle) and of role B
    int xcd;             // deal each role's blocks to the XCDs in contiguous row bands (nA % 8 == 0)
};
constexpr int kRowsA = 4;

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

// role B's fast-path horizontal taps: bytes c0 .. c0 + 10 of a row (c0 = 2 mod 4)
// as the [1 4 6 4 1] sums of four level-1 columns
__device__ __forceinline__ void pyr_row_h4(const uint8_t* row, int base, int* hs)
{
    const uint32_t* q = reinterpret_cast<const uint32_t*>(row + base);
    const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
    const uint32_t s0 = __builtin_amdgcn_alignbyte(w1, w0, 2), s1 = __builtin_amdgcn_alignbyte(w2, w1, 2),
                   s2 = __builtin_amdgcn_alignbyte(w3, w2, 2);
    int px[11];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        px[k] = byte_of(s0, k);
        px[4 + k] = byte_of(s1, k);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) px[8 + k] = byte_of(s2, k);
#pragma unroll
    for (int k = 0; k < 4; ++k) hs[k] = pyr5(px[2 * k], px[2 * k + 1], px[2 * k + 2], px[2 * k + 3], px[2 * k + 4]);
}

// role B, one padded level-1 row py, 4 pixels from padded column 4t
__device__ __forceinline__ void pyr_role_b_row(const PyrRolesArgs& a, int py, int t)
{
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
        const int base = (2 * x0 - 2) & ~3;
        int hs[5][4];
#pragma unroll
        for (int j = 0; j < 5; ++j) pyr_row_h4(a.src + (size_t)(2 * y + j - 2) * a.spitch, base, hs[j]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v |= (uint32_t)((pyr5(hs[0][k], hs[1][k], hs[2][k], hs[3][k], hs[4][k]) + 128) >> 8) << (8 * k);
    } else {
#pragma nounroll
        for (int k = 0; k < 4; ++k) v |= (uint32_t)pyr_down_at(a, y, reflect101(4 * t + k - a.pad1, a.w1)) << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(a.d1 + (size_t)py * a.p1 + 4 * t) = v;
}

__global__ __launch_bounds__(kRoleThreads) void pyr_build_kernel(PyrRolesArgs a)
{
    int b = blockIdx.x;
    const int tid = threadIdx.x;
    if (b < a.nA) {  // ---- role A: the padded copy of the source, a.ra rows per thread
        if (b >= a.nAr) return;
        if (a.xcd) b = xcd_swizzle(b, a.nAr);
        const int item = b * kRoleThreads + tid;
        const int pg = item / a.wa4, t = item - pg * a.wa4;
        const int hp = a.sh + 2 * a.cpad;
        if (a.a16) {  // 16 bytes per row: dwordx4 loads (all rows first) and stores in the frame's interior
            const int x0 = 16 * t - a.cpad;
            const int py0 = pg * a.ra;
            if (py0 >= hp) return;
            const int nr = hp - py0 < a.ra ? hp - py0 : a.ra;
            uint4 v[kRowsA];
            if (x0 >= 0 && x0 + 15 < a.sw) {
#pragma unroll
                for (int r = 0; r < kRowsA; ++r)
                    if (r < nr)
                        v[r] = *reinterpret_cast<const uint4*>(
                            a.src + (size_t)reflect101(py0 + r - a.cpad, a.sh) * a.spitch + x0);
            } else {
                // unrolled with constant indices: a runtime index into v[] makes the
                // compiler move v[] to LDS (16 KB per workgroup, each load waited on)
#pragma unroll
                for (int r = 0; r < kRowsA; ++r) {
                    if (r >= nr) break;
                    const uint8_t* srow = a.src + (size_t)reflect101(py0 + r - a.cpad, a.sh) * a.spitch;
                    uint32_t q[4];
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        q[d] = 0;
                        for (int k = 0; k < 4; ++k)
                            q[d] |= (uint32_t)srow[reflect101(x0 + 4 * d + k, a.sw)] << (8 * k);
                    }
                    v[r] = make_uint4(q[0], q[1], q[2], q[3]);
                }
            }
#pragma unroll
            for (int r = 0; r < kRowsA; ++r)
                if (r < nr) *reinterpret_cast<uint4*>(a.copy + (size_t)(py0 + r) * a.cpitch + 16 * t) = v[r];
            return;
        }
        const int py = pg;  // 4 bytes per thread, one row
        if (py >= hp) return;
        const uint8_t* srow = a.src + (size_t)reflect101(py - a.cpad, a.sh) * a.spitch;
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
    if (a.xcd) b = xcd_swizzle(b, a.nB);
    {  // ---- role B: the level below, 4 pixels of a.rb rows per thread
        const int item = b * kRoleThreads + tid;
        const int pg = item / a.wb4, t = item - pg * a.wb4;
        const int hp1 = a.h1 + 2 * a.pad1;
        const int py0 = pg * a.rb;
        if (py0 >= hp1) return;
        if (a.rb == 2) {
            // two in-image rows y, y + 1 share their 7 source rows
            const int y = py0 - a.pad1, x0 = 4 * t - a.pad1;
            if (a.vec && y >= 1 && 2 * y + 4 < a.sh && y + 1 < a.h1 && x0 >= 1 && 2 * x0 + 8 < a.sw &&
                x0 + 3 < a.w1 && (x0 & 1) == 0) {
                const int base = (2 * x0 - 2) & ~3;
                int hs[7][4];
#pragma unroll
                for (int j = 0; j < 7; ++j) pyr_row_h4(a.src + (size_t)(2 * y + j - 2) * a.spitch, base, hs[j]);
                uint32_t v0 = 0, v1 = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v0 |= (uint32_t)((pyr5(hs[0][k], hs[1][k], hs[2][k], hs[3][k], hs[4][k]) + 128) >> 8) << (8 * k);
                    v1 |= (uint32_t)((pyr5(hs[2][k], hs[3][k], hs[4][k], hs[5][k], hs[6][k]) + 128) >> 8) << (8 * k);
                }
                *reinterpret_cast<uint32_t*>(a.d1 + (size_t)py0 * a.p1 + 4 * t) = v0;
                *reinterpret_cast<uint32_t*>(a.d1 + (size_t)(py0 + 1) * a.p1 + 4 * t) = v1;
                return;
            }
            pyr_role_b_row(a, py0, t);
            if (py0 + 1 < hp1) pyr_role_b_row(a, py0 + 1, t);
            return;
        }
        pyr_role_b_row(a, py0, t);
    }
}

// levels 0 and 1 of pyr from the frame in one launch
static hipError_t launch_pyr_fuse01(const uint8_t* src, int spitch, const tbdk_pyr& pyr, hipStream_t s, int rows_a,
                                    int rows_b, int xcd, bool skip_l0)
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
    a.ra = a.a16 ? rows_a : 1;
    a.rb = rows_b;
    a.nAr = blocks((long)a.wa4 * ((S.height + 2 * S.pad + a.ra - 1) / a.ra));
    a.nA = xcd ? (a.nAr + 7) & ~7 : a.nAr;
    if (skip_l0) a.nA = a.nAr = 0;  // level 0 is the frame itself: role B only
    a.nB = blocks((long)a.wb4 * ((D1.height + 2 * D1.pad + a.rb - 1) / a.rb));
    a.xcd = xcd;
    hipLaunchKernelGGL(pyr_build_kernel, dim3(a.nA + a.nB), dim3(kRoleThreads), 0, s, a);
    return hipGetLastError();
}

// ---- levels 0, 1 and 2 in one launch (pyr_fuse 2, opt-in for A/B runs) -------
//
// One workgroup per tile of TX x TY level-2 pixels (level 1: 2TX x 2TY, the
// frame: 4TX x 4TY), every byte of the frame read once into LDS (16-byte loads
// of the tile plus its halo, rows and columns reflect-101 at the frame's edges),
// then from LDS:
//   level 0: the tile's frame pixels written as the padded copy (16-byte stores);
//   level 1: pyrDown_ over the tile plus a 2-pixel halo, separably (the
//            horizontal [1 4 6 4 1] sums of the halo rows at the level-1 columns
//            into LDS as int16, then the vertical taps and (s + 128) >> 8 -- the
//            same integers as the 5x5 sum), halo entries outside the level at
//            their reflect-101 coordinate (the reference makes level 2 from the
//            isolated level 1 with BORDER_REFLECT_101, pyramids.cpp:795-800);
//   level 2: pyrDown_ of the level-1 values in LDS.
// The reflect-101 frame of each level: a pixel at distance 1..pad from an edge
// is also stored at its mirror position outside the level (for rows, columns
// and both), so every padded byte is written by the workgroup that owns its
// source pixel (requires pad <= size - 2 on every level built here; other
// pyramids take the two-role path).
constexpr int kFusedThreads = 256;
#ifndef TBDK_PYR_FUSED_STOP  // timing probes only: return after this phase (wrong results)
#define TBDK_PYR_FUSED_STOP 99
#endif

struct PyrFusedArgs {
    const uint8_t* src;
    int spitch, w0, h0;
    int vec16;                 // src and spitch 16-byte aligned
    uint8_t* d[3];             // level data (padded origin)
    int pitch[3], pad[3], w[3], h[3];
    int nlv;                   // levels written here: 2 or 3
    int tiles_x, ntiles;
};

// store one byte of level L at in-level (y, x) and at every mirror position of
// the level's reflect-101 frame
__device__ __forceinline__ void fused_put_mirrors(const PyrFusedArgs& a, int L, int y, int x, uint8_t v,
                                                  bool skip_self)
{
    const int p = a.pad[L], w = a.w[L], h = a.h[L];
    int ys[3], nys = 0, xs[3], nxs = 0;
    ys[nys++] = y;
    if (y >= 1 && y <= p) ys[nys++] = -y;
    if (y >= h - 1 - p && y <= h - 2) ys[nys++] = 2 * (h - 1) - y;
    xs[nxs++] = x;
    if (x >= 1 && x <= p) xs[nxs++] = -x;
    if (x >= w - 1 - p && x <= w - 2) xs[nxs++] = 2 * (w - 1) - x;
    uint8_t* base = a.d[L] + (size_t)p * a.pitch[L] + p;
    for (int i = 0; i < nys; ++i)
        for (int j = 0; j < nxs; ++j)
            if (!(skip_self && j == 0)) base[(ptrdiff_t)ys[i] * a.pitch[L] + xs[j]] = v;
}

// the row mirrors of a 16-byte chunk of level L at in-level (y, x0 .. x0+15),
// plus the column mirrors of its bytes (x0 multiple of 16; n valid bytes)
__device__ __forceinline__ void fused_put_chunk(const PyrFusedArgs& a, int L, int y, int x0, uint4 v, int n)
{
    const int p = a.pad[L], w = a.w[L], h = a.h[L];
    uint8_t* base = a.d[L] + (size_t)p * a.pitch[L] + p;
    int ys[3], nys = 0;
    ys[nys++] = y;
    if (y >= 1 && y <= p) ys[nys++] = -y;
    if (y >= h - 1 - p && y <= h - 2) ys[nys++] = 2 * (h - 1) - y;
    const bool aligned = ((p & 15) == 0) && n == 16;
    for (int i = 0; i < nys; ++i) {
        uint8_t* row = base + (ptrdiff_t)ys[i] * a.pitch[L];
        if (aligned) {
            *reinterpret_cast<uint4*>(row + x0) = v;
        } else {
            const uint32_t q[4] = {v.x, v.y, v.z, v.w};
            for (int k = 0; k < n; ++k) row[x0 + k] = (uint8_t)(q[k >> 2] >> (8 * (k & 3)));
        }
    }
    // column mirrors: only chunks that touch the first / last pad + 1 columns
    if (x0 <= p || x0 + n - 1 >= w - 1 - p) {
        const uint32_t q[4] = {v.x, v.y, v.z, v.w};
        for (int k = 0; k < n; ++k) {
            const int x = x0 + k;
            if ((x >= 1 && x <= p) || (x >= w - 1 - p && x <= w - 2))
                fused_put_mirrors(a, L, y, x, (uint8_t)(q[k >> 2] >> (8 * (k & 3))), true);
        }
    }
}

__device__ __forceinline__ int pyr_w5(int a, int b, int c, int d, int e) { return c * 6 + (b + d) * 4 + a + e; }

__device__ __forceinline__ int byte_at(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e, int k)
{
    const uint32_t w = k < 4 ? a : k < 8 ? b : k < 12 ? c : k < 16 ? d : e;
    return (int)((w >> (8 * (k & 3))) & 255u);
}

// four horizontal pyrDown_ sums from the 11 bytes starting at byte `o` (0..7)
// of the 20 LDS bytes at p (8-byte aligned): outputs k = 0..3 use bytes
// o + 2k .. o + 2k + 4
__device__ __forceinline__ void hsum4(const uint8_t* p, int o, int (&h)[4])
{
    const uint2 a = *reinterpret_cast<const uint2*>(p);
    const uint2 b = *reinterpret_cast<const uint2*>(p + 8);
    const uint32_t c = *reinterpret_cast<const uint32_t*>(p + 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int v[5];
#pragma unroll
        for (int t = 0; t < 5; ++t) v[t] = byte_at(a.x, a.y, b.x, b.y, c, o + 2 * k + t);
        h[k] = pyr_w5(v[0], v[1], v[2], v[3], v[4]);
    }
}

template <int TX, int TY>
__global__ __launch_bounds__(kFusedThreads) void pyr_fused_kernel(PyrFusedArgs a)
{
    // frame window: rows [4Y - 6, 4Y + 4TY + 3), columns [4X - 16, 4X + 4TX + 16)
    constexpr int FH = 4 * TY + 9, FW = 4 * TX + 32;
    // level-1 window: rows [2Y - 2, 2Y + 2TY + 1) (NY1), columns in GX1 groups of
    // four from 2X - 4 (covers [2X - 2, 2X + 2TX]); stored with level-1 column l
    // at LDS column l - (2X - 16), so the tile's own columns start 16-aligned
    constexpr int NY1 = 2 * TY + 3, GX1 = TX / 2 + 2, HW = 4 * GX1, L1W = 2 * TX + 32;
    __shared__ __attribute__((aligned(16))) uint8_t sF[FH * FW];   // the frame window; then the level-2 row sums
    __shared__ __attribute__((aligned(16))) int16_t sH[FH * HW];   // horizontal level-1 sums
    __shared__ __attribute__((aligned(16))) uint8_t sL1[NY1 * L1W];
    int16_t* const sH2 = reinterpret_cast<int16_t*>(sF);             // [NY1][TX], after sF's last use
    static_assert(NY1 * TX * 2 <= FH * FW, "level-2 sums alias the frame window");

    const int tid = threadIdx.x;
    const int t = xcd_swizzle(blockIdx.x, gridDim.x);  // neighbouring tiles on one XCD (halo rows in its L2)
    const int TXi = t % a.tiles_x, TYi = t / a.tiles_x;
    const int X = TXi * TX, Y = TYi * TY;              // level-2 tile origin
    const int F0x = 4 * X - 16, F0y = 4 * Y - 6;
    const int w1 = a.w[1], h1 = a.h[1];

    // ---- 1. the frame window into LDS (rows and columns reflect-101 at the frame's edges)
    for (int i = tid; i < FH * (FW / 16); i += kFusedThreads) {
        const int r = i / (FW / 16), c = i - r * (FW / 16);
        const int gy = reflect101(F0y + r, a.h0), gx = F0x + 16 * c;
        const uint8_t* srow = a.src + (size_t)gy * a.spitch;
        uint4 v;
        if (a.vec16 && gx >= 0 && gx + 15 < a.w0) {
            v = *reinterpret_cast<const uint4*>(srow + gx);
        } else {
            uint32_t q[4];
#pragma unroll
            for (int dd = 0; dd < 4; ++dd) {
                q[dd] = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) q[dd] |= (uint32_t)srow[reflect101(gx + 4 * dd + k, a.w0)] << (8 * k);
            }
            v = make_uint4(q[0], q[1], q[2], q[3]);
        }
        *reinterpret_cast<uint4*>(sF + r * FW + 16 * c) = v;
    }
    __syncthreads();

    if (TBDK_PYR_FUSED_STOP <= 1) return;
    // ---- 2. level 0: the tile's frame pixels (window rows 6 .., columns 16 ..)
    for (int i = tid; i < 4 * TY * (TX / 4); i += kFusedThreads) {
        const int r = i / (TX / 4), c = i - r * (TX / 4);
        const int y = 4 * Y + r, x = 4 * X + 16 * c;
        if (y >= a.h0 || x >= a.w0) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(sF + (r + 6) * FW + 16 + 16 * c);
        fused_put_chunk(a, 0, y, x, v, min(16, a.w0 - x));
    }
    if (TBDK_PYR_FUSED_STOP <= 2) return;
    // ---- 3. horizontal level-1 sums of every window row, four level-1 columns
    //      l0 .. l0+3 (l0 = 2X - 4 + 4g) per item, each at its reflect-101 column
    for (int i = tid; i < FH * GX1; i += kFusedThreads) {
        const int r = i / GX1, g = i - r * GX1;
        const int l0 = 2 * X - 4 + 4 * g;
        const uint8_t* row = sF + r * FW;
        int h[4];
        if (l0 >= 0 && l0 + 3 < w1) {
            hsum4(row + 8 * g, 6, h);  // frame columns 2 l0 - 2 .. 2 l0 + 8 = window bytes 8g + 6 ..
        } else {
            // columns past w1 + 1 feed no level-2 pixel: clamped so their reflection stays in the window
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint8_t* q = row + (2 * reflect101(min(l0 + k, w1 + 1), w1) - 2 - F0x);
                h[k] = pyr_w5(q[0], q[1], q[2], q[3], q[4]);
            }
        }
        uint2 o;
        o.x = (uint32_t)(uint16_t)h[0] | ((uint32_t)(uint16_t)h[1] << 16);
        o.y = (uint32_t)(uint16_t)h[2] | ((uint32_t)(uint16_t)h[3] << 16);
        *reinterpret_cast<uint2*>(sH + r * HW + 4 * g) = o;
    }
    __syncthreads();
    if (TBDK_PYR_FUSED_STOP <= 3) return;
    // ---- 4. level-1 window values, rows at their reflect-101 rows
    for (int i = tid; i < NY1 * GX1; i += kFusedThreads) {
        const int r = i / GX1, g = i - r * GX1;
        const int ry = reflect101(min(2 * Y - 2 + r, h1 + 1), h1);
        const int16_t* hc = sH + (2 * ry - 2 - F0y) * HW + 4 * g;
        int v[5][4];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint2 q = *reinterpret_cast<const uint2*>(hc + j * HW);
            v[j][0] = (int)(int16_t)(q.x & 0xFFFFu);
            v[j][1] = (int)(int16_t)(q.x >> 16);
            v[j][2] = (int)(int16_t)(q.y & 0xFFFFu);
            v[j][3] = (int)(int16_t)(q.y >> 16);
        }
        uint32_t o = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o |= (uint32_t)((pyr_w5(v[0][k], v[1][k], v[2][k], v[3][k], v[4][k]) + 128) >> 8) << (8 * k);
        *reinterpret_cast<uint32_t*>(sL1 + r * L1W + 12 + 4 * g) = o;
    }
    __syncthreads();
    if (TBDK_PYR_FUSED_STOP <= 4) return;
    // ---- 5. level 1: the tile's pixels (window rows 2 .., LDS columns 16 ..)
    for (int i = tid; i < 2 * TY * (TX / 8); i += kFusedThreads) {
        const int r = i / (TX / 8), c = i - r * (TX / 8);
        const int y = 2 * Y + r, x = 2 * X + 16 * c;
        if (y >= h1 || x >= w1) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(sL1 + (r + 2) * L1W + 16 + 16 * c);
        fused_put_chunk(a, 1, y, x, v, min(16, w1 - x));
    }
    if (a.nlv < 3) return;
    // ---- 6. horizontal level-2 sums of the level-1 window rows, level-2 columns
    //      X + 4q .. X + 4q + 3 (level-1 columns 2X + 8q - 2 .. = LDS bytes 8q + 14 ..)
    for (int i = tid; i < NY1 * (TX / 4); i += kFusedThreads) {
        const int r = i / (TX / 4), q4 = i - r * (TX / 4);
        int h[4];
        hsum4(sL1 + r * L1W + 8 * q4 + 8, 6, h);
        uint2 o;
        o.x = (uint32_t)(uint16_t)h[0] | ((uint32_t)(uint16_t)h[1] << 16);
        o.y = (uint32_t)(uint16_t)h[2] | ((uint32_t)(uint16_t)h[3] << 16);
        *reinterpret_cast<uint2*>(sH2 + r * TX + 4 * q4) = o;
    }
    __syncthreads();
    // ---- 7. level 2: the tile, four pixels per item
    for (int i = tid; i < TY * (TX / 4); i += kFusedThreads) {
        const int r = i / (TX / 4), c = i - r * (TX / 4);
        const int y = Y + r, x = X + 4 * c;
        if (y >= a.h[2] || x >= a.w[2]) continue;
        const int16_t* hc = sH2 + (2 * r) * TX + 4 * c;
        int v[5][4];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint2 q = *reinterpret_cast<const uint2*>(hc + j * TX);
            v[j][0] = (int)(int16_t)(q.x & 0xFFFFu);
            v[j][1] = (int)(int16_t)(q.x >> 16);
            v[j][2] = (int)(int16_t)(q.y & 0xFFFFu);
            v[j][3] = (int)(int16_t)(q.y >> 16);
        }
        uint32_t o = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o |= (uint32_t)((pyr_w5(v[0][k], v[1][k], v[2][k], v[3][k], v[4][k]) + 128) >> 8) << (8 * k);
        const int n = min(4, a.w[2] - x);
        const int p = a.pad[2], w = a.w[2], h = a.h[2];
        uint8_t* base = a.d[2] + (size_t)p * a.pitch[2] + p;
        int ys[3], nys = 0;
        ys[nys++] = y;
        if (y >= 1 && y <= p) ys[nys++] = -y;
        if (y >= h - 1 - p && y <= h - 2) ys[nys++] = 2 * (h - 1) - y;
        for (int j = 0; j < nys; ++j) {
            uint8_t* row = base + (ptrdiff_t)ys[j] * a.pitch[2];
            if (n == 4) *reinterpret_cast<uint32_t*>(row + x) = o;
            else
                for (int k = 0; k < n; ++k) row[x + k] = (uint8_t)(o >> (8 * k));
        }
        if (x <= p || x + n - 1 >= w - 1 - p)
            for (int k = 0; k < n; ++k) {
                const int xx = x + k;
                if ((xx >= 1 && xx <= p) || (xx >= w - 1 - p && xx <= w - 2))
                    fused_put_mirrors(a, 2, y, xx, (uint8_t)(o >> (8 * k)), true);
            }
    }
}

// the fused build applies when the frame window's 16-byte loads and stores
// line up and every level it writes has room for a one-bounce reflect-101 frame
static bool pyr_fused_ok(const tbdk_pyr& pyr)
{
    if (pyr.nlevels < 2 || pyr.cn > 1 || pyr.depth != TBDK_DEPTH_8U) return false;
    const int nlv = pyr.nlevels >= 3 ? 3 : 2;
    for (int l = 0; l < nlv; ++l) {
        const tbdk_level& L = pyr.lv[l];
        if (L.pad > L.width - 2 || L.pad > L.height - 2 || (L.pad & 15) || (L.pitch & 15) ||
            (reinterpret_cast<uintptr_t>(L.data) & 15))
            return false;
    }
    return true;
}

static hipError_t launch_pyr_fused(const uint8_t* src, int spitch, const tbdk_pyr& pyr, hipStream_t s, int* built)
{
    PyrFusedArgs a;
    a.src = src;
    a.spitch = spitch;
    a.w0 = pyr.lv[0].width;
    a.h0 = pyr.lv[0].height;
    a.vec16 = ((reinterpret_cast<uintptr_t>(src) | (uintptr_t)spitch) & 15) == 0;
    a.nlv = pyr.nlevels >= 3 ? 3 : 2;
    for (int l = 0; l < 3; ++l) {
        const tbdk_level& L = pyr.lv[l < a.nlv ? l : a.nlv - 1];
        a.d[l] = L.data;
        a.pitch[l] = L.pitch;
        a.pad[l] = L.pad;
        a.w[l] = L.width;
        a.h[l] = L.height;
    }
    if (a.nlv < 3) {  // level-2 geometry still sizes the tiles
        a.w[2] = (a.w[1] + 1) / 2;
        a.h[2] = (a.h[1] + 1) / 2;
    }
    // big tiles when they alone give the chip ~2 workgroups per CU
    const int w2 = (a.w[1] + 1) / 2, h2 = (a.h[1] + 1) / 2;
    const long big = (long)((w2 + 63) / 64) * ((h2 + 15) / 16);
    if (big >= 480) {
        a.tiles_x = (w2 + 63) / 64;
        a.ntiles = (int)big;
        hipLaunchKernelGGL((pyr_fused_kernel<64, 16>), dim3(a.ntiles), dim3(kFusedThreads), 0, s, a);
    } else {
        a.tiles_x = (w2 + 31) / 32;
        a.ntiles = a.tiles_x * ((h2 + 7) / 8);
        hipLaunchKernelGGL((pyr_fused_kernel<32, 8>), dim3(a.ntiles), dim3(kFusedThreads), 0, s, a);
    }
    *built = a.nlv;
    return hipGetLastError();
}

// every level of a u8 pyramid from the frame: levels 0 and 1 in one launch
// (fuse), or one launch per level
hipError_t launch_pyr_levels(const uint8_t* img, int pitch, const tbdk_pyr& pyr, int fuse, int rows, int xcd,
                             hipStream_t s, bool skip_l0)
{
    hipError_t e;
    int level = 1;
    if (skip_l0) {  // the two-role launch without its copy role (levels >= 2 from level 1 as usual)
        if (pyr.nlevels < 2) return hipSuccess;
        rows = rows < 1 ? 1 : rows > kRowsA ? kRowsA : rows;
        e = launch_pyr_fuse01(img, pitch, pyr, s, rows, rows > 1 ? 2 : 1, xcd, true);
        level = 2;
    } else if (fuse >= 2 && pyr_fused_ok(pyr)) {
        e = launch_pyr_fused(img, pitch, pyr, s, &level);
    } else if (fuse && pyr.nlevels >= 2) {
        rows = rows < 1 ? 1 : rows > kRowsA ? kRowsA : rows;
        e = launch_pyr_fuse01(img, pitch, pyr, s, rows, rows > 1 ? 2 : 1, xcd, false);
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
