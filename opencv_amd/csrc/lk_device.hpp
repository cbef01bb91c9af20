// lk_device.hpp — device helpers shared by the register-resident PyrLK kernels
// (klt_lk_strip.hip, klt_lk_multi.hip): fixed-point bilinear weights and dot
// products in the reference's integer arithmetic (LKTrackerInvoker,
// video/src/lkpyramid.cpp:227-303), buffer loads of packed pixel pairs.
#pragma once
#include "tbdk_internal.hpp"

namespace tbdk {
namespace lkdev {

constexpr int W_BITS = 14, W_BITS1 = 14;

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));  // packed 16-bit VALU ops (v_pk_*_u16)

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ s16x2 as_s16x2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as_u32(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }

__device__ __forceinline__ int sdot2(uint32_t a, uint32_t b, int c)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b), c, false);
}

// bilinear of a packed pixel pair on two rows: (p0 . w0 + p1 . w1 + round) >> shift
// (the reference's _mm_madd_epi16 products and CV_DESCALE, lkpyramid.cpp:288-303)
__device__ __forceinline__ int bilin(uint32_t p0, uint32_t p1, uint32_t w0, uint32_t w1, int shift)
{
    return sdot2(p0, w0, sdot2(p1, w1, 1 << (shift - 1))) >> shift;
}

// the same with the rounding term taken from an SGPR by the three-operand
// v_dot2_i32_i16 (the compiler otherwise materialises it with a v_mov per call
// for the accumulating v_dot2c form)
template <int SHIFT>
__device__ __forceinline__ int bilin_s(uint32_t p0, uint32_t p1, uint32_t w0, uint32_t w1, int round_sgpr)
{
    int t;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(t) : "v"(p1), "v"(w1), "s"(round_sgpr));
    return sdot2(p0, w0, t) >> SHIFT;
}

// iw00..iw11 = cvRound(w * 2^14), iw11 = 2^14 - the others (lkpyramid.cpp:227-234),
// packed as (w00, w01) and (w10, w11) int16 pairs.
// cvRound(p * 2^14) for p = (1-a)(1-b) etc. in [0, 1]: p * 2^14 is exact, so
// fma(p, 2^14, 1.5 * 2^23) rounds p * 2^14 to the nearest integer, ties to even
// (the ulp of the sum is 1), and the integer sits in the low mantissa bits of
// the result (the constant's low 16 bits are zero): no round / convert
// instructions, and each pair is one byte permute.
__device__ __forceinline__ void bilinear_weights(float fa, float fb, uint32_t& w0, uint32_t& w1)
{
    constexpr float kMagic = 12582912.f;  // 1.5 * 2^23
    const float ga = 1.f - fa, gb = 1.f - fb;
    const uint32_t b00 = __float_as_uint(__builtin_fmaf(ga * gb, (float)(1 << W_BITS), kMagic));
    const uint32_t b01 = __float_as_uint(__builtin_fmaf(fa * gb, (float)(1 << W_BITS), kMagic));
    const uint32_t b10 = __float_as_uint(__builtin_fmaf(ga * fb, (float)(1 << W_BITS), kMagic));
    // low 16 bits of 2^14 - w00 - w01 - w10 (the constant's part cancels modulo 2^16)
    const uint32_t b11 = (uint32_t)(1 << W_BITS) - (b00 + b01 + b10);
    w0 = __builtin_amdgcn_perm(b01, b00, 0x05040100u);
    w1 = __builtin_amdgcn_perm(b11, b10, 0x05040100u);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

// (pixel off, pixel off+1) of the 8 bytes at aligned offset, as an int16 pair
__device__ __forceinline__ uint32_t load_pair_u8(__amdgpu_buffer_rsrc_t rs, uint32_t aligned, int soff, uint32_t sel)
{
    const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, aligned, soff, 0);
    const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs, aligned + 4, soff, 0);
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// (pixel off, pixel off+1) as an int16 pair from ONE unaligned dword load
// (gfx950 serves unaligned buffer dword loads; one load and one VGPR per row
// instead of an aligned dword pair)
__device__ __forceinline__ uint32_t load_pair_u8_ua(__amdgpu_buffer_rsrc_t rs, uint32_t off, int soff)
{
    const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rs, off, soff, 0);
    return __builtin_amdgcn_perm(v, v, 0x0C010C00u);
}

// ---- unpadded levels (the TBD loop's level 0 read straight from the frame):
// windows that cross the level's edge take reflect-101 coordinates per byte,
// the values the padded copy (lkpyramid.cpp:726-740) holds there

// reflect-101 of c into [0, n), for -n < c < 2n - 1
__device__ __forceinline__ int refl101(int c, int n)
{
    c = c < 0 ? -c : c;
    return c >= n ? 2 * (n - 1) - c : c;
}

// pixels col .. col + 3 of `row` as one dword (byte k = pixel col + k)
__device__ __forceinline__ uint32_t load4_refl(__amdgpu_buffer_rsrc_t rs, int pitch, int w, int h, int row, int col)
{
    const int yo = refl101(row, h) * pitch;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, (uint32_t)(yo + refl101(col + k, w)), 0, 0) << (8 * k);
    return v;
}

// (pixel col, pixel col + 1) of `row` as an int16 pair, as load_pair_u8_ua
__device__ __forceinline__ uint32_t load_pair_refl(__amdgpu_buffer_rsrc_t rs, int pitch, int w, int h, int row, int col)
{
    const int yo = refl101(row, h) * pitch;
    const uint32_t a = __builtin_amdgcn_raw_buffer_load_b8(rs, (uint32_t)(yo + refl101(col, w)), 0, 0);
    const uint32_t b = __builtin_amdgcn_raw_buffer_load_b8(rs, (uint32_t)(yo + refl101(col + 1, w)), 0, 0);
    return a | (b << 16);
}

// v_perm selector picking bytes (off & 3) and (off & 3) + 1 of the 8 loaded
// bytes, zero-extended to two int16
__device__ __forceinline__ uint32_t pair_sel(uint32_t off)
{
    return 0x0C000C00u | ((off & 3u) + (((off & 3u) + 1u) << 16));
}

}  // namespace lkdev
}  // namespace tbdk
