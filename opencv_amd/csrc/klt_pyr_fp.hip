// klt_pyr_fp.hip — pyramid builds of the floating-point pixel paths (fp16 and
// fp32 levels, SURVEY.md §8f-4 / BASELINE configs[4]) for gfx950, as
// role-split launches that read every source once and write every plane once.
//
// The levels and derivative planes are the ones klt_f16.hip defines (and the
// oracle restates, oracle/klt16_oracle.c orc16_pyr_down / orc16_scharr and the
// orc32_* twins): pyrDown_<FltCast<float,8>>'s scalar order
// (imgproc/src/pyramids.cpp:775-777, 856) and calcSharrDeriv's formula
// (video/src/lkpyramid.cpp:86-131) in fp32, levels rounded to the storage type.
//
// Launch plan for L levels (L launches instead of 2 + L):
//   launch 1: level 0's padded copy of the frame, level 1 straight from the
//             frame (pyrDown taps reflected in the frame, which is what level 0's
//             reflect-101 frame holds), level 0's Scharr plane from the frame;
//   launch i (2..L): level i from level i-1's padded plane, level i-1's Scharr
//             plane from the same plane.
// Every role reads its taps as aligned dword runs (one run per source row,
// realigned with v_alignbyte) and writes 8- to 64-byte vectors; only threads
// whose taps leave the source (frame edges) take the per-element reflect path.
// The old one-launch-per-plane kernels stay in klt_f16.hip behind
// ctx option pyr_fuse=0 for A/B and as a second bit-exact witness.
#include "tbdk_internal.hpp"

#include <stddef.h>

namespace tbdk {

namespace {

typedef _Float16 half_t;

enum { K_U8 = 0, K_U16 = 1, K_F32 = 2, K_F16 = 3 };
enum { R_COPY = 0, R_DOWN = 1, R_SCHARR = 2 };

template <int KIND>
struct Kind {
    static constexpr int ES = KIND == K_U8 ? 1 : KIND == K_F32 ? 4 : 2;
};

// a source plane: p is the interior origin; `avail` columns/rows of reflect-101
// frame exist around it (0 for a caller's frame, pad for a padded level);
// vec: row starts are 4-byte aligned
struct Src {
    const uint8_t* p;
    int pitch, w, h, avail, vec;
};

// a destination plane: p is the padded plane's top-left corner
struct Dst {
    uint8_t* p;
    int pitch, w, h, pad;
};

struct Job {
    int role, kind;
    Src s;
    Dst d;
    int ux, rows, bx, b0;  // threads per row, rows, blocks per row, first block
    int rpt;               // rows per thread (<= kCopyRows / kDownRows / kScharrRows by role)
    int nb;                // blocks of the job (b0 is a multiple of 8: job block b runs on XCD b % 8)
};

struct Jobs {
    Job j[3];
    int n;
    int xcd;  // deal each job's blocks to the XCDs in contiguous row bands (xcd_swizzle)
};

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

// raw element bits at q (1, 2 or 4 bytes)
template <int KIND>
__device__ __forceinline__ uint32_t elem_bits(const uint8_t* q)
{
    if constexpr (Kind<KIND>::ES == 1) return *q;
    else if constexpr (Kind<KIND>::ES == 2) return *reinterpret_cast<const uint16_t*>(q);
    else return *reinterpret_cast<const uint32_t*>(q);
}

// element i of a realigned dword stream, as float
template <int KIND>
__device__ __forceinline__ float from_stream(const uint32_t* al, int i)
{
    if constexpr (KIND == K_U8) return (float)((al[i >> 2] >> (8 * (i & 3))) & 0xFFu);
    else if constexpr (KIND == K_U16) return (float)((al[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
    else if constexpr (KIND == K_F16)
        return (float)__builtin_bit_cast(half_t, (uint16_t)((al[i >> 1] >> (16 * (i & 1))) & 0xFFFFu));
    else return __builtin_bit_cast(float, al[i]);
}

template <int N, int KIND>
struct Run {
    static constexpr int ES = Kind<KIND>::ES;
    static constexpr int NA = (N * ES + 3) / 4;  // dwords of the realigned run
    static constexpr int ND = NA + 1;            // dwords loaded (<= 6 bytes past the run)
};

// The N elements of row r from column x (x may be negative for padded sources)
// as a realigned dword stream al[NA]: aligned dword loads + v_alignbyte where
// the run and its dwords lie inside the source, else one reflected element at a
// time.  Loads only; the caller extracts after issuing every row's loads.
template <int N, int KIND>
__device__ __forceinline__ void row_raw(const Src& s, int r, int x, uint32_t* al)
{
    typedef Run<N, KIND> R;
    constexpr int ES = R::ES;
    bool fast = s.vec && r >= -s.avail && r < s.h + s.avail && x >= -s.avail && x + N <= s.w + s.avail;
    const uint8_t* row = s.p + (ptrdiff_t)r * s.pitch;
    const uintptr_t ad = (uintptr_t)(row + (ptrdiff_t)x * ES);
    const uintptr_t a = ad & ~(uintptr_t)3;
    // on the last row the loaded dwords must end inside the row's bytes
    if (fast && r == s.h - 1 + s.avail) fast = a + 4 * R::ND <= (uintptr_t)(row + (ptrdiff_t)(s.w + s.avail) * ES);
    if (fast) {
        const uint32_t* d = reinterpret_cast<const uint32_t*>(a);
        const uint32_t o = (uint32_t)(ad & 3);
        uint32_t dw[R::ND];
#pragma unroll
        for (int k = 0; k < R::ND; ++k) dw[k] = d[k];
#pragma unroll
        for (int k = 0; k < R::NA; ++k) al[k] = __builtin_amdgcn_alignbyte(dw[k + 1], dw[k], o);
    } else {
        const uint8_t* rr = s.p + (ptrdiff_t)reflect101(r, s.h) * s.pitch;
#pragma unroll
        for (int k = 0; k < R::NA; ++k) al[k] = 0;
#pragma unroll
        for (int i = 0; i < N; ++i)
            al[i * ES / 4] |= elem_bits<KIND>(rr + (ptrdiff_t)reflect101(x + i, s.w) * ES) << (8 * ((i * ES) & 3));
    }
}

__device__ __forceinline__ uint32_t hbits(float f) { return __builtin_bit_cast(uint16_t, (half_t)f); }

constexpr int kCopyRows = 4, kScharrRows = 4, kDownRows = 2;

// level 0: 8 values of padded rows py0.. (kCopyRows) from padded column 8t
template <int KIND, bool F32>
__device__ __forceinline__ void role_copy(const Job& j, int t, int py0)
{
    typedef Run<8, KIND> R;
    uint32_t raw[kCopyRows][R::NA];
    const int nr = j.rows - py0 < j.rpt ? j.rows - py0 : j.rpt;
#pragma unroll
    for (int k = 0; k < kCopyRows; ++k)
        if (k < nr) row_raw<8, KIND>(j.s, py0 + k - j.d.pad, 8 * t - j.d.pad, raw[k]);
#pragma unroll
    for (int k = 0; k < kCopyRows; ++k) {
        if (k >= nr) break;
        uint8_t* q = j.d.p + (size_t)(py0 + k) * j.d.pitch;
        if constexpr (F32) {
            float4* o = reinterpret_cast<float4*>(q) + 2 * t;
            if constexpr (KIND == K_F32) {
                o[0] = make_float4(__builtin_bit_cast(float, raw[k][0]), __builtin_bit_cast(float, raw[k][1]),
                                   __builtin_bit_cast(float, raw[k][2]), __builtin_bit_cast(float, raw[k][3]));
                o[1] = make_float4(__builtin_bit_cast(float, raw[k][4]), __builtin_bit_cast(float, raw[k][5]),
                                   __builtin_bit_cast(float, raw[k][6]), __builtin_bit_cast(float, raw[k][7]));
            } else {
                float v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = from_stream<KIND>(raw[k], i);
                o[0] = make_float4(v[0], v[1], v[2], v[3]);
                o[1] = make_float4(v[4], v[5], v[6], v[7]);
            }
        } else if constexpr (KIND == K_F16) {
            reinterpret_cast<uint4*>(q)[t] = make_uint4(raw[k][0], raw[k][1], raw[k][2], raw[k][3]);
        } else {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = from_stream<KIND>(raw[k], i);
            reinterpret_cast<uint4*>(q)[t] = make_uint4(hbits(v[0]) | hbits(v[1]) << 16, hbits(v[2]) | hbits(v[3]) << 16,
                                                        hbits(v[4]) | hbits(v[5]) << 16, hbits(v[6]) | hbits(v[7]) << 16);
        }
    }
}

__device__ __forceinline__ float hsum5(const float* v)
{
    return v[2] * 6.f + (v[1] + v[3]) * 4.f + v[0] + v[4];
}

// horizontal pass of pyrDown for 4 consecutive outputs from an 11-element run
template <int KIND>
__device__ __forceinline__ void hrow4(const uint32_t* al, float* r)
{
    float v[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) v[i] = from_stream<KIND>(al, i);
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = hsum5(v + 2 * c);
}

template <bool F32>
__device__ __forceinline__ void store_down(const Job& j, int t, int py, const float (*r)[4])
{
    float o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
        o[c] = (r[2][c] * 6.f + (r[1][c] + r[3][c]) * 4.f + r[0][c] + r[4][c]) * (1.f / 256.f);
    uint8_t* q = j.d.p + (size_t)py * j.d.pitch;
    if constexpr (F32) reinterpret_cast<float4*>(q)[t] = make_float4(o[0], o[1], o[2], o[3]);
    else reinterpret_cast<uint2*>(q)[t] = make_uint2(hbits(o[0]) | hbits(o[1]) << 16, hbits(o[2]) | hbits(o[3]) << 16);
}

// pyrDown: 4 values of one padded destination row py from padded column 4t
template <int KIND, bool F32>
__device__ __forceinline__ void down_row(const Job& j, int t, int py)
{
    const int ry = reflect101(py - j.d.pad, j.d.h);
    const int cx = 4 * t - j.d.pad;
    float r[5][4];
    if (cx >= 0 && cx + 4 <= j.d.w) {
        uint32_t raw[5][Run<11, KIND>::NA];
#pragma unroll
        for (int k = 0; k < 5; ++k) row_raw<11, KIND>(j.s, 2 * ry - 2 + k, 2 * cx - 2, raw[k]);
#pragma unroll
        for (int k = 0; k < 5; ++k) hrow4<KIND>(raw[k], r[k]);
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int rx = reflect101(cx + c, j.d.w);
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                uint32_t raw[Run<5, KIND>::NA];
                row_raw<5, KIND>(j.s, 2 * ry - 2 + k, 2 * rx - 2, raw);
                float v[5];
#pragma unroll
                for (int i = 0; i < 5; ++i) v[i] = from_stream<KIND>(raw, i);
                r[k][c] = hsum5(v);
            }
        }
    }
    store_down<F32>(j, t, py, r);
}

// pyrDown: padded destination rows py0, py0+1 (kDownRows); interior row pairs
// share their 7 source rows, rows of the reflect frame go one at a time
template <int KIND, bool F32>
__device__ __forceinline__ void role_down(const Job& j, int t, int py0)
{
    const int cx = 4 * t - j.d.pad;
    const int y0 = py0 - j.d.pad;
    if (j.rpt == 1) {
        down_row<KIND, F32>(j, t, py0);
    } else if (y0 >= 0 && y0 + 2 <= j.d.h && cx >= 0 && cx + 4 <= j.d.w) {
        uint32_t raw[7][Run<11, KIND>::NA];
#pragma unroll
        for (int k = 0; k < 7; ++k) row_raw<11, KIND>(j.s, 2 * y0 - 2 + k, 2 * cx - 2, raw[k]);
        float r[7][4];
#pragma unroll
        for (int k = 0; k < 7; ++k) hrow4<KIND>(raw[k], r[k]);
        store_down<F32>(j, t, py0, r);
        store_down<F32>(j, t, py0 + 1, r + 2);
    } else {
        down_row<KIND, F32>(j, t, py0);
        if (py0 + 1 < j.rows) down_row<KIND, F32>(j, t, py0 + 1);
    }
}

// Scharr pairs of 8 interior pixels from column 8t, rows y0.. (kScharrRows)
template <int KIND, bool F32>
__device__ __forceinline__ void role_scharr(const Job& j, int t, int y0)
{
    typedef Run<10, KIND> R;
    const int x0 = 8 * t;
    uint32_t raw[kScharrRows + 2][R::NA];
    const int nr = j.s.h - y0 < j.rpt ? j.s.h - y0 : j.rpt;
#pragma unroll
    for (int k = 0; k < kScharrRows + 2; ++k)
        if (k < nr + 2) row_raw<10, KIND>(j.s, y0 - 1 + k, x0 - 1, raw[k]);
    const int n = j.s.w - x0;
#pragma unroll
    for (int rr = 0; rr < kScharrRows; ++rr) {
        if (rr >= nr) break;
        float t0[10], t1[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            const float a = from_stream<KIND>(raw[rr], k), b = from_stream<KIND>(raw[rr + 1], k),
                        c = from_stream<KIND>(raw[rr + 2], k);
            t0[k] = (a + c) * 3.f + b * 10.f;
            t1[k] = c - a;
        }
        float ix[8], iy[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            ix[k] = t0[k + 2] - t0[k];
            iy[k] = (t1[k + 2] + t1[k]) * 3.f + t1[k + 1] * 10.f;
        }
        uint8_t* q = j.d.p + (size_t)(y0 + rr + j.d.pad) * j.d.pitch;
        if constexpr (F32) {
            float2* o = reinterpret_cast<float2*>(q) + j.d.pad + x0;
            if (n >= 8) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    reinterpret_cast<float4*>(o)[k] = make_float4(ix[2 * k], iy[2 * k], ix[2 * k + 1], iy[2 * k + 1]);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k < n) o[k] = make_float2(ix[k], iy[k]);
            }
        } else {
            uint32_t p[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) p[k] = hbits(ix[k]) | hbits(iy[k]) << 16;
            uint32_t* o = reinterpret_cast<uint32_t*>(q) + j.d.pad + x0;
            if (n >= 8) {
                reinterpret_cast<uint4*>(o)[0] = make_uint4(p[0], p[1], p[2], p[3]);
                reinterpret_cast<uint4*>(o)[1] = make_uint4(p[4], p[5], p[6], p[7]);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k < n) o[k] = p[k];
            }
        }
    }
}

template <int KIND, bool F32>
__device__ __forceinline__ void run_role(const Job& j, int t, int rg)
{
    if (j.role == R_COPY) role_copy<KIND, F32>(j, t, rg * j.rpt);
    else if (j.role == R_DOWN) role_down<KIND, F32>(j, t, rg * j.rpt);
    else role_scharr<KIND, F32>(j, t, rg * j.rpt);
}

template <bool F32>
__global__ void __launch_bounds__(256) pyr_fp_jobs_kernel(Jobs js)
{
    const int b = blockIdx.x;
    int i = 0;
    while (i + 1 < js.n && b >= js.j[i + 1].b0) ++i;
    const Job& j = js.j[i];
    if (b - j.b0 >= j.nb) return;  // alignment gap before the next job
    const int rb = js.xcd ? xcd_swizzle(b - j.b0, j.nb) : b - j.b0;
    const int row = rb / j.bx;  // row group
    const int t = (rb - row * j.bx) * 256 + (int)threadIdx.x;
    if (t >= j.ux) return;
    if constexpr (F32) {
        if (j.kind == K_U8) run_role<K_U8, true>(j, t, row);
        else if (j.kind == K_U16) run_role<K_U16, true>(j, t, row);
        else run_role<K_F32, true>(j, t, row);
    } else {
        if (j.kind == K_U8) run_role<K_U8, false>(j, t, row);
        else run_role<K_F16, false>(j, t, row);
    }
}

Src frame_src(const uint8_t* img, int pitch, int w, int h)
{
    return Src{img, pitch, w, h, 0, ((uintptr_t)img % 4 == 0 && pitch % 4 == 0) ? 1 : 0};
}

Src level_src(const tbdk_level& L, int es)
{
    return Src{L.data + (size_t)L.pad * L.pitch + (size_t)L.pad * es, L.pitch, L.width, L.height, L.pad, 1};
}

Dst level_dst(const tbdk_level& L)
{
    return Dst{L.data, L.pitch, L.width, L.height, L.pad};
}

void add_job(Jobs& js, int& nb, int role, int kind, const Src& s, const Dst& d, int rows)
{
    Job& j = js.j[js.n++];
    j.role = role;
    j.kind = kind;
    j.s = s;
    j.d = d;
    if (role == R_COPY) {
        j.ux = (d.w + 2 * d.pad + 7) / 8;
        j.rows = d.h + 2 * d.pad;
    } else if (role == R_DOWN) {
        j.ux = (d.w + 2 * d.pad + 3) / 4;
        j.rows = d.h + 2 * d.pad;
    } else {
        j.ux = (s.w + 7) / 8;
        j.rows = s.h;
    }
    const int cap = role == R_COPY ? kCopyRows : role == R_DOWN ? kDownRows : kScharrRows;
    j.rpt = rows < 1 ? 1 : rows > cap ? cap : rows;
    j.bx = (j.ux + 255) / 256;
    j.b0 = (nb + 7) & ~7;
    j.nb = j.bx * ((j.rows + j.rpt - 1) / j.rpt);
    nb = j.b0 + j.nb;
}

}  // namespace

// kind: K_U8 / K_U16 / K_F32 / K_F16 frame; f32: fp32 levels (else fp16); rows: rows per thread
// (ctx option pyr_rows; the level-1 rows go in pairs at most)
hipError_t launch_pyr_build_fp(const uint8_t* img, int pitch, int kind, bool f32, const tbdk_pyr& pyr, int rows,
                               int xcd, hipStream_t s)
{
    const int es = f32 ? 4 : 2;
    const int L = pyr.nlevels;
    const Src fr = frame_src(img, pitch, pyr.lv[0].width, pyr.lv[0].height);
    for (int i = 1; i <= L; ++i) {
        Jobs js;
        js.n = 0;
        js.xcd = xcd;
        int nb = 0;
        if (i == 1) {
            add_job(js, nb, R_COPY, kind, fr, level_dst(pyr.lv[0]), rows);
            if (L > 1) add_job(js, nb, R_DOWN, kind, fr, level_dst(pyr.lv[1]), rows);
            add_job(js, nb, R_SCHARR, kind, fr, level_dst(pyr.dv[0]), rows);
        } else {
            const int lk = f32 ? K_F32 : K_F16;
            const Src ls = level_src(pyr.lv[i - 1], es);
            if (i < L) add_job(js, nb, R_DOWN, lk, ls, level_dst(pyr.lv[i]), rows);
            add_job(js, nb, R_SCHARR, lk, ls, level_dst(pyr.dv[i - 1]), rows);
        }
        if (f32) hipLaunchKernelGGL(pyr_fp_jobs_kernel<true>, dim3(nb), dim3(256), 0, s, js);
        else hipLaunchKernelGGL(pyr_fp_jobs_kernel<false>, dim3(nb), dim3(256), 0, s, js);
    }
    return hipGetLastError();
}

}  // namespace tbdk
