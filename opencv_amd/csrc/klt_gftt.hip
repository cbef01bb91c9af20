// klt_gftt.hip — Shi-Tomasi corners (goodFeaturesToTrack, min-eigenvalue
// variant) over many isolated ROIs of a frame, for gfx950.
//
// Per-ROI semantics are those of cv::goodFeaturesToTrack on the ROI as an
// isolated image (imgproc/src/featureselect.cpp:361-516 with
// cornerMinEigenVal, corner.cpp:52-101,237-326), in the float/double
// evaluation order documented in oracle/gftt_oracle.c; built with
// -ffp-contract=off so every expression rounds exactly as written.
//
// Two launches, all ROIs of a frame batched in each:
//   1. gftt_eig   : one workgroup per 56-column strip of a ROI, its waves
//                   walking row segments: Sobel 3x3 (reflect-101 inside the
//                   ROI) -> cov = (Dx^2, DxDy, Dy^2) -> the boxFilter's row
//                   sums in double (neighbour columns by DPP wave shifts) ->
//                   the reference's running ColumnSum walked top to bottom ->
//                   min eigenvalue; per-strip max and the rows' 3x3
//                   local-maximum ballots (the threshold-independent half of
//                   the reference's threshold + dilate test)
//   2. gftt_select: one 512-thread workgroup per ROI: candidates (local
//                   maxima above max*q), sort by
//                   (value desc, address desc) — the reference's deterministic
//                   tie-break (featureselect.cpp:56-64) — then the greedy
//                   min-distance walk (:421-503) by one wave, 64 candidates per
//                   step over a byte image of the ROI; in-step conflicts are
//                   resolved in lane order so exactly the sequential walk's
//                   corners are accepted.
#include <atomic>
#include <cfloat>
#include <cmath>
#include <type_traits>

#include "tbdk_internal.hpp"

namespace tbdk {

namespace {

__device__ __forceinline__ int refl(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// float -> int order-preserving key (for atomicMax on floats of either sign)
__device__ __forceinline__ int fkey(float f)
{
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float fkey_inv(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF); }

}  // namespace

// ROI r of the launch: from the kernel arguments when the table travels there
// (GfttArgs::inl), else from the table in memory
__device__ __forceinline__ GfttRoi roi_at(const GfttArgs& a, int r)
{
    if (a.ninl > 0) {
        const GfttRoiC c = a.inl[r];
        return GfttRoi{c.x, c.y, c.w, c.h, c.off, c.moff, c.cblk};
    }
    return a.rois[r];
}

__device__ __forceinline__ int roi_of_cblock(const GfttArgs& a, int b)
{
    int lo = 0, hi = a.nroi - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((a.ninl > 0 ? a.inl[mid].cblk : a.rois[mid].cblk) <= b) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// DPP wave shifts (GFX9): lane i receives lane i-1 (shr) / lane i+1 (shl)
// (the lane without a source reads 0 by bound_ctrl, so no old value has to be
// materialised first)
__device__ __forceinline__ float from_left(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float from_right(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xF, 0xF, true));
}

// Sobel rows of one image row at columns (x-1, x, x+1) in the reference's
// filter-engine order (see oracle/gftt_oracle.c): rx = [-1 0 1], ry = [k 2k k]
struct SobelRow {
    float rx, ry;
};
__device__ __forceinline__ SobelRow sobel_row(float s0, float s1, float s2, float k, float k2)
{
    float t = -1.f * s0;
    t = t + 0.f * s1;
    t = t + 1.f * s2;
    float u = k * s0;
    u = u + k2 * s1;
    u = u + k * s2;
    return SobelRow{t, u};
}

// Fused Sobel -> cov -> boxFilter -> min eigenvalue for one 56-column strip of
// a ROI per workgroup.  Lane L holds ROI column x0 - 4 + L (lanes 4..59 produce
// output, four halo lanes per side); each lane loads only its own pixel of a
// row and gets its neighbours by DPP wave shifts; lanes outside the ROI hold
// their reflect-101 column (see eig_srow).
//
// The box filter is the reference's running ColumnSum (box_filter.simd.hpp:
// 176-273), per channel: SUM = (0 + rs(-1)) + rs(0); per row y:
// s = SUM + rs(y+1); out = (float)s; SUM = s - rs(y-1), rows reflect-101.
// The strip's rows are split into kEigWaves segments, one wave each, all three
// channels per wave, walked concurrently.  A segment starting at y0 > 0 starts
// its SUM fresh as (0 + rs(y0-1)) + rs(y0), which is the reference's running
// value exactly when every earlier chain operation was exact; this is checked
// where it matters: segment k is right iff segment k-1 was right and the SUM
// k-1 ends with equals k's fresh start (segment 0 starts as the reference
// does).  From the first mismatch on (not observed on natural images, forced
// by the "gftt_eig_redo" option in the tests) the segments are walked again one
// after another, each from its predecessor's final SUM: the reference's
// sequential order.
// 4 since round 6: 256-thread workgroups find CU room beside the loop's PyrLK
// waves sooner (loop +1 % over 8 rounds with the compact candidates; standalone
// the 8-segment walk is faster, 19.5 against 23.6 us for 76 ROIs)
#ifndef TBDK_GFTT_EIG_WAVES
#define TBDK_GFTT_EIG_WAVES 4
#endif
constexpr int kEigWaves = TBDK_GFTT_EIG_WAVES;  // row segments (waves) per strip
constexpr int kEigPref = 8;   // pixel rows in flight per wave (the eigenvalue-plane kernel)
// ... in the compact-candidate kernel: 4 keeps it at <= 128 VGPRs (8: 148),
// so its waves fit where one of the loop's PyrLK waves (121) has ended
#ifndef TBDK_GFTT_EIG_PREF_C
#define TBDK_GFTT_EIG_PREF_C 4
#endif
#ifndef TBDK_GFTT_WALK_PRIO
#define TBDK_GFTT_WALK_PRIO 3  // s_setprio of gftt_select's walking wave
#endif
#ifndef GFTT_ESTAMP  // eigenvalue-walk phase hooks for tools/ probes (no-ops in the library build)
#define GFTT_ESTAMP(i)
#endif

struct EigLane {
    __amdgpu_buffer_rsrc_t rs;
    int x, H, hm2, pitch;
    bool mir, out_lane;  // mir: a lane outside the ROI holding its reflect-101 column
    float k, k2;
};

__device__ __forceinline__ float eig_ld(const EigLane& g, int row)
{
    return (float)__builtin_amdgcn_raw_buffer_load_b8(g.rs, g.x, row * g.pitch, 0);
}

// Sobel row terms of the pixel row whose own value is v (neighbours by DPP).
// Every lane holds the pixel of its column's reflect-101 image (lanes left or
// right of the ROI: the mirrored column), so the neighbours of an in-ROI lane
// are the reference's reflected pixels as they are; a mirrored lane sees its
// column's neighbours in the opposite order and swaps them, and then holds that
// column's Sobel terms and covariances exactly — the box filter's reflect-101
// of the cov image (cov(-1) = cov(1)) with no per-channel fix-up.
__device__ __forceinline__ SobelRow eig_srow(const EigLane& g, float v)
{
    const float l = from_left(v), rr = from_right(v);
    return sobel_row(g.mir ? rr : l, v, g.mir ? l : rr, g.k, g.k2);
}

// the three cov channels of one row and their boxFilter row sums ((l + c) + r in double)
__device__ __forceinline__ void eig_rowsums(const EigLane& g, const SobelRow& p, const SobelRow& c,
                                            const SobelRow& n, double (&out)[3])
{
    const float dx = (p.rx + n.rx) * g.k + (c.rx * g.k2 + 0.f);
    const float dy = (n.ry - p.ry) + 0.f;
    const float cv[3] = {dx * dx, dx * dy, dy * dy};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float l = from_left(cv[ch]), rr = from_right(cv[ch]);
        out[ch] = (double)l + (double)cv[ch] + (double)rr;
    }
}

// Walk rows [ys, ye) of the strip (own rows [y0, y1) plus one halo row on
// each side inside the ROI): box sums from SUM (fresh: the start above, at
// ys), eigenvalues of the own rows to E, their max key into best, and for own
// interior rows the ballot of lanes whose value is >= all 8 neighbours (the
// threshold-independent half of the reference's threshold + 3x3 dilate test)
// into lm.  S0 = the SUM the walk started from; Scap = the SUM before row
// ycap (the next segment's fresh-start row); S = the SUM after the last row.
// Compact (GfttArgs::compact): no eigenvalue plane; with each row's
// local-maximum ballot, the values of its set lanes only, in lane order, at the
// start of the strip row's own columns (column ccol + rank of the lane's bit),
// which is all gftt_select reads when quality <= 1 (see there).
template <bool compact, int PREF = compact ? TBDK_GFTT_EIG_PREF_C : kEigPref>
__device__ __forceinline__ void eig_segment(const EigLane& g, float* __restrict__ E, uint64_t* __restrict__ lm,
                                            int w, int ep, int y0, int y1, int ys, int ye, int ycap, bool fresh,
                                            double (&S)[3], double (&S0)[3], double (&Scap)[3], int& best, int ccol)
{
    const int H = g.H;
    auto pix = [&](int yy) { return eig_ld(g, refl(yy, H)); };
    auto pix_fwd = [&](int yy) { return eig_ld(g, yy < H ? yy : g.hm2); };  // yy in [0, H]
    const int lane = threadIdx.x & 63;
    const bool x_in = g.out_lane && g.x >= 1 && g.x <= w - 2;
    double qa[3], qb[3];  // rs(y - 1), rs(y)
    {
        const int rm = refl(ys - 1, H);  // the box filter reflects cov rows
        eig_rowsums(g, eig_srow(g, pix(rm - 1)), eig_srow(g, pix(rm)), eig_srow(g, pix(rm + 1)), qa);
    }
    SobelRow wa = eig_srow(g, pix(ys)), wb = eig_srow(g, pix(ys + 1));
    eig_rowsums(g, eig_srow(g, pix(ys - 1)), wa, wb, qb);
    if (fresh) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) S[ch] = (0.0 + qa[ch]) + qb[ch];
    }
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) S0[ch] = S[ch];
    float e1 = 0.f, e2 = 0.f;  // eigenvalues of rows y - 1, y - 2
    // E and lm through buffer stores: a lane that must not write gets an offset
    // past the buffer, which the hardware drops, so the steady rows below stay
    // one straight-line block (no exec-mask branches between rows)
    const __amdgpu_buffer_rsrc_t rE =
        __builtin_amdgcn_make_buffer_rsrc(E - g.x, (short)0, ep * H * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rL = __builtin_amdgcn_make_buffer_rsrc(lm, (short)0, lm ? H * 8 : 0, 0x00020000);
    constexpr uint32_t kDrop = 0x80000000u;
    const uint32_t eoff = g.out_lane ? (uint32_t)g.x * 4u : kDrop;
    // one walked row y (cur = pixel row y + 2); the flags are compile-time true
    // in the steady rows
    auto row = [&](auto steady, int y, float cur, bool has_next, bool store, bool lmx) {
        constexpr bool ST = decltype(steady)::value;
        double in[3];
        SobelRow wc = wb;
        if (ST || has_next) {  // entering cov row y + 1 (image rows y, y+1, y+2)
            wc = eig_srow(g, cur);
            eig_rowsums(g, wa, wb, wc, in);
        } else {  // rs(refl(H)) == rs(H - 2) == rs(y - 1)
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) in[ch] = qa[ch];
        }
        float box[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const double t = S[ch] + in[ch];
            box[ch] = (float)t;
            S[ch] = t - qa[ch];
            qa[ch] = qb[ch];
            qb[ch] = in[ch];
        }
        wa = wb;
        wb = wc;
        const float aa = box[0] * 0.5f, bb = box[1], cc = box[2] * 0.5f;
        const float t = aa - cc;
        const float e = (aa + cc) - sqrtf(bb * bb + t * t);
        if (ST || store) {
            if constexpr (!compact)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(e), rE, eoff == kDrop ? kDrop : eoff + (uint32_t)(y * ep * 4), 0, 0);
            const int kk = fkey(e);
            best = (g.out_lane && kk > best) ? kk : best;
        }
        if (ST || lmx) {  // row y - 1's 3x3 neighbourhood is now complete
            float m = fmaxf(e2, e);
            m = fmaxf(m, fmaxf(from_left(e2), from_right(e2)));
            m = fmaxf(m, fmaxf(from_left(e1), from_right(e1)));
            m = fmaxf(m, fmaxf(from_left(e), from_right(e)));
            const bool lmax = x_in && e1 >= m;
            const uint64_t bal = __ballot(lmax);
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 bv = {(unsigned)bal, (unsigned)(bal >> 32)};
            __builtin_amdgcn_raw_buffer_store_b64(bv, rL, lane == 0 ? (uint32_t)((y - 1) * 8) : kDrop, 0, 0);
            if constexpr (compact) {  // row y - 1's candidates, packed in lane order
                const uint32_t rk =
                    __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(e1), rE,
                                                      lmax ? (uint32_t)(((y - 1) * ep + ccol + (int)rk) * 4) : kDrop, 0, 0);
            }
        }
        e2 = e1;
        e1 = e;
    };
    // any row, flags at run time (the capture of Scap before row ycap included)
    auto generic = [&](int y) {
        if (y == ycap) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) Scap[ch] = S[ch];
        }
        const int yc = y - 1;
        row(std::false_type{}, y, y + 1 < H ? pix_fwd(y + 2) : 0.f, y + 1 < H, y >= y0 && y < y1,
            yc >= y0 && yc < y1 && yc >= 1 && yc <= H - 2);
    };
    // steady rows [sa, sb): own rows with a complete 3x3 row above, a next row,
    // and not the capture row; the rest of [ys, ye) by generic rows
    const int sa = max(max(y0 + 1, 2), ys);
    int sb = min(min(y1, H - 1), ye);
    if (ycap >= 0) sb = min(sb, ycap);
    int y = ys;
    if (sb - sa >= PREF) {
        for (; y < sa; ++y) generic(y);
        float nxt[PREF];
#pragma unroll
        for (int j = 0; j < PREF; ++j) nxt[j] = pix_fwd(y + 2 + j);
        for (; y + PREF <= sb; y += PREF) {
            float cur[PREF];
#pragma unroll
            for (int j = 0; j < PREF; ++j) cur[j] = nxt[j];
#pragma unroll
            for (int j = 0; j < PREF; ++j) nxt[j] = pix_fwd(min(y + PREF + 2 + j, H));  // in flight
#pragma unroll
            for (int j = 0; j < PREF; ++j) row(std::true_type{}, y + j, cur[j], true, true, true);
        }
    }
    for (; y < ye; ++y) generic(y);
}

// compact (GfttArgs::compact, see eig_segment): one instantiation per mode,
// so each has its own register budget
template <bool compact>
__global__ __launch_bounds__(64 * kEigWaves) void gftt_eig_kernel(GfttArgs a)
{
    __shared__ double s_cap[kEigWaves][3][64];
    __shared__ double s_drift[3][64];
    __shared__ int s_best[kEigWaves];
    __shared__ int s_bad;
    const int r = roi_of_cblock(a, blockIdx.x);
    const GfttRoi R = roi_at(a, r);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int H = R.h;

    EigLane g;
    const int strip = blockIdx.x - R.cblk;
    const int xc = strip * kGfttStrip - kGfttHalo + lane;  // this lane's ROI column
    g.out_lane = lane >= kGfttHalo && lane < kGfttHalo + kGfttStrip && xc < R.w;
    // the lane's column of the reflect-101 image (borderInterpolate, REFLECT_101);
    // only columns -2 .. w+1 are read by an output (its cov at -1 .. w), lanes
    // farther out take any in-ROI column
    {
        const int w = R.w;
        int xm = xc < -2 || xc > w + 1 ? min(max(xc, 0), w - 1) : xc;
        if (w == 1) {
            xm = 0;
        } else {
#pragma unroll
            for (int it = 0; it < 2; ++it) {  // two reflections reach [0, w) from -2 .. w+1 for w >= 2
                if (xm < 0) xm = -xm;
                if (xm >= w) xm = 2 * (w - 1) - xm;
            }
        }
        g.x = xm;
        g.mir = xc < 0 || xc >= w;
    }
    const double scale = 1.0 / ((double)(1 << 2) * 3 * 255.0);
    g.k = (float)(1.0 * scale);
    g.k2 = (float)(2.0 * scale);
    g.H = H;
    g.hm2 = H >= 2 ? H - 2 : 0;
    g.pitch = a.pitch;
    g.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.img + (size_t)R.y * a.pitch + R.x), (short)0,
                                             a.pitch * H, 0x00020000);
    float* E = a.eig + R.off + g.x;
    // local-maximum words of this strip (ROIs of at least 3x3; never written otherwise)
    uint64_t* lm = a.lmax + R.moff + (size_t)strip * H;
    const bool has_lm = R.w >= 3 && H >= 3;
    const int ccol = strip * kGfttStrip;  // the strip's first output column

    const int L = (H + kEigWaves - 1) / kEigWaves;  // own rows per segment
    const int y0 = wv * L, y1 = min(H, y0 + L);
    const bool live = y0 < y1;
    const int ys = y0 > 0 ? y0 - 1 : 0, ye = min(H, y1 + 1);
    const int ycap = y1 < H ? y1 - 1 : -1;  // the next segment starts fresh at y1 - 1
    int best = INT_MIN;
    double S[3], S0[3], Scap[3];
    // lanes whose box sums reach an output: the eigenvalues of lanes 3..60 (the
    // local-maximum test of output lanes 4..59 reads their neighbours) inside the ROI;
    // the outer halo lanes and clamped columns carry sums nothing reads
    const bool need = lane >= kGfttHalo - 1 && lane <= kGfttHalo + kGfttStrip && xc >= 0 && xc < R.w;
    // segment `from` on: the first whose start may differ from the reference's SUM
    auto first_mismatch = [&](int from) {
        if (threadIdx.x == 0) s_bad = kEigWaves;
        __syncthreads();
        if (live && wv > from) {
            bool diff = a.eig_redo != 0 && wv == from + 1;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) diff |= need && S0[ch] != s_cap[wv - 1][ch][lane];
            if (__any(diff) && lane == 0) atomicMin(&s_bad, wv);
        }
        __syncthreads();
        return s_bad;
    };
    GFTT_ESTAMP(0);
    if (live) {
        eig_segment<compact>(g, E, has_lm ? lm : nullptr, R.w, gftt_epitch(R.w), y0, y1, ys, ye, ycap, true, S, S0,
                             Scap, best, ccol);
        if (ycap >= 0) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) s_cap[wv][ch][lane] = Scap[ch];
        }
    }
    int bad = first_mismatch(0);
    GFTT_ESTAMP(1);
    // Cold: segment `bad` is walked again from its predecessor's final SUM (the
    // reference's value: the predecessor's own start was verified), and the
    // segments after it concurrently from their fresh starts plus the drift
    // d = true - fresh found at `bad` (a rounding in the chain shifts every later
    // SUM by the same amount unless another rounding intervenes); the
    // boundaries are checked again.  Each round fixes at least segment `bad`.
    while (bad < kEigWaves) {
        if (wv == bad && live) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) s_drift[ch][lane] = s_cap[bad - 1][ch][lane] - S0[ch];
        }
        __syncthreads();
        if (wv >= bad && live) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch)
                S[ch] = wv == bad ? s_cap[bad - 1][ch][lane] : S0[ch] + s_drift[ch][lane];
        }
        __syncthreads();  // s_cap is rewritten below
        if (wv >= bad && live) {
            best = INT_MIN;
            eig_segment<compact>(g, E, has_lm ? lm : nullptr, R.w, gftt_epitch(R.w), y0, y1, ys, ye, ycap, false, S,
                                 S0, Scap, best, ccol);
            if (ycap >= 0) {
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) s_cap[wv][ch][lane] = Scap[ch];
            }
        }
        bad = first_mismatch(bad);
    }
    // per-strip max (minMaxLoc is order independent)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int v = __shfl_xor(best, o);
        best = v > best ? v : best;
    }
    if (lane == 0) s_best[wv] = best;
    __syncthreads();
    GFTT_ESTAMP(2);
    if (threadIdx.x == 0) {
        int m = s_best[0];
#pragma unroll
        for (int k = 1; k < kEigWaves; ++k) m = s_best[k] > m ? s_best[k] : m;
        a.blk_max[blockIdx.x] = m;
    }
}

// Candidate sort key: the reference order (value desc, then address desc,
// featureselect.cpp:56-64) is the descending order of
//   (orderable bits of the float value) << 32 | (y << 16 | x)
__device__ __forceinline__ uint64_t cand_key(float v, int y, int x)
{
    return ((uint64_t)((uint32_t)fkey(v) ^ 0x80000000u) << 32) | (uint32_t)((y << 16) | x);
}

constexpr int kSelThreads = 512;

// phase hooks for tools/ probes (no-ops in the library build)
#ifndef GFTT_STAMP
#define GFTT_STAMP(i)
#define GFTT_TDECL
#define GFTT_T(i)
#define GFTT_TDUMP
#endif

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int d)
{
    const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
    const int l2 = __shfl_xor(lo, d), h2 = __shfl_xor(hi, d);
    return ((uint64_t)(uint32_t)h2 << 32) | (uint32_t)l2;
}

// Bitonic sort of np2 keys, descending, E keys per thread in registers
// (element e = tid * E + u): stages with j < E swap registers, E <= j < 64E
// exchange across lanes of the wave (no barrier), only j >= 64E go through LDS.
template <int E>
__device__ __forceinline__ void sort_keys(uint64_t* keys, int np2, int tid)
{
    uint64_t x[E];
    const bool active = tid * E < np2;
#pragma unroll
    for (int u = 0; u < E; ++u) x[u] = active ? keys[tid * E + u] : 0ull;
    bool lds_dirty = false;
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j < E) {
#pragma unroll
                for (int jj = E / 2; jj >= 1; jj >>= 1) {  // compile-time register indices
                    if (jj != j) continue;
#pragma unroll
                    for (int u = 0; u < E; ++u) {
                        if (u & jj) continue;
                        const int e = tid * E + u;
                        const bool desc = (e & k) == 0;
                        const uint64_t p = x[u], q = x[u | jj];
                        const bool sw = desc ? p < q : p > q;
                        x[u] = sw ? q : p;
                        x[u | jj] = sw ? p : q;
                    }
                }
            } else if (j < 64 * E) {
                const int d = j / E;
                const bool lower = (tid & d) == 0;
#pragma unroll
                for (int u = 0; u < E; ++u) {
                    const uint64_t y = shfl_xor_u64(x[u], d);
                    const int e = tid * E + u;
                    const bool desc = (e & k) == 0;
                    const bool take_max = lower == desc;
                    x[u] = take_max ? (x[u] > y ? x[u] : y) : (x[u] < y ? x[u] : y);
                }
            } else {
                if (lds_dirty) __syncthreads();  // previous LDS stage's reads are done
                if (active)
#pragma unroll
                    for (int u = 0; u < E; ++u) keys[tid * E + u] = x[u];
                __syncthreads();
                if (active)
#pragma unroll
                    for (int u = 0; u < E; ++u) {
                        const int e = tid * E + u;
                        const uint64_t y = keys[e ^ j];
                        const bool desc = (e & k) == 0;
                        const bool take_max = ((e & j) == 0) == desc;
                        x[u] = take_max ? (x[u] > y ? x[u] : y) : (x[u] < y ? x[u] : y);
                    }
                lds_dirty = true;
            }
        }
    }
    __syncthreads();
    if (active)
#pragma unroll
        for (int u = 0; u < E; ++u) keys[tid * E + u] = x[u];
    __syncthreads();
}

// Sort of exactly kSelThreads (512) keys, descending (the partial selection's
// usual case): each wave sorts its 64 keys in registers (a 21-stage bitonic
// network over the wave's lanes, no barrier), then every key's final place is
// its rank: its index in its own run plus, for each of the other seven sorted
// runs, the count of keys ahead of it there (branchless binary searches, the
// seven runs' reads in flight together; >= for runs of lower wave index and >
// for higher ones, so the equal padding keys get distinct places).  Same result
// as the 45-stage bitonic sort over the workgroup with its six LDS stages.
// lane ^ J of a 32-bit value without the LDS unit where DPP reaches it:
// quad_perm for 1 and 2, a row shift each way and a select for 4 and 8,
// ds_swizzle (no address VGPR) for 16, ds_bpermute for 32
template <int J>
__device__ __forceinline__ int xor_lane(int v, int lane)
{
    if constexpr (J == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);
    else if constexpr (J == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);
    else if constexpr (J == 4 || J == 8) {
        const int up = __builtin_amdgcn_mov_dpp(v, 0x100 | J, 0xF, 0xF, true);  // row_shl: lane + J
        const int dn = __builtin_amdgcn_mov_dpp(v, 0x110 | J, 0xF, 0xF, true);  // row_shr: lane - J
        return (lane & J) ? dn : up;
    } else if constexpr (J == 16) return __builtin_amdgcn_ds_swizzle(v, 0x1F | (16 << 10));
    else return __shfl_xor(v, J);
}
template <int J>
__device__ __forceinline__ uint64_t xor_lane_u64(uint64_t v, int lane)
{
    const int lo = xor_lane<J>((int)(uint32_t)v, lane), hi = xor_lane<J>((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ void sort_keys_512(uint64_t* keys, int tid)
{
    static_assert(kSelThreads == 512, "eight runs of 64");
    const int lane = tid & 63, w = tid >> 6;
    uint64_t x = keys[tid];
    auto stage = [&](auto jc, int k) {
        constexpr int j = decltype(jc)::value;
        const uint64_t y = xor_lane_u64<j>(x, lane);
        const bool desc = (lane & k) == 0 || k == 64;
        const bool take_max = ((lane & j) == 0) == desc;
        x = take_max ? (x > y ? x : y) : (x < y ? x : y);
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    using I16 = std::integral_constant<int, 16>;
    using I32 = std::integral_constant<int, 32>;
    stage(I1{}, 2);
    stage(I2{}, 4), stage(I1{}, 4);
    stage(I4{}, 8), stage(I2{}, 8), stage(I1{}, 8);
    stage(I8{}, 16), stage(I4{}, 16), stage(I2{}, 16), stage(I1{}, 16);
    stage(I16{}, 32), stage(I8{}, 32), stage(I4{}, 32), stage(I2{}, 32), stage(I1{}, 32);
    stage(I32{}, 64), stage(I16{}, 64), stage(I8{}, 64), stage(I4{}, 64), stage(I2{}, 64), stage(I1{}, 64);
    keys[tid] = x;  // the wave's own run (no other wave reads or writes it yet)
    __syncthreads();
    int rank = lane;
    int pos[8];
    bool all[8];  // the whole run is ahead (a count of 64, which the 6-step search cannot reach)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint64_t c = keys[r * 64 + 63];
        all[r] = r < w ? c >= x : c > x;
        pos[r] = 0;
    }
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint64_t c = keys[r * 64 + pos[r] + st - 1];
            const bool ahead = r < w ? c >= x : c > x;
            pos[r] += ahead ? st : 0;
        }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) rank += r != w ? (all[r] ? 64 : pos[r]) : 0;
    __syncthreads();
    keys[rank] = x;
    __syncthreads();
}

// Bitonic sort of np2 keys in LDS only (every stage a compare-exchange pass
// over LDS pairs): the path for ROIs with more than 4 * kSelThreads candidates.
// Slower than sort_keys, but it keeps the kernel's register footprint at that
// of sort_keys<4> (the register-resident sorts of 8-32 keys per thread needed
// 169 VGPRs, which made every select workgroup wait for PyrLK waves to drain).
__device__ __forceinline__ void sort_keys_lds(uint64_t* keys, int np2, int tid)
{
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = tid; p < np2 / 2; p += kSelThreads) {
                const int e = ((p & ~(j - 1)) << 1) | (p & (j - 1));  // lower element of the pair
                const uint64_t x = keys[e], y = keys[e | j];
                const bool desc = (e & k) == 0;
                if (desc ? x < y : x > y) {
                    keys[e] = y;
                    keys[e | j] = x;
                }
            }
            __syncthreads();
        }
    }
}

// Greedy-walk distance test of one candidate against the byte image (image
// mode): for every window pixel closer than min_distance, 255 = an accepted
// corner (the candidate is rejected), 1..64 = a candidate of this step in lane
// v-1 (recorded in inb when it precedes this lane).  RAD is the window radius;
// all window rows are read before any is examined (one LDS round trip).
// Candidates sit on integer pixels, so "closer than min_distance" is the same
// set of window offsets for every candidate ((float)(dx*dx + dy*dy) < md2,
// featureselect.cpp:466-481 with integer dx, dy): one uniform byte mask per
// window row.  Byte values 1..64 never have the top bit that 255 has, so the
// rejection test is one mask over the row; only this step's candidates inside
// the mask are visited one by one.
template <int RAD>
__device__ __forceinline__ void window_test(const uint8_t* img, int rw, int rh, int ix, int iy, float fx, float fy,
                                            int lane, double md2, bool& good, unsigned long long& inb)
{
    constexpr int NR = 2 * RAD + 1;
    constexpr bool THREE = NR + 7 > 16;  // the shifted window can need a third word
    constexpr uint64_t kHi = 0x8080808080808080ull, kLo7 = 0x7F7F7F7F7F7F7F7Full;
    const int x0 = ix - RAD;
    if constexpr (RAD <= 2) {
        // windows of <= 5 bytes: one dword-aligned 8-byte read per row holds the
        // row's window after a shift of < 4 bytes, so each row is one 64-bit
        // word (the general path below shifts a 16-byte pair)
        uint64_t cv = 0;
#pragma unroll
        for (int t = 0; t < NR; ++t) {
            const int xx = x0 + t;
            cv |= ((xx >= 0 && xx < rw) ? 0xFFull : 0ull) << (8 * t);
        }
        uint64_t wv[NR];
        int sh[NR];
#pragma unroll
        for (int d = 0; d < NR; ++d) {
            const int yy = iy - RAD + d;
            const int yc = yy < 0 ? 0 : (yy >= rh ? rh - 1 : yy);
            const int base = yc * rw + x0;  // may be < 0 (first row, x0 < 0) or past the row: masked
            const int al = base > 0 ? (base & ~3) : 0;
            const uint32_t* wp = reinterpret_cast<const uint32_t*>(img + al);
            wv[d] = (uint64_t)wp[0] | ((uint64_t)wp[1] << 32);
            sh[d] = base - al;  // in [-RAD, 3]
        }
        uint64_t rej = 0;
#pragma unroll
        for (int d = 0; d < NR; ++d) {
            const int yy = iy - RAD + d;
            if (yy < 0 || yy >= rh) continue;
            uint64_t close = 0;
#pragma unroll
            for (int t = 0; t < NR; ++t) {
                const float ddx = (float)(t - RAD), ddy = (float)(d - RAD);
                close |= (((double)(ddx * ddx + ddy * ddy) < md2 && !(d == RAD && t == RAD)) ? 0xFFull : 0ull)
                         << (8 * t);
            }
            const uint64_t v = (sh[d] >= 0 ? wv[d] >> (8 * sh[d]) : wv[d] << (-8 * sh[d])) & cv & close;
            rej |= v & kHi;
            uint64_t nz = (((v & kLo7) + kLo7) | v) & ~v & kHi;
            while (nz) {
                const int t = __builtin_ctzll(nz) >> 3;
                nz &= nz - 1ull;
                const int c = (int)((v >> (8 * t)) & 0xFF);
                if (c - 1 < lane) inb |= 1ull << (c - 1);  // earlier in this step
            }
        }
        if (rej) good = false;
        (void)fx;
        (void)fy;
        return;
    }
    uint64_t cv_lo = 0, cv_hi = 0;  // 0xFF for window bytes whose column lies inside the ROI
#pragma unroll
    for (int t = 0; t < NR; ++t) {
        const int xx = x0 + t;
        const uint64_t b = (xx >= 0 && xx < rw) ? 0xFFull : 0ull;
        if (t < 8) cv_lo |= b << (8 * t);
        else cv_hi |= b << (8 * (t - 8));
    }
    uint64_t w0[NR], w1[NR], w2[NR];
    int sh[NR];
#pragma unroll
    for (int d = 0; d < NR; ++d) {
        const int yy = iy - RAD + d;
        const int yc = yy < 0 ? 0 : (yy >= rh ? rh - 1 : yy);  // out-of-ROI rows: read any row, masked below
        const int base = yc * rw + x0;                       // may be < 0 or past the row: masked
        const int al = base > 0 ? (base & ~7) : 0;
        const uint64_t* wp = reinterpret_cast<const uint64_t*>(img + al);
        w0[d] = wp[0];
        w1[d] = wp[1];
        w2[d] = THREE ? wp[2] : 0ull;
        sh[d] = base - al;  // in [-RAD, 7]
    }
    uint64_t rej = 0;
#pragma unroll
    for (int d = 0; d < NR; ++d) {
        const int yy = iy - RAD + d;
        if (yy < 0 || yy >= rh) continue;
        // uniform: the offsets of this row closer than min_distance
        uint64_t close_lo = 0, close_hi = 0;
#pragma unroll
        for (int t = 0; t < NR; ++t) {
            const float ddx = (float)(t - RAD), ddy = (float)(d - RAD);
            const uint64_t b = ((double)(ddx * ddx + ddy * ddy) < md2 && !(d == RAD && t == RAD)) ? 0xFFull : 0ull;
            if (t < 8) close_lo |= b << (8 * t);
            else close_hi |= b << (8 * (t - 8));
        }
        uint64_t lo, hi;
        if (sh[d] >= 0) {
            const int b8 = 8 * sh[d];
            lo = sh[d] ? (w0[d] >> b8) | (w1[d] << (64 - b8)) : w0[d];
            hi = sh[d] ? (w1[d] >> b8) | (w2[d] << (64 - b8)) : w1[d];
        } else {  // window starts before the image (first row, x0 < 0)
            const int b8 = -8 * sh[d];
            lo = w0[d] << b8;
            hi = (w1[d] << b8) | (w0[d] >> (64 - b8));
        }
        lo &= cv_lo & close_lo;
        hi &= cv_hi & close_hi;
        rej |= (lo | hi) & kHi;  // an accepted corner (255) closer than min_distance
        // this step's candidates (1..64) in the mask: nonzero bytes without the top bit
        uint64_t nz_lo = (((lo & kLo7) + kLo7) | lo) & ~lo & kHi;
        uint64_t nz_hi = (((hi & kLo7) + kLo7) | hi) & ~hi & kHi;
        while (nz_lo | nz_hi) {
            int t;
            uint64_t src;
            if (nz_lo) {
                t = __builtin_ctzll(nz_lo) >> 3;
                nz_lo &= nz_lo - 1ull;
                src = lo;
            } else {
                t = __builtin_ctzll(nz_hi) >> 3;
                nz_hi &= nz_hi - 1ull;
                src = hi;
                t += 8;
            }
            const int v = (int)((src >> (8 * (t & 7))) & 0xFF);
            if (v - 1 < lane) inb |= 1ull << (v - 1);  // earlier in this step
        }
    }
    if (rej) good = false;
    (void)fx;
    (void)fy;
}

// Partial selection (round 3): the greedy walk consumes the candidates in
// descending key order and stops after max_corners accepted corners, typically
// ~280 of ~700 candidates (1080p x 128 bench boxes: at most 312 of up to 2082).
// Instead of sorting all of them, the 448 largest keys (plus the ties of the
// 16-bit key prefix that reaches them) are found by a two-pass radix select on
// the key's top 16 bits, moved to the front, and only they are sorted (512
// keys); the others wait, unsorted, behind them.  Should the walk run out of
// the sorted part before it is done, it takes the rest in descending order 64
// at a time (wave-wide max selection); the walk's result does not depend on
// how the candidates are batched, so the corners are the same.
#ifndef TBDK_GFTT_PARTIAL
#define TBDK_GFTT_PARTIAL 1  // 0: sort every candidate (A/B builds)
#endif
constexpr int kSelTarget = 448;
constexpr int kSelRegs = 8;  // keys per thread held in registers while partitioning

// wave 0: the bin where the running count from the top first reaches target,
// and the count of keys in the bins above it (hist: 256 bins in LDS)
__device__ __forceinline__ void radix_pick(const int* hist, int target, int lane, int* out_bin, int* out_above)
{
    int h[4], t = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        h[u] = hist[4 * lane + u];
        t += h[u];
    }
    int suf = t;  // inclusive suffix sum over lanes >= lane
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_down(suf, d, 64);
        suf += lane + d < 64 ? o : 0;
    }
    int above = suf - t;  // keys in the bins of the lanes above
    if (above < target && suf >= target) {
#pragma unroll
        for (int u = 3; u >= 0; --u) {
            if (above + h[u] >= target) {
                *out_bin = 4 * lane + u;
                *out_above = above;
                break;
            }
            above += h[u];
        }
    }
}

// wave 0: the next (up to) 64 largest keys of an unsorted array (taken keys
// are zeroed), lane l receiving the l-th; 0 when none is left
__device__ uint64_t take_next64(uint64_t* rest, int nrest, int lane)
{
    uint64_t mine = 0ull;
    for (int c = 0; c < 64; ++c) {
        uint64_t best = 0ull;
        int bi = -1;
        for (int j = lane; j < nrest; j += 64) {
            const uint64_t v = rest[j];
            if (v > best) {
                best = v;
                bi = j;
            }
        }
        uint64_t m = best;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint64_t o = shfl_xor_u64(m, d);
            m = o > m ? o : m;
        }
        if (m == 0ull) break;  // wave-uniform
        if (bi >= 0 && best == m) rest[bi] = 0ull;  // keys are unique: one owner
        if (lane == c) mine = m;
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
    return mine;
}

// LDS layout of the select kernel (one dynamic region):
//   keys  : cap uint64 sort keys
//   acc   : max_corners float2 accepted positions + 64 float2 (list mode)
//   img   : img_bytes, one byte per ROI pixel (image mode): 0 empty,
//           1..64 candidate of the current step (lane + 1), 255 accepted corner
// RMAX: the largest distance-window radius this instance handles (the walk's
// window rows are register arrays: radius 6 needs 156 VGPRs, radius 2 68, and
// a select workgroup's eight waves only find room next to PyrLK waves at the
// smaller size); the host picks the instance from min_distance.
template <int RMAX>
__global__ __launch_bounds__(kSelThreads) void gftt_select_kernel(GfttArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t* keys = reinterpret_cast<uint64_t*>(smem);
    float2* acc = reinterpret_cast<float2*>(keys + a.cap);
    float2* bxy = acc + a.max_corners;
    uint8_t* img = reinterpret_cast<uint8_t*>(acc + ((a.max_corners + 65) & ~1));  // 16-byte aligned
    const int r = blockIdx.x;
    const GfttRoi R = roi_at(a, r);
    const int tid = threadIdx.x;
    __shared__ int s_total;
    GFTT_STAMP(0);
    const int area = R.w * R.h;
    // image mode: the ROI's byte image fits and the distance window is small
    const bool use_dist = a.min_distance >= 1.0;
    const double md2 = a.min_distance * a.min_distance;
    int rad = (int)ceil(a.min_distance) - 1;  // |d| <= rad can be closer than min_distance
    if ((double)(rad + 1) * (rad + 1) < md2) rad++;
    const bool img_mode = use_dist && area <= a.img_bytes && rad <= 6;
    if (img_mode)
        for (int i = tid * 16; i < area; i += kSelThreads * 16) *reinterpret_cast<uint4*>(img + i) = make_uint4(0, 0, 0, 0);

    // ---- candidates (featureselect.cpp: threshold-to-zero at max*q, 3x3
    // dilate, interior pixels equal to the dilation): ROI max = max of its
    // strips' maxima; with max > 0 (so thr > 0) a pixel is a candidate iff its
    // value > thr and it is >= all 8 neighbours (any larger neighbour exceeds
    // thr too), i.e. its local-maximum bit from the eigenvalue walk is set.
    // thr <= 0 (no positive eigenvalue in the ROI): the literal test.
    // this thread's first local-maximum word is loaded together with the strip
    // maxima (the threshold needs all of them; the word needs none): one global
    // round trip fewer before the value loads
    const int nstrip = (R.w + kGfttStrip - 1) / kGfttStrip;
    const int nw = R.w >= 3 && R.h >= 3 ? nstrip * R.h : 0;
    const uint64_t word0 = tid < nw ? a.lmax[R.moff + tid] : 0ull;
    int mk = INT_MIN;
    {
        int b = R.cblk;
        const int e = R.cblk + nstrip;
        for (; b + 4 <= e; b += 4) {  // four maxima in flight
            const int m0 = a.blk_max[b], m1 = a.blk_max[b + 1], m2 = a.blk_max[b + 2], m3 = a.blk_max[b + 3];
            mk = max(max(mk, max(m0, m1)), max(m2, m3));
        }
        for (; b < e; ++b) mk = a.blk_max[b] > mk ? a.blk_max[b] : mk;
    }
    const float thr = (float)((double)fkey_inv(mk) * a.quality);
    if (tid == 0) s_total = 0;
    __syncthreads();
    const float* Ep = a.eig + R.off;
    if (R.w >= 3 && R.h >= 3) {
        if (thr > 0.f) {
            for (int wi = tid; wi < nw; wi += kSelThreads) {
                const int st = wi / R.h, y = wi - st * R.h;
                if (y < 1 || y > R.h - 2) continue;
                uint64_t word = wi == tid ? word0 : a.lmax[R.moff + wi];
                const float* Er = Ep + (size_t)y * gftt_epitch(R.w) + st * kGfttStrip - kGfttHalo;
                // compact: the word's values packed in bit order at the strip row's first columns
                const float* Ec = Er + kGfttHalo;
                int rk = 0;
                while (word) {  // up to 8 value loads in flight per round
                    int xs[8];
                    float vs[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        xs[u] = -1;
                        if (word) {
                            xs[u] = __builtin_ctzll(word);
                            word &= word - 1ull;
                            vs[u] = a.compact ? Ec[rk++] : Er[xs[u]];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (xs[u] >= 0 && vs[u] > thr) {
                            const int q = atomicAdd(&s_total, 1);
                            if (q < a.cap) keys[q] = cand_key(vs[u], y, st * kGfttStrip + xs[u] - kGfttHalo);
                        }
                    }
                }
            }
        } else if (!a.compact) {
            // (compact mode runs with quality <= 1 only: thr = max * q >= max when
            // max <= 0, so no value exceeds thr and the ROI has no candidate)
            const int iw = R.w - 2, n = iw * (R.h - 2), ep = gftt_epitch(R.w);
            for (int p = tid; p < n; p += kSelThreads) {
                const int y = p / iw + 1, x = p - (y - 1) * iw + 1;
                const float* Ec = Ep + (size_t)y * ep + x;
                const float v = Ec[0] > thr ? Ec[0] : 0.f;
                if (v == 0.f) continue;
                float m = v;
#pragma unroll
                for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                    for (int dx = -1; dx <= 1; ++dx) {
                        const float q0 = Ec[dy * ep + dx];
                        const float q = q0 > thr ? q0 : 0.f;
                        m = q > m ? q : m;
                    }
                if (v == m) {
                    const int q = atomicAdd(&s_total, 1);
                    if (q < a.cap) keys[q] = cand_key(v, y, x);
                }
            }
        }
    }
    __syncthreads();
    GFTT_STAMP(4);
    const int total = s_total;
    if (total > a.cap) {  // candidate buffer overflow: report, never silently truncate
        if (tid == 0) a.counts[r] = -1;
        return;
    }
    // ---- partial selection (see kSelTarget): the largest keys to the front
    int S = total, nrest = 0;  // sorted part keys[0, S); the rest keys[kSelThreads, kSelThreads + nrest)
    if (TBDK_GFTT_PARTIAL && total > kSelThreads && total <= kSelRegs * kSelThreads && total + kSelThreads + 64 <= a.cap) {
        __shared__ int hist[256];
        __shared__ int s_pick[4];  // first-pass bin, keys above it; prefix, S
        __shared__ int s_cnt[2];
        if (tid < 256) hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < total; i += kSelThreads) atomicAdd(&hist[(int)(keys[i] >> 56)], 1);
        __syncthreads();
        if (tid < 64) radix_pick(hist, kSelTarget, tid, &s_pick[0], &s_pick[1]);
        __syncthreads();
        const int b1 = s_pick[0], above1 = s_pick[1];
        if (tid < 256) hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < total; i += kSelThreads) {
            const uint64_t k = keys[i];
            if ((int)(k >> 56) == b1) atomicAdd(&hist[(int)(k >> 48) & 255], 1);
        }
        __syncthreads();
        if (tid < 64) {
            // second pass: the bin within b1 (the lane that holds it writes)
            int b2 = -1, above2 = 0;
            radix_pick(hist, kSelTarget - above1, tid, &b2, &above2);
            if (b2 >= 0) {
                s_pick[2] = (b1 << 8) | b2;
                s_pick[3] = above1 + above2 + hist[b2];
            }
        }
        if (tid == 0) s_cnt[0] = s_cnt[1] = 0;
        __syncthreads();
        const int sel = s_pick[3];
        if (sel <= kSelThreads) {  // else: a wide tie of key prefixes, sort everything
            const uint32_t t16 = (uint32_t)s_pick[2];
            uint64_t kr[kSelRegs];
#pragma unroll
            for (int u = 0; u < kSelRegs; ++u) {
                const int i = tid + u * kSelThreads;
                kr[u] = i < total ? keys[i] : 0ull;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kSelRegs; ++u) {
                if (tid + u * kSelThreads >= total) continue;
                if ((uint32_t)(kr[u] >> 48) >= t16) keys[atomicAdd(&s_cnt[0], 1)] = kr[u];
                else keys[kSelThreads + atomicAdd(&s_cnt[1], 1)] = kr[u];
            }
            __syncthreads();
            S = sel;
            nrest = total - sel;
        }
    }
    GFTT_STAMP(5);
    int np2 = kSelThreads;
    while (np2 < S) np2 <<= 1;
    for (int i = S + tid; i < np2; i += kSelThreads) keys[i] = 0ull;  // sorts last
    __syncthreads();
    GFTT_STAMP(1);
    switch (np2 / kSelThreads) {
    case 1: sort_keys_512(keys, tid); break;
    case 2: sort_keys<2>(keys, np2, tid); break;
    case 4: sort_keys<4>(keys, np2, tid); break;
    default: sort_keys_lds(keys, np2, tid); break;
    }
    GFTT_STAMP(2);
    if (tid >= 64) return;
    // the walk is one wave's serial chain on the frame's critical path: ahead of
    // the throughput-bound PyrLK waves sharing its SIMD for instruction issue
    // (+0.6 % frames/s in three alternating loop runs out of three)
    __builtin_amdgcn_s_setprio(TBDK_GFTT_WALK_PRIO);

    // ---- greedy walk in sorted order (featureselect.cpp:421-503), 64 candidates per step
    const int lane = tid;
    const int maxc = a.max_corners;
    float2* out = a.corners + (size_t)r * a.corner_stride;
    int n = 0;
    bool done = false;
    GFTT_TDECL;
    int i0 = 0, rem = nrest;
    while (!done) {
        GFTT_T(0);
        // the sorted part 64 at a time, then (rarely) the rest in descending order
        uint64_t key;
        bool valid;
        if (i0 < S) {
            const int i = i0 + lane;
            valid = i < S;
            key = valid ? keys[i] : 0ull;
            i0 += 64;
        } else {
            if (rem <= 0) break;  // wave-uniform
            key = take_next64(keys + kSelThreads, nrest, lane);
            valid = key != 0ull;
            rem -= 64;
        }
        const uint32_t kk = (uint32_t)key;
        const int ix = (int)(kk & 0xFFFF), iy = (int)(kk >> 16);
        const float fx = (float)ix, fy = (float)iy;
        bool good = valid;
        unsigned long long inb = 0ull;  // earlier lanes of this step closer than min_distance
        if (img_mode) {
            if (valid) img[iy * R.w + ix] = (uint8_t)(lane + 1);
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            GFTT_T(1);
            if (valid) {
                switch (rad) {  // uniform; rad <= RMAX (host)
                case 0: window_test<0>(img, R.w, R.h, ix, iy, fx, fy, lane, md2, good, inb); break;
                case 1: window_test<1>(img, R.w, R.h, ix, iy, fx, fy, lane, md2, good, inb); break;
                case 2: window_test<2>(img, R.w, R.h, ix, iy, fx, fy, lane, md2, good, inb); break;
                default:
                    if constexpr (RMAX > 2) {
                        switch (rad) {
                        case 3: window_test<3>(img, R.w, R.h, ix, iy, fx, fy, lane, md2, good, inb); break;
                        case 4: window_test<4>(img, R.w, R.h, ix, iy, fx, fy, lane, md2, good, inb); break;
                        case 5: window_test<5>(img, R.w, R.h, ix, iy, fx, fy, lane, md2, good, inb); break;
                        default: window_test<6>(img, R.w, R.h, ix, iy, fx, fy, lane, md2, good, inb); break;
                        }
                    }
                    break;
                }
            }
        } else if (use_dist) {  // list mode: every accepted corner, then this step's pairs
            bxy[lane] = make_float2(fx, fy);
            for (int q = 0; q < n && good; ++q) {
                const float2 pq = acc[q];
                const float dx = fx - pq.x, dy = fy - pq.y;
                if ((double)(dx * dx + dy * dy) < md2) good = false;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            for (int j = 0; j < lane; ++j) {
                const float2 pj = bxy[j];
                const float dx = fx - pj.x, dy = fy - pj.y;
                if ((double)(dx * dx + dy * dy) < md2) inb |= 1ull << j;
            }
        }
        // sequential acceptance: lanes without in-step dependencies are final;
        // the others, in order, are accepted iff no accepted earlier lane conflicts
        GFTT_T(2);
        const unsigned long long goodm = __ballot(good);
        const unsigned long long depm = __ballot(good && inb != 0ull);
        unsigned long long accm = goodm & ~depm;
        unsigned long long pend = depm;
        while (pend) {
            const int k = __builtin_ctzll(pend);
            pend &= pend - 1ull;
            const unsigned long long ik =
                ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(inb >> 32), k) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)inb, k);
            if (!(ik & accm)) accm |= 1ull << k;
        }
        GFTT_T(3);
        // maxCorners: only the first (maxc - n) accepted of this step count
        const int got = __popcll(accm);
        if (n + got >= maxc) {
            int keepn = maxc - n;
            unsigned long long m = accm, t = 0ull;
            while (keepn-- > 0) {
                const unsigned long long low = m & (~m + 1ull);
                t |= low;
                m &= m - 1ull;
            }
            accm = t;
            done = true;
        }
        GFTT_T(4);
        const bool mine = (accm >> lane) & 1ull;
        if (mine) {
            const int pos = n + __popcll(accm & ((1ull << lane) - 1ull));
            if (!img_mode) acc[pos] = make_float2(fx, fy);
            out[pos] = make_float2(fx + (float)R.x, fy + (float)R.y);
        }
        if (img_mode && valid) img[iy * R.w + ix] = mine ? (uint8_t)255 : (uint8_t)0;
        n += __popcll(accm);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): img[] / acc[] visible to the next step
        __builtin_amdgcn_wave_barrier();
        GFTT_T(5);
    }
    GFTT_TDUMP;
    GFTT_STAMP(3);
    if (lane == 0) a.counts[r] = n;
}

size_t gftt_select_smem(int cap, int max_corners, int img_bytes)
{
    return sizeof(uint64_t) * (size_t)cap +
           sizeof(float2) * (size_t)((max_corners + 65) & ~1) + (size_t)img_bytes + 32;  // + window over-read
}

// LDS plan: the byte image for ROIs up to max_area pixels when that leaves
// room for >= 4096 sort keys, else list mode with the largest key array
void gftt_plan(GfttArgs& a, int max_area)
{
    const long lds = 160L * 1024 - 2048;  // static LDS (counters, radix histogram) stays out of the dynamic budget
    const long fixed = (long)gftt_select_smem(0, a.max_corners, 0);
    long img = ((long)max_area + 15) & ~15L;
    long room = lds - fixed - img;
    if (room < 8L * 4096) {
        img = 0;
        room = lds - fixed;
    }
    int cap = 512;
    while (cap < kGfttCap && 8L * cap * 2 <= room) cap <<= 1;
    a.cap = cap;
    a.img_bytes = (int)img;
}

hipError_t launch_gftt_eig(const GfttArgs& a, hipStream_t s)
{
    if (a.compact) hipLaunchKernelGGL(gftt_eig_kernel<true>, dim3(a.ncblk), dim3(64 * kEigWaves), 0, s, a);
    else hipLaunchKernelGGL(gftt_eig_kernel<false>, dim3(a.ncblk), dim3(64 * kEigWaves), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_gftt(const GfttArgs& a, hipStream_t s, hipEvent_t after_eig)
{
    const hipError_t e0 = launch_gftt_eig(a, s);
    if (e0 != hipSuccess) return e0;
    if (after_eig) {
        const hipError_t e = hipEventRecord(after_eig, s);
        if (e != hipSuccess) return e;
    }
    return launch_gftt_select(a, s);
}

hipError_t launch_gftt_select(const GfttArgs& a, hipStream_t s)
{
    const size_t smem = gftt_select_smem(a.cap, a.max_corners, a.img_bytes);
    // > 64 KiB of dynamic LDS must be opted into (160 KiB per CU on gfx950);
    // done once per device, for the whole LDS, off the per-frame path
    static std::atomic<unsigned long long> opted{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(opted.load(std::memory_order_acquire) & bit)) {
        for (const void* k : {reinterpret_cast<const void*>(&gftt_select_kernel<2>),
                              reinterpret_cast<const void*>(&gftt_select_kernel<6>)}) {
            hipFuncAttributes fa;
            e = hipFuncGetAttributes(&fa, k);
            if (e != hipSuccess) return e;
            e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(160L * 1024 - (long)fa.sharedSizeBytes));
            if (e != hipSuccess) return e;
        }
        opted.fetch_or(bit, std::memory_order_acq_rel);
    }
    // the distance window's radius, as the kernel derives it
    const double md2 = a.min_distance * a.min_distance;
    int rad = (int)ceil(a.min_distance) - 1;
    if ((double)(rad + 1) * (rad + 1) < md2) rad++;
    if (a.min_distance >= 1.0 && rad > 2)
        hipLaunchKernelGGL(gftt_select_kernel<6>, dim3(a.nroi), dim3(kSelThreads), smem, s, a);
    else
        hipLaunchKernelGGL(gftt_select_kernel<2>, dim3(a.nroi), dim3(kSelThreads), smem, s, a);
    return hipGetLastError();
}

}  // namespace tbdk
