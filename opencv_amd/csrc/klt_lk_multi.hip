// klt_lk_multi.hip — sparse pyramidal LK with several points per wave (gfx950).
//
// Same algorithm and bit-identical results as klt_lk_strip.hip / klt_lk.hip
// (CPU calcOpticalFlowPyrLK numerics, LKTrackerInvoker video/src/lkpyramid.cpp:178-695,
// exact integer sums rounded once to float), laid out so that the per-point
// bookkeeping of a Newton step is shared by P = 64 / WW points:
//   * lane = one window column x of one point: point k of the wave owns lanes
//     [1 + k*WW, 1 + (k+1)*WW) (win 21: 3 points, lane 0 idle), and each lane
//     keeps all WH rows of its column (I patch x32, interpolated Scharr Ix/Iy,
//     the J column pairs) in VGPRs for every Newton iteration of the level;
//   * the bilinear weights, the 2x2 solve and the stopping tests run once per
//     lane for all P points at the cost of one (they are per-point values held
//     by every lane of the point), where the one-point-per-wave kernel spends a
//     wave-wide instruction on a single point's scalar math;
//   * per-point sums over the point's WW lanes: prefix scans over the wave with
//     six DPP adds (row_shr 1/2/4/8, row_bcast 15/31), each lane reading its
//     point's segment (end - start) back by ds_bpermute; exact for any window
//     by a lo/hi split of every partial with the hi parts of up to three sums
//     packed into one scan (seg_sum_exact), rounded once to float — the same
//     value as the exact int64 sum of the other kernels;
//   * control flow stays wave-uniform (levels, Newton steps while any point is
//     active, J reloads when any point's integer origin moved), so every DPP and
//     bpermute runs with all lanes on; a point that stopped keeps its values by
//     selects.
#include <type_traits>

#include "lk_device.hpp"

namespace tbdk {

namespace {

using namespace lkdev;

// inclusive prefix sum over the 64 lanes (all lanes active), modulo 2^32
__device__ __forceinline__ uint32_t scan64(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// M independent scans advanced step by step together: each DPP reads a value
// written two or more instructions earlier, so no wait states are needed
// between the dependent adds of one scan (a lone scan64 needs one per step)
template <int M>
__device__ __forceinline__ void scan64_n(uint32_t (&v)[M])
{
#define TBDK_SCAN_STEP(ctrl, rmask, bc)                                                                    \
    _Pragma("unroll") for (int m = 0; m < M; ++m) v[m] +=                                                  \
        (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[m], ctrl, rmask, 0xF, bc);
    TBDK_SCAN_STEP(0x111, 0xF, true)   // row_shr:1
    TBDK_SCAN_STEP(0x112, 0xF, true)   // row_shr:2
    TBDK_SCAN_STEP(0x114, 0xF, true)   // row_shr:4
    TBDK_SCAN_STEP(0x118, 0xF, true)   // row_shr:8
    TBDK_SCAN_STEP(0x142, 0xA, false)  // row_bcast:15 -> rows 1, 3
    TBDK_SCAN_STEP(0x143, 0xC, false)  // row_bcast:31 -> rows 2, 3
#undef TBDK_SCAN_STEP
}

// segment total of a scanned value: prefix at the point's last lane minus the
// prefix at the lane before its first (lane 0 is idle and holds 0, so every
// point has such a lane)
__device__ __forceinline__ uint32_t seg_total(uint32_t scanned, int e4, int s4)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute(e4, (int)scanned) -
           (uint32_t)__builtin_amdgcn_ds_bpermute(s4, (int)scanned);
}

// Exact per-point sums of N <= 3 int32 lane partials (|partial| < 2^30): every
// lane gets its own point's sum, rounded once to float.  Each partial is split
// as hi * 2^26 + lo (0 <= lo < 2^26, -16 <= hi < 16).  The lo parts are scanned
// one per value (a point's lo total is below 21 * 2^26 < 2^31, exact as a
// modulo-2^32 difference); the hi parts of all N values share ONE scan, packed
// in 11-bit fields (a point's hi total lies in [-16*21, 15*21] and every field
// below the top one is recovered by sign extension).  hi * 2^26 + lo in double
// is the exact integer sum; the one float rounding gives the same value as the
// exact int64 sum of the other kernels.  e4 / s4: byte addresses of the point's
// last lane and of the lane before its first.
//
// Fast path, taken by the whole wave when every partial lies in (-2^FB, 2^FB):
// a point's total is then below 31 * 2^26 < 2^31 in magnitude (FB 26: windows
// up to 31 wide), or 63 * 2^25 (FB 25: a point spread over all 63 lanes, the
// one-point steps below), exact as a modulo-2^32 difference of plain scans, and
// its int -> float conversion is the same single rounding.  The split path
// holds for segments of up to 63 lanes (lo totals below 63 * 2^26 < 2^32, hi
// totals in [-16 * 63, 15 * 63], inside an 11-bit field).
template <int N, int FB = 26>
__device__ __forceinline__ void seg_sum_exact(const int (&v)[N], int e4, int s4, float (&out)[N], bool* split = nullptr)
{
    static_assert(N >= 1 && N <= 3, "three 11-bit fields per packed scan");
    static_assert(FB <= 26, "hi parts are v >> 26");
    bool big = false;
#pragma unroll
    for (int k = 0; k < N; ++k) big |= (uint32_t)v[k] + (1u << FB) >= (2u << FB);
    const bool slow = __builtin_amdgcn_ballot_w64(big) != 0;  // wave-uniform
    if (split) *split = slow;
    if (!slow) {
        uint32_t sv[N];
#pragma unroll
        for (int k = 0; k < N; ++k) sv[k] = (uint32_t)v[k];
        scan64_n(sv);
#pragma unroll
        for (int k = 0; k < N; ++k) out[k] = (float)(int)seg_total(sv[k], e4, s4);
        return;
    }
    uint32_t sc[N + 1];  // lo parts, then the packed hi parts
    sc[N] = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        sc[k] = (uint32_t)v[k] & 0x3FFFFFFu;
        sc[N] += (uint32_t)(v[k] >> 26) << (11 * k);
    }
    scan64_n(sc);
    int h = (int)seg_total(sc[N], e4, s4);
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int hk = k + 1 < N ? (int)((uint32_t)h << 21) >> 21 : h;  // sign-extended low field
        h = (h - hk) >> 11;
        const uint32_t l = seg_total(sc[k], e4, s4);
        out[k] = (float)((double)hk * 67108864.0 + (double)l);  // exact in double, one rounding
    }
}

// per-point sum of small lane values (no split: |total| < 2^31)
__device__ __forceinline__ int seg_sum_small(int v, int e4, int s4)
{
    return (int)seg_total(scan64((uint32_t)v), e4, s4);
}

// p0 . w0 + p1 . w1 + c: the reference's bilinear sum started from a per-row
// VGPR constant (the three-operand v_dot2_i32_i16 keeps c; the compiler
// otherwise copies c and accumulates with v_dot2c)
__device__ __forceinline__ int bilin_c(uint32_t p0, uint32_t p1, uint32_t w0, uint32_t w1, int c)
{
    int t;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(t) : "v"(p1), "v"(w1), "v"(c));
    return sdot2(p0, w0, t);
}

// (t0 >> SH, t1 >> SH) as int16 x 2 in two instructions: t0 >> SH, then the
// SDWA form of the second shift writes only the high word (WORD_1) of the
// result, keeping the low word
template <int SH>
__device__ __forceinline__ uint32_t pack_shr(int t0, int t1)
{
    uint32_t d = (uint32_t)(t0 >> SH);
    asm("v_ashrrev_i32_sdwa %0, %2, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(d)
        : "v"(t1), "i"(SH));
    return d;
}
__device__ __forceinline__ uint32_t pack_diff(int t0, int t1) { return pack_shr<9>(t0, t1); }

__device__ __forceinline__ bool any_lane(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }


}  // namespace

// waves per workgroup (tuning builds may change it; the kernel uses no LDS, so
// one-wave workgroups let a finished wave's slot be refilled at once)
// I x32 kept as packed row pairs and subtracted from the J pairs by one packed
// op per row pair (1), or folded into each row's J rounding constant (0, one
// VGPR per row; tuning builds)
// How I enters the Newton step's b sums (tuning builds may change it):
//   0: folded into each row's J rounding constant (one VGPR per row)
//   1: I pairs packed by rows, one v_pk_sub per row pair and step
//   2: b = sum(Jd * g) - sum(I * g): the second sum (per lane, per level) is
//      made once in the level setup, so the step needs no I at all; the final
//      error recomputes the I rows from the level
#ifndef TBDK_LK_IPACK
#define TBDK_LK_IPACK 1  // derivative-plane instance (94 VGPRs -> 5 waves per SIMD)
#endif
#ifndef TBDK_LK_IPACK_FLY
#define TBDK_LK_IPACK_FLY 0  // Scharr-on-the-fly instance
#endif

#ifndef TBDK_LK_MULTI_WAVES
#define TBDK_LK_MULTI_WAVES 1
#endif
// The interpolated (Ix, Iy) row pairs of the level (constant through its Newton
// steps) kept in LDS instead of VGPRs (1): the level setup writes them once, each
// step reads them back (one ds_read_b64 per row pair), so the kernel's register
// peak drops by 2 * NP VGPRs and more waves fit per SIMD (tuning builds: 0 keeps
// them in VGPRs)
#ifndef TBDK_LK_GLDS
#define TBDK_LK_GLDS 0
#endif
// A launch ends with its slowest wave: the few points that run to 30 Newton
// steps on a level (and the waves that carry them) finish long after the
// rest.  A wave that has taken more than TBDK_LK_PRIO_STEPS steps raises its
// issue priority (s_setprio), so on a shared SIMD its instructions go first and
// the straggler runs near its lone-wave speed (0: off)
#ifndef TBDK_LK_PRIO_STEPS
#define TBDK_LK_PRIO_STEPS 0
#endif
constexpr int kMultiWaves = TBDK_LK_MULTI_WAVES;

// Probe builds (-DTBDK_LK_TRACE, tools/probe_lk_trace.py): every wave writes
// one record of sixteen u64 (at its launch's base + its wave index, no atomics:
// a device-wide atomic counter serialises the waves' exits) to a device buffer
// set by tbdk_probe_lk_trace():
// start / end (s_memrealtime, 100 MHz), HW_ID | XCC_ID << 32, n << 32 | wave,
// the launch's point-list key, Newton steps | reloads << 16 | max iters << 32,
// then 16 u32 phase stamps (ticks after start): per level L, [4L] its start,
// [4L+1] the setup's G sums done, [4L+2] the first J window loaded (the probe
// waits for it there), [4L+3] its Newton steps done; [12] the error pass done;
// [13] the point's coordinates arrived (start: the wave's first instruction),
// [14] the first level's source rows arrived (FLY; the probe waits for them
// there), [15] its window terms done (before the G sums); bits 48.. of the
// steps word: the levels whose G sums took seg_sum_exact's split path.  Not in
// the product library.
#ifdef TBDK_LK_TRACE
__device__ unsigned long long* g_lk_trace;
__device__ unsigned int g_lk_trace_cap;
static unsigned g_lk_trace_next;  // host: records handed out so far
#endif

#ifdef TBDK_LK_MULTI_MINW  // waves per SIMD the register allocation must allow (tuning builds)
#define TBDK_MULTI_BOUNDS __launch_bounds__(64 * TBDK_LK_MULTI_WAVES, TBDK_LK_MULTI_MINW)
#else
#define TBDK_MULTI_BOUNDS __launch_bounds__(64 * TBDK_LK_MULTI_WAVES)
#endif

// FLY: the Scharr derivatives of the window are computed from the u8 level in
// the level setup instead of read from the pyramid's derivative planes (same
// values; the planes need not exist).
// DENSE (klt_dense.hip, cv::cuda::DensePyrLKOpticalFlow): the points are the
// pixel grid, and a point's interpolated window (I x32, Ix, Iy) is read from
// the level's case images instead of interpolated in the setup: the window of
// pixel (x, y) at level L has the sub-pixel phase (x mod 2^L, y mod 2^L) / 2^L
// and origin (x >> L, y >> L) - half, so every window element is element
// (y >> L) - half + r, (x >> L) - half + c of the case image of that phase,
// the same integers the planes setup computes (the phase's weights applied to
// the same pyramid and derivative-plane values).  The Newton steps are this
// kernel's.  Outputs: the flow (next - pixel) and the status plane.
template <int WW, int WH, bool FLY, bool DENSE = false>
__global__ TBDK_MULTI_BOUNDS void lk_multi_kernel(LkArgs a)
{
    static_assert(!DENSE || (!FLY && TBDK_LK_IPACK == 1), "dense mode: the planes instance's packed I pairs");
    constexpr int P = 64 / WW;         // points per wave
    constexpr int NP = (WH + 1) / 2;   // packed row pairs (rows 2q, 2q+1)
    constexpr int IM = FLY ? TBDK_LK_IPACK_FLY : TBDK_LK_IPACK;
    constexpr bool IPACK = IM == 1, ILIN = IM == 2;
    constexpr bool GL = TBDK_LK_GLDS != 0;
    constexpr bool kSoloOk = P >= 2 && !GL && !ILIN;  // one-point steps (LkArgs::solo_min)
    // GL: this wave's (Ix, Iy) row pairs, [row pair][lane] (8 B per lane: b64 accesses)
    __shared__ uint2 sg[GL ? NP * kMultiWaves : 1][64];
    const int lane = threadIdx.x & 63;
    uint2(*const sgw)[64] = &sg[GL ? (threadIdx.x >> 6) * NP : 0];
    // point k of the wave owns lanes [1 + k*WW, 1 + (k+1)*WW); lane 0 (and any
    // lane past the last point) is idle with k == P and contributes 0
    const int k = lane == 0 ? P : (lane - 1) / WW;
    const int x = k < P ? lane - 1 - k * WW : 0;
    const int wave = xcd_swizzle(blockIdx.x, gridDim.x) * kMultiWaves + (threadIdx.x >> 6);
    // the point's index in a segmented list (seg_point) and its coordinates: the
    // segment's count and the point are loaded together, the point speculatively
    // (index s * stride + j lies inside segment s's stride-sized row of the
    // loop's point buffers whether or not j < count), so a wave's start pays one
    // memory round trip before its first level's rows, not two
#ifdef TBDK_LK_TRACE
    const unsigned long long tr_t0 = __builtin_amdgcn_s_memrealtime();  // the wave's first instruction
#endif
    int i = -1;
    float p0x = 0.f, p0y = 0.f;
    if constexpr (DENSE) {
        i = k < P && wave * P + k < a.n ? wave * P + k : -1;
    } else {
        const int kk = wave * P + k;
        if (k < P && kk < a.n) {
            if (!a.seg_counts) {
                i = kk;
                p0x = a.prev_pts[2 * i];
                p0y = a.prev_pts[2 * i + 1];
            } else {
                const int seg = kk / a.seg_stride, j = kk - seg * a.seg_stride;
                const int s = a.seg_ninl > 0 ? (int)a.seg_inl[seg] : a.seg_list ? a.seg_list[seg] : seg;
                const int cand = s * a.seg_stride + j;
                const int cnt = a.seg_counts[s];
                const float cx = a.prev_pts[2 * cand], cy = a.prev_pts[2 * cand + 1];
                if (j < cnt) {
                    i = cand;
                    p0x = cx;
                    p0y = cy;
                }
            }
        }
    }
    const bool valid = i >= 0;
    if (!any_lane(valid)) return;  // wave-uniform
#ifdef TBDK_LK_TRACE
    int tr_steps = 0, tr_reloads = 0;
    unsigned tr_gsplit = 0;  // levels whose G sums took seg_sum_exact's split path
    auto tr_stamp = [&](int idx) {
        const unsigned r = a.trace_base + (unsigned)wave;
        const unsigned d = (unsigned)(__builtin_amdgcn_s_memrealtime() - tr_t0);
        if (lane == 0 && r < g_lk_trace_cap) reinterpret_cast<unsigned*>(g_lk_trace + 16ull * r + 6)[idx] = d;
    };
#else
    auto tr_stamp = [](int) {};
#endif
#ifdef TBDK_LK_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the point's coordinates have arrived
    tr_stamp(13);
#endif
    const int e4 = 4 * (k * WW + WW), s4 = 4 * (k * WW);  // last lane of the point, lane before its first
    const int rnd9 = __builtin_amdgcn_readfirstlane(1 << (W_BITS1 - 5 - 1));
    const int rnd14 = __builtin_amdgcn_readfirstlane(1 << (W_BITS1 - 1));

    const float FLT_SCALE = 1.f / (1 << 20);
    const float halfx = (WW - 1) * 0.5f, halfy = (WH - 1) * 0.5f;
    const int gy = DENSE && valid ? i / a.dense_w : 0, gx = DENSE && valid ? i - gy * a.dense_w : 0;  // DENSE: the pixel
    if constexpr (DENSE) {
        p0x = (float)gx;
        p0y = (float)gy;
    }
    float outx = 0.f, outy = 0.f;
    if ((a.flags & TBDK_OPTFLOW_USE_INITIAL_FLOW) && valid) {
        outx = a.next_pts[2 * i];
        outy = a.next_pts[2 * i + 1];
    }
    int status = 1, nit = 0;
#if TBDK_LK_PRIO_STEPS > 0
    int wsteps = 0;  // Newton steps this wave has run (wave-uniform)
#endif
#if defined(TBDK_LK_PROBE_RELOADS) && TBDK_LK_PROBE_RELOADS == 2
    int nrl = 0;
#endif
    float errv = 0.f;

    for (int level = a.max_level; level >= 0; --level) {
        const LkLevel L = a.lv[level];
        tr_stamp(4 * level);
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
        uint32_t w0, w1;
        bilinear_weights(prevx - ipx, prevy - ipy, w0, w1);

        uint32_t jp[WH + 1];
        const int hp = L.h + 2 * L.ipad;
        // an unpadded level (pad 0: the TBD loop's level 0, the frame itself) is
        // bounded exactly; padded levels carry 256 bytes of over-read room
        const __amdgpu_buffer_rsrc_t rI = make_rsrc(L.I, L.ipitch * hp + (L.ipad ? 256 : 0));
        const __amdgpu_buffer_rsrc_t rD = make_rsrc(L.D, L.dpitch * (L.h + 2 * L.dpad) + 256);
        const __amdgpu_buffer_rsrc_t rJ = make_rsrc(L.J, L.jpitch * (L.h + 2 * L.jpad) + (L.jpad ? 256 : 0));
        // the J window rows jy0 .. jy0 + WH at columns jx0 + x, jx0 + x + 1 into jp;
        // on an unpadded level a wave with a window across the edge takes the
        // reflect-101 path (wave-uniform)
        auto load_j = [&](bool on, int jx0, int jy0) {
            if (L.jpad == 0 &&
                any_lane(on && (jx0 + x < 0 || jx0 + x + 1 >= L.w || jy0 < 0 || jy0 + WH >= L.h))) {
#pragma unroll
                for (int r = 0; r <= WH; ++r)
                    jp[r] = on ? load_pair_refl(rJ, L.jpitch, L.w, L.h, jy0 + r, jx0 + x) : 0u;
                return;
            }
            const uint32_t joff = on ? (uint32_t)((jy0 + L.jpad) * L.jpitch + jx0 + x + L.jpad) : 0u;
#pragma unroll
            for (int r = 0; r <= WH; ++r) jp[r] = load_pair_u8_ua(rJ, joff, r * L.jpitch);
        };

        nextx -= halfx;
        nexty -= halfy;
        int pinx = (int)floorf(nextx), piny = (int)floorf(nexty);

        // ---- per row: ic = round - I x32 * 2^9, so that the J bilinear sum
        // started from ic and shifted right by 9 is diff = J x32 - I x32 itself
        // (2^9 * I is a multiple of the divisor: floor((X - 2^9 I) / 2^9) =
        // floor(X / 2^9) - I); Ix, Iy packed by row pairs as int16 x 2
        uint32_t ipk[IPACK ? NP : 1];  // I x32 of rows (2q, 2q+1) as int16 x 2
        int ic[IM == 0 ? WH : 1];
        int cgx = 0, cgy = 0;  // ILIN: this lane's sum(I x32 * Ix), sum(I x32 * Iy)
        uint32_t gxk[NP], gyk[NP];
        float A11, A12, A22;
        {
            int acc[3] = {0, 0, 0};
            // one row pair of the setup: I x32 (-> ic), the interpolated Ix / Iy
            // packed by row pairs (-> gxk, gyk) and the G sums, from the window
            // rows' (I(x), I(x+1)), (Ix(x), Ix(x+1)), (Iy(x), Iy(x+1)) pairs
            // dw0/dw1: the weights of the derivative rows r (top) and r+1 (bottom) of
            // the pair's first row, dw2/dw3 those of rows r+1 and r+2 of its second
            // (w0, w1 unless the level frame's zero rule masks a row or a column)
            auto pair_step = [&](int q, uint32_t ip0, uint32_t ip1, uint32_t ip2, uint32_t dx0, uint32_t dx1,
                                 uint32_t dx2, uint32_t dy0, uint32_t dy1, uint32_t dy2, uint32_t dw0, uint32_t dw1,
                                 uint32_t dw2, uint32_t dw3) {
                const int r = 2 * q;
                const bool two = r + 1 < WH;
                uint32_t ipq = 0;
                if constexpr (IPACK || ILIN) {
                    const int i0 = bilin_s<0>(ip0, ip1, w0, w1, rnd9);
                    const int i1 = two ? bilin_s<0>(ip1, ip2, w0, w1, rnd9) : 0;
                    ipq = pack_shr<W_BITS1 - 5>(i0, i1);
                    if constexpr (IPACK) ipk[q] = ipq;
                } else {
                    ic[r] = rnd9 - (bilin_s<W_BITS1 - 5>(ip0, ip1, w0, w1, rnd9) << 9);
                    if (two) ic[r + 1] = rnd9 - (bilin_s<W_BITS1 - 5>(ip1, ip2, w0, w1, rnd9) << 9);
                }
                // interpolated Ix / Iy of rows r, r+1, shifted and packed (pack_shr)
                const int x0 = bilin_s<0>(dx0, dx1, dw0, dw1, rnd14);
                const int x1 = two ? bilin_s<0>(dx1, dx2, dw2, dw3, rnd14) : 0;
                const int y0 = bilin_s<0>(dy0, dy1, dw0, dw1, rnd14);
                const int y1 = two ? bilin_s<0>(dy1, dy2, dw2, dw3, rnd14) : 0;
                gxk[q] = pack_shr<W_BITS1>(x0, x1);
                gyk[q] = pack_shr<W_BITS1>(y0, y1);
                if constexpr (GL) sgw[q][lane] = make_uint2(gxk[q], gyk[q]);
                if constexpr (ILIN) {
                    cgx = sdot2(ipq, gxk[q], cgx);
                    cgy = sdot2(ipq, gyk[q], cgy);
                }
                acc[0] = sdot2(gxk[q], gxk[q], acc[0]);
                acc[1] = sdot2(gxk[q], gyk[q], acc[1]);
                acc[2] = sdot2(gyk[q], gyk[q], acc[2]);
            };
            if constexpr (FLY) {
                // calcSharrDeriv (lkpyramid.cpp:55-144) of the window, from the
                // padded u8 level: one unaligned dword per row holds columns
                // x-1 .. x+2, rows -1 .. WH+1.  The reference's vertical-then-
                // horizontal integer passes are linear, so they are evaluated in the
                // other order, each source row's horizontal terms shared by the
                // three derivative rows that read it: per row j the u16 pairs
                // lo = (x-1, x), hi = (x+1, x+2), mid = (x, x+1) (mid is also the I
                // pair), hd = hi - lo and sm = 3 (lo + hi) + 10 mid; then for
                // derivative row r (source rows r, r+1, r+2)
                //   (Ix(x), Ix(x+1)) = 3 (hd_r + hd_r+2) + 10 hd_r+1,
                //   (Iy(x), Iy(x+1)) = sm_r+2 - sm_r,
                // the same integers as t0 = 3(a+c) + 10b, t1 = c - a then
                // t0(x+1) - t0(x-1), 3 (t1(x-1) + t1(x+1)) + 10 t1(x) (|Ix|, |Iy|
                // <= 4080: exact modulo 2^16).  The level's reflect-101 frame is the
                // reference's row / column reflection.
                const uint32_t ioff = act ? (uint32_t)((ipy - 1 + L.ipad) * L.ipitch + ipx + x - 1 + L.ipad) : 0u;
                uint32_t u[WH + 3];
                if (L.ipad == 0 &&
                    any_lane(act && (ipx + x - 1 < 0 || ipx + x + 2 >= L.w || ipy - 1 < 0 || ipy + WH + 1 >= L.h))) {
#pragma unroll
                    for (int r = 0; r < WH + 3; ++r)
                        u[r] = act ? load4_refl(rI, L.ipitch, L.w, L.h, ipy - 1 + r, ipx + x - 1) : 0u;
                } else {
#pragma unroll
                    for (int r = 0; r < WH + 3; ++r)
                        u[r] = __builtin_amdgcn_raw_buffer_load_b32(rI, ioff, r * L.ipitch, 0);
                }
#ifdef TBDK_LK_TRACE
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the level's source rows have arrived
                if (level == a.max_level) tr_stamp(14);
#endif
                // Outside the level the derivative planes hold BORDER_CONSTANT 0
                // (lkpyramid.cpp:1357).  A zero derivative contributes nothing to the
                // bilinear sums, so the rule is applied to the derivative weights:
                // the column halves (x, x+1) outside [0, w) by cm, derivative rows
                // outside [0, h) by the per-lane row bits vm (three ops a row, for
                // all waves: a wave-uniform masked / unmasked split needs more
                // VGPRs than it saves)
                const uint32_t cm = ((unsigned)(ipx + x) < (unsigned)L.w ? 0x0000FFFFu : 0u) |
                                    ((unsigned)(ipx + x + 1) < (unsigned)L.w ? 0xFFFF0000u : 0u);
                const int rlo = min(max(-ipy, 0), 32), rhi = min(max(L.h - ipy, 0), 32);
                const uint32_t vm = (uint32_t)(((1ull << rhi) - 1ull) & ~((1ull << rlo) - 1ull));
                const uint32_t wd0 = w0 & cm, wd1 = w1 & cm;
                auto rowbit = [&](int r) { return (uint32_t)((int)(vm << (31 - r)) >> 31); };  // row r valid: ~0
                auto src = [&](int j, uint32_t& mid, uint32_t& hd, uint32_t& sm) {
                    const u16x2 lo = as_u16x2(__builtin_amdgcn_perm(0u, u[j], 0x0C010C00u));
                    const u16x2 hi = as_u16x2(__builtin_amdgcn_perm(0u, u[j], 0x0C030C02u));
                    mid = __builtin_amdgcn_perm(0u, u[j], 0x0C020C01u);
                    hd = as_u32(hi - lo);
                    sm = as_u32((lo + hi) * (unsigned short)3 + as_u16x2(mid) * (unsigned short)10);
                };
                // derivative row r from the source rows' terms (a, b, c = rows r, r+1, r+2)
                auto drow = [&](uint32_t hda, uint32_t hdb, uint32_t hdc, uint32_t sma, uint32_t smc, uint32_t& dx,
                                uint32_t& dy) {
                    dx = as_u32((as_u16x2(hda) + as_u16x2(hdc)) * (unsigned short)3 + as_u16x2(hdb) * (unsigned short)10);
                    dy = as_u32(as_u16x2(smc) - as_u16x2(sma));
                };
                // rolling window over the source rows: (m, h, s) of rows j-2, j-1, j
                uint32_t m0, h0, s0, m1, h1, s1, m2, h2, s2;
                src(0, m0, h0, s0);
                src(1, m1, h1, s1);
                src(2, m2, h2, s2);
                uint32_t dxa, dya;
                drow(h0, h1, h2, s0, s2, dxa, dya);  // derivative row 0
                uint32_t ipa = m1;                   // I row 0
                uint32_t ra = rowbit(0);
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    const int r = 2 * q;
                    // rows r+1 (source r+3) and r+2 (source r+4)
                    m0 = m1; h0 = h1; s0 = s1;
                    m1 = m2; h1 = h2; s1 = s2;
                    src(r + 3, m2, h2, s2);
                    uint32_t dxb, dyb, dxc = 0, dyc = 0, ipc = 0;
                    drow(h0, h1, h2, s0, s2, dxb, dyb);
                    const uint32_t ipb = m1;
                    const uint32_t rb = rowbit(r + 1);
                    uint32_t rc = 0;
                    if (r + 1 < WH) {
                        m0 = m1; h0 = h1; s0 = s1;
                        m1 = m2; h1 = h2; s1 = s2;
                        src(r + 4, m2, h2, s2);
                        drow(h0, h1, h2, s0, s2, dxc, dyc);
                        ipc = m1;
                        rc = rowbit(r + 2);
                    }
                    pair_step(q, ipa, ipb, ipc, dxa, dxb, dxc, dya, dyb, dyc, wd0 & ra, wd1 & rb, wd0 & rb, wd1 & rc);
                    ipa = ipc;
                    dxa = dxc;
                    dya = dyc;
                    ra = rc;
                }
            } else if constexpr (DENSE) {
                // the window from case image (gx, gy) mod 2^level: element (r, x) at
                // level position (ipy + r, ipx + x); per row pair two 8-byte loads
                // of (I x32 | Ix << 16, Iy) and the same packing as pair_step
                const int msk = (1 << level) - 1;
                // (inactive lanes: the case-0 image's top-left corner, in bounds)
                const int64_t cbase = act ? (int64_t)(((gy & msk) << level) | (gx & msk)) * L.cstride +
                                                (int64_t)ipy * L.cpitch + ipx + x
                                          : -(int64_t)(WH / 2) * L.cpitch - WW / 2;
                const uint2* cw = L.C + cbase;
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    const int r = 2 * q;
                    const uint2 e0 = cw[(int64_t)r * L.cpitch];
                    const uint2 e1 = r + 1 < WH ? cw[(int64_t)(r + 1) * L.cpitch] : make_uint2(0u, 0u);
                    ipk[q] = __builtin_amdgcn_perm(e1.x, e0.x, 0x05040100u);  // (I x32 of rows r, r+1)
                    gxk[q] = __builtin_amdgcn_perm(e1.x, e0.x, 0x07060302u);  // (Ix of rows r, r+1)
                    gyk[q] = __builtin_amdgcn_perm(e1.y, e0.y, 0x05040100u);  // (Iy of rows r, r+1)
                    acc[0] = sdot2(gxk[q], gxk[q], acc[0]);
                    acc[1] = sdot2(gxk[q], gyk[q], acc[1]);
                    acc[2] = sdot2(gyk[q], gyk[q], acc[2]);
                }
            } else {
                uint32_t ip[WH + 1], dxp[WH + 1], dyp[WH + 1];
                const uint32_t ioff = act ? (uint32_t)((ipy + L.ipad) * L.ipitch + ipx + x + L.ipad) : 0u;
                const uint32_t doff = act ? (uint32_t)((ipy + L.dpad) * L.dpitch + (ipx + x + L.dpad) * 4) : 0u;
#pragma unroll
                for (int r = 0; r <= WH; ++r) {
                    ip[r] = load_pair_u8_ua(rI, ioff, r * L.ipitch);
                    const uint32_t d0 = __builtin_amdgcn_raw_buffer_load_b32(rD, doff, r * L.dpitch, 0);
                    const uint32_t d1 = __builtin_amdgcn_raw_buffer_load_b32(rD, doff + 4, r * L.dpitch, 0);
                    dxp[r] = __builtin_amdgcn_perm(d1, d0, 0x05040100u);  // (Ix(x), Ix(x+1))
                    dyp[r] = __builtin_amdgcn_perm(d1, d0, 0x07060302u);  // (Iy(x), Iy(x+1))
                }
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    const int r = 2 * q;
                    const int r2 = r + 2 <= WH ? r + 2 : WH;
                    pair_step(q, ip[r], ip[r + 1], ip[r2], dxp[r], dxp[r + 1], dxp[r2], dyp[r], dyp[r + 1], dyp[r2],
                              w0, w1, w0, w1);
                }
            }
            if constexpr (IPACK) {
                // materialise the I pairs here: left to the compiler, their bilinear
                // sums sink below the G reduction and the J loads, where the I
                // rows they read are then still live (+22 VGPRs at the peak)
#pragma unroll
                for (int q = 0; q < NP; ++q) asm volatile("" : "+v"(ipk[q]));
            }
#ifdef TBDK_LK_TRACE
            __builtin_amdgcn_sched_barrier(0);
            if (level == a.max_level) tr_stamp(15);  // the first level's window terms done (before the G sums)
            __builtin_amdgcn_sched_barrier(0);
#endif
            if (k >= P) acc[0] = acc[1] = acc[2] = 0;
            float s[3];
#ifdef TBDK_LK_TRACE
            bool tr_split = false;
            seg_sum_exact<3>(acc, e4, s4, s, &tr_split);
            tr_gsplit |= tr_split ? 1u << level : 0u;
#else
            seg_sum_exact<3>(acc, e4, s4, s);
#endif
            tr_stamp(4 * level + 1);
            // J columns at the first Newton position, loaded after the G sums (with
            // the loads in flight during the sums the kernel needs 148 VGPRs, 3
            // waves per SIMD; this way 116, 4 waves)
            {
                const bool jin = act && !(pinx < -WW || pinx >= L.w || piny < -WH || piny >= L.h);
                load_j(jin, pinx, piny);
#ifdef TBDK_LK_TRACE
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
                tr_stamp(4 * level + 2);
            }
            // A = float(exact sum) * 2^-20   (lkpyramid.cpp:438-440)
            A11 = s[0] * FLT_SCALE;
            A12 = s[1] * FLT_SCALE;
            A22 = s[2] * FLT_SCALE;
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
        // The remaining Newton steps of point ks, the wave's only active one, from
        // step j on (the stepping of the loop below, the same integers and float
        // operations): its window's rows are dealt to the P lane groups, group g
        // holding row pairs [g*NPG, (g+1)*NPG) of every column (the I terms and
        // the interpolated Ix / Iy pairs moved over by ds_bpermute from the
        // point's own lanes, the J rows loaded per group), so a step costs each
        // lane NPG row pairs instead of NP; the per-point values are broadcast
        // from the point's first lane and the result goes back to its lanes.
        auto solo_steps = [&](int ks, int j) {
            constexpr int NPG = (NP + P - 1) / P;  // row pairs per lane group
            constexpr int RG = 2 * NPG;            // window rows per lane group
            const int sl = 1 + ks * WW;            // the point's first lane
            const int src = k < P ? 4 * (sl + x) : 0;  // this lane's column of the point (bpermute address)
            const int g = k < P ? k : 0;
            uint32_t gx2[NPG], gy2[NPG], ip2[IPACK ? NPG : 1];
            int ic2[IM == 0 ? RG : 1];
#pragma unroll
            for (int t = 0; t < NPG; ++t) gx2[t] = gy2[t] = 0u;
            if constexpr (IPACK) {
#pragma unroll
                for (int t = 0; t < NPG; ++t) ip2[t] = 0u;
            }
            if constexpr (IM == 0) {
#pragma unroll
                for (int t = 0; t < RG; ++t) ic2[t] = 0;
            }
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const uint32_t tx = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)gxk[q]);
                const uint32_t ty = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)gyk[q]);
                gx2[q % NPG] = g == q / NPG ? tx : gx2[q % NPG];
                gy2[q % NPG] = g == q / NPG ? ty : gy2[q % NPG];
                if constexpr (IPACK) {
                    const uint32_t ti = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)ipk[q]);
                    ip2[q % NPG] = g == q / NPG ? ti : ip2[q % NPG];
                }
            }
            if constexpr (IM == 0) {
#pragma unroll
                for (int r = 0; r < WH; ++r) {
                    const int ti = __builtin_amdgcn_ds_bpermute(src, ic[r]);
                    ic2[r % RG] = g == r / RG ? ti : ic2[r % RG];
                }
            }
            if (k >= P) {  // lane 0 (and lanes past the last point) add nothing
#pragma unroll
                for (int t = 0; t < NPG; ++t) gx2[t] = gy2[t] = 0u;
            }
            auto bc = [&](float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), sl)); };
            float snx = bc(nextx), sny = bc(nexty), sox = bc(outx), soy = bc(outy), spdx = bc(pdx), spdy = bc(pdy);
            const float sA11 = bc(A11), sA12 = bc(A12), sA22 = bc(A22), sD = bc(D);
            // rows rbase .. rbase + RG of the window at J origin (jx0, jy0) of a padded
            // level (an unpadded one takes no one-point steps); rows past the window
            // (the last group) feed only pairs whose Ix / Iy halves are zero, and a
            // row past the level's buffer reads 0
            const int rbase = g * RG;
            uint32_t jp2[RG + 1];
            auto load_j2 = [&](int jx0, int jy0) {
                const uint32_t joff = (uint32_t)((jy0 + rbase + L.jpad) * L.jpitch + jx0 + x + L.jpad);
#pragma unroll
                for (int r = 0; r <= RG; ++r) jp2[r] = load_pair_u8_ua(rJ, joff, r * L.jpitch);
            };
            int qx = INT_MIN, qy = 0, snit = 0;
            bool sout = false;
            for (; j < a.max_count; ++j) {
                const int inx = (int)floorf(snx), iny = (int)floorf(sny);
                if (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h) {
                    sout = true;
                    break;
                }
                ++snit;
#ifdef TBDK_LK_TRACE
                ++tr_steps;
#endif
                if (inx != qx || iny != qy) {
#ifdef TBDK_LK_TRACE
                    ++tr_reloads;
#endif
                    load_j2(inx, iny);
                    qx = inx;
                    qy = iny;
                }
                uint32_t v0, v1;
                bilinear_weights(snx - inx, sny - iny, v0, v1);
                int b[2] = {0, 0};
#pragma unroll
                for (int t = 0; t < NPG; ++t) {
                    uint32_t d;
                    if constexpr (IPACK) {
                        const uint32_t jv = pack_diff(bilin_s<0>(jp2[2 * t], jp2[2 * t + 1], v0, v1, rnd9),
                                                      bilin_s<0>(jp2[2 * t + 1], jp2[2 * t + 2], v0, v1, rnd9));
                        d = as_u32(as_s16x2(jv) - as_s16x2(ip2[t]));
                    } else {
                        d = pack_diff(bilin_c(jp2[2 * t], jp2[2 * t + 1], v0, v1, ic2[2 * t]),
                                      bilin_c(jp2[2 * t + 1], jp2[2 * t + 2], v0, v1, ic2[2 * t + 1]));
                    }
                    b[0] = sdot2(d, gx2[t], b[0]);
                    b[1] = sdot2(d, gy2[t], b[1]);
                }
                float fb[2];
                seg_sum_exact<2, 25>(b, 4 * (P * WW), 0, fb);  // lanes 1 .. P*WW (lane 0 adds 0)
                const float fb1 = fb[0] * FLT_SCALE;
                const float fb2 = fb[1] * FLT_SCALE;
                const float ddx = (sA12 * fb2 - sA22 * fb1) * sD;
                const float ddy = (sA12 * fb1 - sA11 * fb2) * sD;
                snx += ddx;
                sny += ddy;
                sox = snx + halfx;
                soy = sny + halfy;
                if ((double)ddx * ddx + (double)ddy * ddy <= a.eps2) break;
                if (j > 0 && (double)fabsf(ddx + spdx) < 0.01 && (double)fabsf(ddy + spdy) < 0.01) {
                    sox -= ddx * 0.5f;
                    soy -= ddy * 0.5f;
                    break;
                }
                spdx = ddx;
                spdy = ddy;
            }
            if (k == ks) {
                outx = sox;
                outy = soy;
#ifdef TBDK_LK_PROBE_ITERS_LV
                nit += snit << (8 * level);
#else
                nit += snit;
#endif
                if (sout && level == 0) status = 0;
            }
            act = false;
        };
        for (int j = 0; j < a.max_count; ++j) {
            if (!any_lane(act)) break;
#ifdef TBDK_LK_TRACE
            ++tr_steps;
#endif
#if TBDK_LK_PRIO_STEPS > 0
            if (++wsteps == TBDK_LK_PRIO_STEPS) __builtin_amdgcn_s_setprio(3);
#endif
            if constexpr (kSoloOk) {
                // one point left stepping (LkArgs::solo_min): its remaining steps
                // on all the wave's lanes, the window rows split over the P lane
                // groups (solo_steps); then the level's Newton phase is over
                if (a.solo_min > 0 && j >= a.solo_min && L.jpad > 0) {
                    const uint64_t heads = __builtin_amdgcn_ballot_w64(act && x == 0 && k < P);
                    if (__builtin_popcountll(heads) == 1) {
                        solo_steps((__builtin_ctzll(heads) - 1) / WW, j);
                        break;
                    }
                }
            }
            const int inx = (int)floorf(nextx), iny = (int)floorf(nexty);
            if (act && (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h)) {
                if (level == 0) status = 0;
                act = false;
            }
#ifdef TBDK_LK_PROBE_ITERS_LV  // probe builds: the Newton steps per level, 8 bits each (level L at bit 8L)
            nit += act ? 1 << (8 * level) : 0;
#else
            nit += act ? 1 : 0;
#endif
            const bool moved = act && (inx != pinx || iny != piny);
#ifdef TBDK_LK_PROBE_RELOADS  // tuning builds: 1 always reloads, 2 counts reloads into iters, 3 never reloads
#if TBDK_LK_PROBE_RELOADS == 2
            nrl += any_lane(moved) ? 1 : 0;
#endif
            if (TBDK_LK_PROBE_RELOADS == 1 || (TBDK_LK_PROBE_RELOADS != 3 && any_lane(moved))) {
#else
            if (any_lane(moved)) {  // uniform: reload the J columns (unchanged for points that did not move)
#endif
#ifdef TBDK_LK_TRACE
                ++tr_reloads;
#endif
                load_j(act, inx, iny);
                pinx = inx;
                piny = iny;
            }
            bilinear_weights(nextx - inx, nexty - iny, w0, w1);
            int b[2] = {0, 0};
            if constexpr (GL) asm volatile("" ::: "memory");  // the (Ix, Iy) pairs are re-read from LDS every step
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const int r = 2 * q;
                // (diff_r, diff_r+1) as int16 x 2, |diff| <= 8160
                uint32_t d;
                if constexpr (ILIN) {
                    // (J x32 of rows r, r+1) as int16 x 2; I enters through cgx / cgy
                    d = r + 1 < WH ? pack_diff(bilin_s<0>(jp[r], jp[r + 1], w0, w1, rnd9),
                                               bilin_s<0>(jp[r + 1], jp[r + 2], w0, w1, rnd9))
                                   : pack_diff(bilin_s<0>(jp[r], jp[r + 1], w0, w1, rnd9), 0);
                } else if constexpr (IPACK) {
                    // (J x32 of rows r, r+1) as int16 x 2, minus the I pair: one packed subtract
                    const uint32_t jv = r + 1 < WH ? pack_diff(bilin_s<0>(jp[r], jp[r + 1], w0, w1, rnd9),
                                                               bilin_s<0>(jp[r + 1], jp[r + 2], w0, w1, rnd9))
                                                   : pack_diff(bilin_s<0>(jp[r], jp[r + 1], w0, w1, rnd9), 0);
                    d = as_u32(as_s16x2(jv) - as_s16x2(ipk[q]));
                } else {
                    d = r + 1 < WH ? pack_diff(bilin_c(jp[r], jp[r + 1], w0, w1, ic[r]),
                                               bilin_c(jp[r + 1], jp[r + 2], w0, w1, ic[r + 1]))
                                   : pack_diff(bilin_c(jp[r], jp[r + 1], w0, w1, ic[r]), 0);
                }
                uint32_t gx = gxk[q], gy = gyk[q];
                if constexpr (GL) {
                    const uint2 g = sgw[q][lane];
                    gx = g.x;
                    gy = g.y;
                }
                b[0] = sdot2(d, gx, b[0]);
                b[1] = sdot2(d, gy, b[1]);
#ifdef TBDK_LK_NEWTON_SB
                if (q % TBDK_LK_NEWTON_SB == TBDK_LK_NEWTON_SB - 1) __builtin_amdgcn_sched_barrier(0);
#endif
            }
            if constexpr (ILIN) {
                // sum((Jd - I) g) = sum(Jd g) - sum(I g): the same lane partial
                // (modulo 2^32 on the way, exact at the end)
                b[0] -= cgx;
                b[1] -= cgy;
            }
            if (k >= P) b[0] = b[1] = 0;
            float fb[2];
            seg_sum_exact<2>(b, e4, s4, fb);
            const float fb1 = fb[0] * FLT_SCALE;
            const float fb2 = fb[1] * FLT_SCALE;
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

        tr_stamp(4 * level + 3);
        if (level == 0 && a.err && (a.flags & TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS) == 0) {
            bool want = valid && status;
            const float npx = outx - halfx, npy = outy - halfy;
            const int inx = (int)floorf(npx), iny = (int)floorf(npy);
            if (want && (inx < -WW || inx >= L.w || iny < -WH || iny >= L.h)) {
                status = 0;
                want = false;
            }
            if (any_lane(want)) {
                // ILIN: the I rows again (the level-0 window at prev, its weights),
                // packed by row pairs before the J rows are loaded (with both row
                // sets live at once this block set the kernel's register peak)
                uint32_t ipr[ILIN ? NP : 1];
                if constexpr (ILIN) {
                    uint32_t iw0, iw1;
                    bilinear_weights(prevx - ipx, prevy - ipy, iw0, iw1);
                    // an unpadded level: reflect-101 when a window crosses its edge
                    const bool irefl = L.ipad == 0 && any_lane(want && (ipx + x < 0 || ipx + x + 1 >= L.w ||
                                                                        ipy < 0 || ipy + WH >= L.h));
                    const uint32_t ioff = want ? (uint32_t)((ipy + L.ipad) * L.ipitch + ipx + x + L.ipad) : 0u;
                    auto irow = [&](int r) -> uint32_t {
                        if (irefl) return want ? load_pair_refl(rI, L.ipitch, L.w, L.h, ipy + r, ipx + x) : 0u;
                        return load_pair_u8_ua(rI, ioff, r * L.ipitch);
                    };
                    // row by row (two rows live), packed by row pairs
                    uint32_t ra = irow(0);
#pragma unroll
                    for (int q = 0; q < NP; ++q) {
                        const int r = 2 * q;
                        const uint32_t rb = irow(r + 1);
                        const uint32_t rc = r + 2 <= WH ? irow(r + 2) : 0u;
                        ipr[q] = pack_shr<W_BITS1 - 5>(bilin_s<0>(ra, rb, iw0, iw1, rnd9),
                                                        r + 1 < WH ? bilin_s<0>(rb, rc, iw0, iw1, rnd9) : 0);
                        asm volatile("" : "+v"(ipr[q]));
                        ra = rc;
                    }
                }
                bilinear_weights(npx - inx, npy - iny, w0, w1);
                load_j(want, inx, iny);
                int e = 0;
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    const int r = 2 * q;
                    int d0;
                    if constexpr (ILIN)
                        d0 = (bilin_s<0>(jp[r], jp[r + 1], w0, w1, rnd9) >> 9) - (int)(int16_t)(ipr[q] & 0xFFFFu);
                    else if constexpr (IPACK)
                        d0 = (bilin_s<0>(jp[r], jp[r + 1], w0, w1, rnd9) >> 9) - (int)(int16_t)(ipk[q] & 0xFFFFu);
                    else
                        d0 = bilin_c(jp[r], jp[r + 1], w0, w1, ic[r]) >> 9;
                    e += d0 < 0 ? -d0 : d0;
                    if (r + 1 < WH) {
                        int d1;
                        if constexpr (ILIN)
                            d1 = (bilin_s<0>(jp[r + 1], jp[r + 2], w0, w1, rnd9) >> 9) - (int)(int16_t)(ipr[q] >> 16);
                        else if constexpr (IPACK)
                            d1 = (bilin_s<0>(jp[r + 1], jp[r + 2], w0, w1, rnd9) >> 9) - (int)(int16_t)(ipk[q] >> 16);
                        else
                            d1 = bilin_c(jp[r + 1], jp[r + 2], w0, w1, ic[r + 1]) >> 9;
                        e += d1 < 0 ? -d1 : d1;
                    }
                }
                if (k >= P) e = 0;
                const float errval = (float)seg_sum_small(e, e4, s4);
                if (want) errv = errval * 1.f / (float)(32 * WW * WH);
                tr_stamp(12);
            }
        }
    }

#ifdef TBDK_LK_TRACE
    {
        int mx = 0;
#pragma unroll
        for (int q = 0; q < P; ++q) mx = max(mx, __builtin_amdgcn_readlane(valid ? nit : 0, 1 + q * WW));
        const unsigned long long tr_t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20); // XCC_ID
        if (lane == 0) {
            const unsigned r = a.trace_base + (unsigned)wave;
            if (r < g_lk_trace_cap) {
                unsigned long long* o = g_lk_trace + 16ull * r;
                o[0] = tr_t0;
                o[1] = tr_t1;
                o[2] = hw | ((unsigned long long)xcc << 32);
                o[3] = ((unsigned long long)(unsigned)a.n << 32) | (unsigned)wave;
                o[4] = a.seg_ninl > 0 ? (1ull << 48) | ((unsigned long long)a.seg_ninl << 16) | a.seg_inl[0]
                                      : (unsigned long long)(uintptr_t)(a.seg_list ? (const void*)a.seg_list
                                                                                   : (const void*)a.prev_pts);
                o[5] = (unsigned)tr_steps | ((unsigned long long)(unsigned)tr_reloads << 16) |
                       ((unsigned long long)(unsigned)mx << 32) | ((unsigned long long)tr_gsplit << 48);
            }
        }
    }
#endif
    if (DENSE && valid && x == 0) {
        *reinterpret_cast<float2*>(reinterpret_cast<uint8_t*>(a.flow) + (size_t)gy * a.flow_pitch + 8 * (size_t)gx) =
            make_float2(outx - (float)gx, outy - (float)gy);
        if (a.dstatus) a.dstatus[(size_t)gy * a.dstatus_pitch + gx] = (uint8_t)status;
        return;
    }
    if (valid && x == 0) {
        a.next_pts[2 * i] = outx;
        a.next_pts[2 * i + 1] = outy;
        a.status[i] = (uint8_t)status;
        if (a.err) a.err[i] = errv;
#if defined(TBDK_LK_PROBE_RELOADS) && TBDK_LK_PROBE_RELOADS == 2
        nit += 1000 * nrl;
#endif
        if (a.iters) a.iters[i] = nit;
    }
}

#define TBDK_MULTI_WINDOWS(X) X(7) X(9) X(11) X(13) X(15) X(17) X(19) X(21) X(23) X(25) X(27) X(29) X(31)

bool lk_multi_supported(int win_w, int win_h)
{
    if (win_w != win_h) return false;
    switch (win_w) {
#define TBDK_CASE(W) case W:
        TBDK_MULTI_WINDOWS(TBDK_CASE)
#undef TBDK_CASE
        return true;
    default:
        return false;
    }
}

hipError_t launch_lk_multi(const LkArgs& a, bool fly, hipStream_t s)
{
    if (!lk_multi_supported(a.win_w, a.win_h)) return hipErrorNotSupported;
    const int per_wg = kMultiWaves * (64 / a.win_w);  // waves of P points
    const dim3 grid((a.n + per_wg - 1) / per_wg), block(64 * kMultiWaves);
#ifdef TBDK_LK_TRACE
    LkArgs at = a;
    at.trace_base = g_lk_trace_next;
    g_lk_trace_next += grid.x * kMultiWaves;
    const LkArgs& la = at;
#else
    const LkArgs& la = a;
#endif
    switch (a.win_w) {
#define TBDK_CASE(W)                                                                    \
    case W:                                                                             \
        if (fly) hipLaunchKernelGGL((lk_multi_kernel<W, W, true>), grid, block, 0, s, la);  \
        else hipLaunchKernelGGL((lk_multi_kernel<W, W, false>), grid, block, 0, s, la); \
        break;
        TBDK_MULTI_WINDOWS(TBDK_CASE)
#undef TBDK_CASE
    default:
        return hipErrorNotSupported;
    }
    return hipGetLastError();
}

hipError_t launch_lk_multi_dense(const LkArgs& a, hipStream_t s)
{
    if (!lk_multi_supported(a.win_w, a.win_h)) return hipErrorNotSupported;
    const int per_wg = kMultiWaves * (64 / a.win_w);  // waves of P points
    const dim3 grid((a.n + per_wg - 1) / per_wg), block(64 * kMultiWaves);
    switch (a.win_w) {
#define TBDK_CASE(W)                                                                          \
    case W:                                                                                   \
        hipLaunchKernelGGL((lk_multi_kernel<W, W, false, true>), grid, block, 0, s, a);       \
        break;
        TBDK_MULTI_WINDOWS(TBDK_CASE)
#undef TBDK_CASE
    default:
        return hipErrorNotSupported;
    }
    return hipGetLastError();
}

}  // namespace tbdk

#ifdef TBDK_LK_TRACE
extern "C" int tbdk_probe_lk_trace(void* buf, unsigned cap)
{
    unsigned long long* p = static_cast<unsigned long long*>(buf);
    cap /= 16;  // records of sixteen u64
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(tbdk::g_lk_trace), &p, sizeof(p)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(tbdk::g_lk_trace_cap), &cap, sizeof(cap)) != hipSuccess)
        return -2;
    tbdk::g_lk_trace_next = 0;
    return 0;
}
// records handed out since tbdk_probe_lk_trace (waves that exit early, with no
// valid point, leave theirs zero)
extern "C" int tbdk_probe_lk_trace_count(unsigned* n)
{
    *n = tbdk::g_lk_trace_next;
    return 0;
}
#endif
