// klt_gftt.hip — Shi-Tomasi corners (goodFeaturesToTrack, min-eigenvalue
// variant) over many isolated ROIs of a frame, for gfx950.
//
// Per-ROI semantics are those of cv::goodFeaturesToTrack on the ROI as an
// isolated image (imgproc/src/featureselect.cpp:361-516 with
// cornerMinEigenVal, corner.cpp:52-101,237-326), in the float/double
// evaluation order documented in oracle/gftt_oracle.c; built with
// -ffp-contract=off so every expression rounds exactly as written.
//
// Three launches, all ROIs of a frame batched in each:
//   1. gftt_rowsum: one thread per ROI pixel: Sobel 3x3 (reflect-101 inside
//                   the ROI) at x-1, x, x+1 -> cov = (Dx^2, DxDy, Dy^2) ->
//                   the boxFilter's horizontal sums in double (RowSum ksize 3,
//                   box_filter.simd.hpp:84-89), three double planes
//   2. gftt_eig   : one thread per ROI column: the reference's running column
//                   sum (ColumnSum, box_filter.simd.hpp:176-273) walked top to
//                   bottom — loads of 8 rows are issued ahead of the dependent
//                   add chain — then the min eigenvalue and a per-ROI max
//   3. gftt_select: one 256-thread workgroup per ROI: threshold-to-zero at
//                   max*q, 3x3 non-max test, candidates compacted into LDS,
//                   bitonic sort by (value desc, address desc) — the
//                   reference's deterministic tie-break (featureselect.cpp:56-64)
//                   — then the greedy min-distance walk (:421-503) by one wave,
//                   64 candidates per step: each lane tests its candidate
//                   against the accepted list, in-batch conflicts become a
//                   64-bit mask, and a scalar pass over the lanes in order
//                   accepts exactly what the sequential walk would.
#include <cfloat>

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

struct Cov {
    float c0, c1, c2;
};

// Sobel (deriv.cpp:414-465 -> sepFilter2D) of ROI column x, row y, then cov
__device__ __forceinline__ Cov sobel_cov(const uint8_t* img, int pitch, const GfttRoi& R, int x, int y)
{
    const double scale = 1.0 / ((double)(1 << 2) * 3 * 255.0);
    const float k = (float)(1.0 * scale), k2 = (float)(2.0 * scale);
    const int xl = refl(x - 1, R.w), xr = refl(x + 1, R.w);
    float rx[3], ry[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const uint8_t* s = img + (size_t)(R.y + refl(y + j - 1, R.h)) * pitch + R.x;
        const float s0 = s[xl], s1 = s[x], s2 = s[xr];
        float t = -1.f * s0;
        t = t + 0.f * s1;
        t = t + 1.f * s2;
        rx[j] = t;
        float u = k * s0;
        u = u + k2 * s1;
        u = u + k * s2;
        ry[j] = u;
    }
    const float dx = (rx[0] + rx[2]) * k + (rx[1] * k2 + 0.f);
    const float dy = (ry[2] - ry[0]) + 0.f;
    return Cov{dx * dx, dx * dy, dy * dy};
}

}  // namespace

__global__ __launch_bounds__(256) void gftt_rowsum_kernel(GfttArgs a)
{
    const int r = blockIdx.y;
    const GfttRoi R = a.rois[r];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= R.w * R.h) return;
    const int y = p / R.w, x = p - y * R.w;
    const Cov l = sobel_cov(a.img, a.pitch, R, refl(x - 1, R.w), y);
    const Cov c = sobel_cov(a.img, a.pitch, R, x, y);
    const Cov q = sobel_cov(a.img, a.pitch, R, refl(x + 1, R.w), y);
    const size_t o = (size_t)R.off + p;
    a.rs0[o] = (double)l.c0 + (double)c.c0 + (double)q.c0;
    a.rs1[o] = (double)l.c1 + (double)c.c1 + (double)q.c1;
    a.rs2[o] = (double)l.c2 + (double)c.c2 + (double)q.c2;
}

__global__ __launch_bounds__(256) void gftt_eig_kernel(GfttArgs a)
{
    constexpr int CH = 8;  // rows loaded ahead of the add chain
    const int r = blockIdx.y;
    const GfttRoi R = a.rois[r];
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= R.w) return;
    const double* p0 = a.rs0 + R.off + x;
    const double* p1 = a.rs1 + R.off + x;
    const double* p2 = a.rs2 + R.off + x;
    float* E = a.eig + R.off + x;
    const size_t W = (size_t)R.w;
    // ColumnSum: SUM = 0 + row(-1), SUM += row(0); per output y:
    // s = SUM + row(y+1); out = (float)s; SUM = s - row(y-1)
    const int rm1 = refl(-1, R.h);
    double m1_0 = p0[rm1 * W], m1_1 = p1[rm1 * W], m1_2 = p2[rm1 * W];  // row y-1
    double m0_0 = p0[0], m0_1 = p1[0], m0_2 = p2[0];                    // row y
    double S0 = 0.0 + m1_0, S1 = 0.0 + m1_1, S2 = 0.0 + m1_2;
    S0 = S0 + m0_0;
    S1 = S1 + m0_1;
    S2 = S2 + m0_2;
    int best = INT_MIN;
    for (int y0 = 0; y0 < R.h; y0 += CH) {
        double q0[CH], q1[CH], q2[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {  // independent loads of rows y0+1 .. y0+CH
            const int yy = y0 + k + 1;
            const size_t row = (size_t)refl(yy < R.h + 1 ? yy : R.h, R.h) * W;
            q0[k] = p0[row];
            q1[k] = p1[row];
            q2[k] = p2[row];
        }
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int y = y0 + k;
            if (y < R.h) {
                const double t0 = S0 + q0[k], t1 = S1 + q1[k], t2 = S2 + q2[k];
                S0 = t0 - m1_0;
                S1 = t1 - m1_1;
                S2 = t2 - m1_2;
                m1_0 = m0_0;
                m1_1 = m0_1;
                m1_2 = m0_2;
                m0_0 = q0[k];
                m0_1 = q1[k];
                m0_2 = q2[k];
                const float aa = (float)t0 * 0.5f, bb = (float)t1, cc = (float)t2 * 0.5f;
                const float t = aa - cc;
                const float e = (aa + cc) - sqrtf(bb * bb + t * t);
                E[(size_t)y * W] = e;
                const int kk = fkey(e);
                best = kk > best ? kk : best;
            }
        }
    }
    atomicMax(&a.roi_max[r], best);
}

struct Cand {
    float v;
    int key;  // (y << 16) | x : same order as the reference's address tie-break
};

// a before b in the reference order: value desc, then address desc
__device__ __forceinline__ bool cand_before(const Cand& a, const Cand& b)
{
    return a.v > b.v || (a.v == b.v && a.key > b.key);
}

// threshold-to-zero at max*q + 3x3 dilate-equality on interior pixels, one
// thread per ROI pixel; candidates appended to the ROI's global list (the
// append order is irrelevant: the list is sorted by (value, address) next)
__global__ __launch_bounds__(256) void gftt_nms_kernel(GfttArgs a)
{
    __shared__ int lcount, lbase;
    const int r = blockIdx.y;
    const GfttRoi R = a.rois[r];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int iw = R.w - 2, ih = R.h - 2;
    if (iw <= 0 || ih <= 0 || (int)(blockIdx.x * blockDim.x) >= iw * ih) return;  // block-uniform
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    bool keep = false;
    float v = 0.f;
    int key = 0;
    if (p < iw * ih) {
        const int y = p / iw + 1, x = p - (y - 1) * iw + 1;
        const float thr = (float)((double)fkey_inv(a.roi_max[r]) * a.quality);
        const float* E = a.eig + R.off + (size_t)y * R.w + x;
        const float v0 = E[0];
        v = v0 > thr ? v0 : 0.f;
        if (v != 0.f) {
            float m = v;
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx) {
                    const float q0 = E[dy * R.w + dx];
                    const float q = q0 > thr ? q0 : 0.f;
                    m = q > m ? q : m;
                }
            keep = v == m;
            key = (y << 16) | x;
        }
    }
    // block-aggregated append: one global atomic per block, not per candidate
    int li = 0;
    if (keep) li = atomicAdd(&lcount, 1);
    __syncthreads();
    if (threadIdx.x == 0) lbase = lcount ? atomicAdd(&a.cand_count[r], lcount) : 0;
    __syncthreads();
    const int slot = lbase + li;
    if (keep && slot < a.cap) reinterpret_cast<Cand*>(a.cand)[(size_t)r * a.cap + slot] = Cand{v, key};
}

constexpr int kSelThreads = 512;

__global__ __launch_bounds__(kSelThreads) void gftt_select_kernel(GfttArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Cand* cand = reinterpret_cast<Cand*>(smem);  // all LDS in the one dynamic region
    float2* acc = reinterpret_cast<float2*>(smem + sizeof(Cand) * a.cap);
    float2* bxy = acc + a.max_corners;  // this step's 64 candidate positions
    uint32_t* occ = reinterpret_cast<uint32_t*>(bxy + 64);
    const int r = blockIdx.x;
    const GfttRoi R = a.rois[r];
    const int tid = threadIdx.x;
    const int total = a.cand_count[r];
    if (total > a.cap) {  // candidate buffer overflow: report, never silently truncate
        if (tid == 0) a.counts[r] = -1;
        return;
    }
    // occupancy bitmap of accepted corners (1 bit per ROI pixel), if it fits
    const int ow = (R.w + 31) / 32 + 1;  // words per row (+1: two-word window reads)
    const bool use_occ = (size_t)ow * R.h * 4 <= (size_t)a.occ_bytes;
    if (use_occ)
        for (int i = tid; i < ow * R.h; i += kSelThreads) occ[i] = 0u;
    int np2 = 1;
    while (np2 < total) np2 <<= 1;
    const Cand* src = reinterpret_cast<const Cand*>(a.cand) + (size_t)r * a.cap;
    for (int i = tid; i < np2; i += kSelThreads) cand[i] = i < total ? src[i] : Cand{-FLT_MAX, -1};
    __syncthreads();
    // bitonic sort, "before" order first; every thread owns np2/2/threads
    // compare-exchange pairs per stage (branch-free indexing, loads batched)
    const int npairs = np2 >> 1;
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int pb = 0; pb < npairs; pb += kSelThreads * 4) {
                int ii[4];
                Cand ci[4], cj[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int pidx = pb + u * kSelThreads + tid;
                    ii[u] = pidx < npairs ? ((pidx & ~(j - 1)) << 1) | (pidx & (j - 1)) : -1;
                    if (ii[u] >= 0) {
                        ci[u] = cand[ii[u]];
                        cj[u] = cand[ii[u] + j];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (ii[u] < 0) continue;
                    const bool up = (ii[u] & k) == 0;
                    const bool swap = up ? cand_before(cj[u], ci[u]) : cand_before(ci[u], cj[u]);
                    if (swap) {
                        cand[ii[u]] = cj[u];
                        cand[ii[u] + j] = ci[u];
                    }
                }
            }
            __syncthreads();
        }
    }
    if (tid >= 64) return;
    // ---- greedy walk in sorted order (featureselect.cpp:421-503), 64 candidates per step
    const int lane = tid;
    const bool use_dist = a.min_distance >= 1.0;
    const double md2 = a.min_distance * a.min_distance;
    int rad = (int)ceil(a.min_distance) - 1;  // |d| <= rad can be closer than min_distance
    if ((double)(rad + 1) * (rad + 1) < md2) rad++;
    const bool occ_ok = use_occ && rad <= 31;
    const int maxc = a.max_corners;
    float2* out = a.corners + (size_t)r * maxc;
    int n = 0;
    bool done = false;
    for (int i0 = 0; i0 < total && !done; i0 += 64) {
        const int i = i0 + lane;
        const bool valid = i < total;
        const int key = valid ? cand[i].key : 0;
        const int ix = key & 0xFFFF, iy = key >> 16;
        const float fx = (float)ix, fy = (float)iy;
        bool good = valid;
        unsigned long long cm = 0ull;
        if (use_dist) {
            bxy[lane] = make_float2(fx, fy);
            if (occ_ok) {  // accepted corners within the window, exact distance test
                for (int dy = -rad; dy <= rad && good; ++dy) {
                    const int yy = iy + dy;
                    if (yy < 0 || yy >= R.h) continue;
                    const int x0 = ix - rad < 0 ? 0 : ix - rad;
                    const int x1 = ix + rad >= R.w ? R.w - 1 : ix + rad;
                    for (int wx = x0 >> 5; wx <= (x1 >> 5) && good; ++wx) {
                        uint32_t bits = occ[yy * ow + wx];
                        while (bits && good) {
                            const int b = __builtin_ctz(bits);
                            bits &= bits - 1u;
                            const int xx = (wx << 5) + b;
                            if (xx < x0 || xx > x1) continue;
                            const float ddx = fx - (float)xx, ddy = fy - (float)yy;
                            if ((double)(ddx * ddx + ddy * ddy) < md2) good = false;
                        }
                    }
                }
            } else {
                for (int q = 0; q < n; ++q) {  // vs corners accepted in earlier steps
                    const float2 pq = acc[q];
                    const float dx = fx - pq.x, dy = fy - pq.y;
                    good = good && !((double)(dx * dx + dy * dy) < md2);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
#pragma unroll 8
            for (int j = 0; j < 64; ++j) {  // vs earlier candidates of this step (LDS broadcast reads)
                const float2 pj = bxy[j];
                const float dx = fx - pj.x, dy = fy - pj.y;
                if (j < lane && (double)(dx * dx + dy * dy) < md2) cm |= 1ull << j;
            }
        }
        const unsigned long long goodm = __ballot(good);
        unsigned long long accm = 0ull;
        int cnt = n;
        for (int k = 0; k < 64; ++k) {  // uniform scalar pass: the sequential acceptance
            if (!((goodm >> k) & 1ull)) continue;
            const unsigned long long ck =
                ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(cm >> 32), k) << 32) |
                (unsigned)__builtin_amdgcn_readlane((int)(unsigned)cm, k);
            if (ck & accm) continue;
            accm |= 1ull << k;
            if (++cnt == maxc) {
                done = true;
                break;
            }
        }
        if ((accm >> lane) & 1ull) {
            const int pos = n + __popcll(accm & ((1ull << lane) - 1ull));
            acc[pos] = make_float2(fx, fy);
            out[pos] = make_float2(fx + (float)R.x, fy + (float)R.y);
            if (occ_ok) atomicOr(&occ[iy * ow + (ix >> 5)], 1u << (ix & 31));
        }
        n = cnt;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): acc[] / occ[] visible to the next step
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) a.counts[r] = n;
}

size_t gftt_select_smem(int cap, int max_corners, int occ_bytes)
{
    return sizeof(Cand) * (size_t)cap + sizeof(float2) * (size_t)(max_corners + 64) + (size_t)occ_bytes;
}

hipError_t launch_gftt(const GfttArgs& a, int max_area, int max_w, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(a.roi_max, 0x80, sizeof(int) * a.nroi, s);  // very negative keys
    if (e == hipSuccess) e = hipMemsetAsync(a.cand_count, 0, sizeof(int) * a.nroi, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gftt_rowsum_kernel, dim3((max_area + 255) / 256, a.nroi), dim3(256), 0, s, a);
    hipLaunchKernelGGL(gftt_eig_kernel, dim3((max_w + 63) / 64, a.nroi), dim3(64), 0, s, a);
    hipLaunchKernelGGL(gftt_nms_kernel, dim3((max_area + 255) / 256, a.nroi), dim3(256), 0, s, a);
    const size_t smem = gftt_select_smem(a.cap, a.max_corners, a.occ_bytes);
    // > 64 KiB of dynamic LDS must be opted into (160 KiB per CU on gfx950)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gftt_select_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gftt_select_kernel, dim3(a.nroi), dim3(kSelThreads), smem, s, a);
    return hipGetLastError();
}

}  // namespace tbdk
