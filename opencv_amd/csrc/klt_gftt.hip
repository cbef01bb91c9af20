// klt_gftt.hip — Shi-Tomasi corners (goodFeaturesToTrack, min-eigenvalue
// variant) over many isolated ROIs of a frame, for gfx950.
//
// Per-ROI semantics are those of cv::goodFeaturesToTrack on the ROI as an
// isolated image (imgproc/src/featureselect.cpp:361-516 with
// cornerMinEigenVal, corner.cpp:52-101,237-326), in the float/double
// evaluation order documented in oracle/gftt_oracle.c; built with
// -ffp-contract=off so every expression rounds exactly as written.
//
// Three launches, all ROIs batched in each (one frame's re-detect set):
//   1. gftt_cov   : one thread per ROI pixel: Sobel 3x3 (reflect-101 inside the
//                   ROI) -> cov = (Dx^2, DxDy, Dy^2), three float planes
//   2. gftt_eig   : one thread per ROI column: boxFilter 3x3 with the reference's
//                   double row sums and running column sum walked top to bottom,
//                   min eigenvalue, per-ROI max (ordered-int atomicMax)
//   3. gftt_select: one 256-thread workgroup per ROI: threshold-to-zero at
//                   max*q, 3x3 non-max test, candidates compacted into LDS,
//                   bitonic sort by (value desc, address desc) — the reference's
//                   deterministic tie-break (featureselect.cpp:56-64) — then the
//                   greedy min-distance walk by one wave with wave-parallel
//                   distance tests against the accepted set.
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

}  // namespace

__global__ __launch_bounds__(256) void gftt_cov_kernel(GfttArgs a)
{
    const int r = blockIdx.y;
    const GfttRoi R = a.rois[r];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= R.w * R.h) return;
    const int y = p / R.w, x = p - y * R.w;
    const double scale = 1.0 / ((double)(1 << 2) * 3 * 255.0);
    const float k = (float)(1.0 * scale), k2 = (float)(2.0 * scale);
    const int xl = refl(x - 1, R.w), xr = refl(x + 1, R.w);
    float rx[3], ry[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const uint8_t* s = a.img + (size_t)(R.y + refl(y + j - 1, R.h)) * a.pitch + R.x;
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
    const size_t o = (size_t)R.off + p;
    a.cov0[o] = dx * dx;
    a.cov1[o] = dx * dy;
    a.cov2[o] = dy * dy;
}

__global__ __launch_bounds__(256) void gftt_eig_kernel(GfttArgs a)
{
    const int r = blockIdx.y;
    const GfttRoi R = a.rois[r];
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= R.w) return;
    const int xl = refl(x - 1, R.w), xr = refl(x + 1, R.w);
    const float* c0 = a.cov0 + R.off;
    const float* c1 = a.cov1 + R.off;
    const float* c2 = a.cov2 + R.off;
    auto rowsum = [&](int yy, double& s0, double& s1, double& s2) {
        const size_t b = (size_t)refl(yy, R.h) * R.w;
        s0 = (double)c0[b + xl] + (double)c0[b + x] + (double)c0[b + xr];
        s1 = (double)c1[b + xl] + (double)c1[b + x] + (double)c1[b + xr];
        s2 = (double)c2[b + xl] + (double)c2[b + x] + (double)c2[b + xr];
    };
    double m0, m1, m2, n0, n1, n2, S0, S1, S2;
    rowsum(-1, m0, m1, m2);
    S0 = 0.0 + m0;
    S1 = 0.0 + m1;
    S2 = 0.0 + m2;
    rowsum(0, n0, n1, n2);
    S0 = S0 + n0;
    S1 = S1 + n1;
    S2 = S2 + n2;
    int best = INT_MIN;
    for (int y = 0; y < R.h; ++y) {
        double p0, p1, p2;
        rowsum(y + 1, p0, p1, p2);  // entering row
        double q0, q1, q2;
        rowsum(y - 1, q0, q1, q2);  // leaving row
        const double t0 = S0 + p0, t1 = S1 + p1, t2 = S2 + p2;
        const float aa = (float)t0 * 0.5f, bb = (float)t1, cc = (float)t2 * 0.5f;
        S0 = t0 - q0;
        S1 = t1 - q1;
        S2 = t2 - q2;
        const float t = aa - cc;
        const float e = (aa + cc) - sqrtf(bb * bb + t * t);
        a.eig[(size_t)R.off + (size_t)y * R.w + x] = e;
        const int kk = fkey(e);
        best = kk > best ? kk : best;
    }
    atomicMax(&a.roi_max[r], best);
}

struct Cand {
    float v;
    int idx;
};

// a before b in the reference order: value desc, then address desc
__device__ __forceinline__ bool cand_before(const Cand& a, const Cand& b)
{
    return a.v > b.v || (a.v == b.v && a.idx > b.idx);
}

__global__ __launch_bounds__(256) void gftt_select_kernel(GfttArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int& s_count = *reinterpret_cast<int*>(smem);  // all LDS in the one dynamic region
    Cand* cand = reinterpret_cast<Cand*>(smem + 16);
    float2* acc = reinterpret_cast<float2*>(smem + 16 + sizeof(Cand) * a.cap);
    const int r = blockIdx.x;
    const GfttRoi R = a.rois[r];
    const int tid = threadIdx.x;
    if (tid == 0) s_count = 0;
    __syncthreads();
    const float maxv = fkey_inv(a.roi_max[r]);
    const float thr = (float)((double)maxv * a.quality);
    const float* E = a.eig + R.off;
    // threshold-to-zero + 3x3 dilate-equal test on interior pixels
    auto ev = [&](int yy, int xx) {
        const float v = E[(size_t)yy * R.w + xx];
        return v > thr ? v : 0.f;
    };
    const int iw = R.w - 2, ih = R.h - 2;
    for (int p = tid; p < (iw > 0 && ih > 0 ? iw * ih : 0); p += blockDim.x) {
        const int y = p / iw + 1, x = p % iw + 1;
        const float v = ev(y, x);
        if (v == 0.f) continue;
        float m = v;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const float q = ev(y + dy, x + dx);
                m = q > m ? q : m;
            }
        if (v == m) {
            const int slot = atomicAdd(&s_count, 1);
            if (slot < a.cap) cand[slot] = Cand{v, y * R.w + x};
        }
    }
    __syncthreads();
    const int total = s_count;
    if (total > a.cap) {  // candidate buffer overflow: report, never silently truncate
        if (tid == 0) a.counts[r] = -1;
        return;
    }
    int np2 = 1;
    while (np2 < total) np2 <<= 1;
    for (int i = total + tid; i < np2; i += blockDim.x) cand[i] = Cand{-FLT_MAX, -1};
    __syncthreads();
    // bitonic sort, "before" order first
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < np2; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const bool up = (i & k) == 0;
                    Cand ci = cand[i], cj = cand[ixj];
                    const bool swap = up ? cand_before(cj, ci) : cand_before(ci, cj);
                    if (swap) {
                        cand[i] = cj;
                        cand[ixj] = ci;
                    }
                }
            }
            __syncthreads();
        }
    }
    // greedy selection (featureselect.cpp:421-503) by wave 0
    if (tid < 64) {
        const int lane = tid;
        int n = 0;
        const bool use_dist = a.min_distance >= 1.0;
        const double md2 = a.min_distance * a.min_distance;
        float2* out = a.corners + (size_t)r * a.max_corners;
        for (int i = 0; i < total; ++i) {
            const int idx = cand[i].idx;
            const int y = idx / R.w, x = idx - y * R.w;
            bool good = true;
            if (use_dist) {
                bool conflict = false;
                for (int q = lane; q < n; q += 64) {
                    const float dx = (float)x - acc[q].x, dy = (float)y - acc[q].y;
                    conflict |= (double)(dx * dx + dy * dy) < md2;
                }
                good = __ballot(conflict) == 0ull;
            }
            if (good) {
                if (lane == 0) {
                    acc[n] = make_float2((float)x, (float)y);
                    out[n] = make_float2((float)(x + R.x), (float)(y + R.y));
                }
                n++;
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): acc[n-1] visible to all lanes
                __builtin_amdgcn_wave_barrier();
                if (a.max_corners > 0 && n == a.max_corners) break;
            }
        }
        if (lane == 0) a.counts[r] = n;
    }
}

size_t gftt_select_smem(int cap, int max_corners)
{
    return 16 + sizeof(Cand) * (size_t)cap + sizeof(float2) * (size_t)(max_corners > 0 ? max_corners : cap);
}

hipError_t launch_gftt(const GfttArgs& a, int max_area, int max_w, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(a.roi_max, 0x80, sizeof(int) * a.nroi, s);  // INT_MIN-ish keys
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gftt_cov_kernel, dim3((max_area + 255) / 256, a.nroi), dim3(256), 0, s, a);
    hipLaunchKernelGGL(gftt_eig_kernel, dim3((max_w + 255) / 256, a.nroi), dim3(256), 0, s, a);
    const size_t smem = gftt_select_smem(a.cap, a.max_corners);
    // > 64 KiB of dynamic LDS must be opted into (160 KiB per CU on gfx950)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gftt_select_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gftt_select_kernel, dim3(a.nroi), dim3(256), smem, s, a);
    return hipGetLastError();
}

}  // namespace tbdk
