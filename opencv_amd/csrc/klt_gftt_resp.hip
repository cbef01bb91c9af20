// klt_gftt_resp.hip — the corner response of goodFeaturesToTrack for the
// modes the fused gftt_eig_kernel does not cover: blockSize != 3 and the
// Harris response (useHarrisDetector), over the same batched ROI table.
//
// cornerEigenValsVecs (corner.cpp:237-326) with ksize 3 on each ROI as an
// isolated u8 image, BORDER_REFLECT_101, every expression in the reference's
// order (-ffp-contract=off; restated in oracle/gftt_oracle.c
// orc_corner_response):
//   1. gftt_resp_cov    : one thread per pixel: the ksize-3 Sobel rows scaled
//                         by 1/(4*blockSize*255) -> cov (Dx^2, DxDy, Dy^2), float
//   2. gftt_resp_rowsum : the boxFilter's RowSum in double (box_filter.simd.hpp:
//                         64-170, cn = 3): ksize 3 and 5 add the taps left to
//                         right (one thread per pixel); other sizes run
//                         s += (S[i+k] - S[i]) along the bordered row, one
//                         thread per row (the chain is sequential)
//   3. gftt_resp_colsum : ColumnSum<double,float> (:175-273) walked down each
//                         column by one thread, then calcMinEigenVal or
//                         calcHarris (:52-152) at the flat index of the pixel
//   4. gftt_resp_lmax   : per 56-column strip, the maximum key and the 3x3
//                         local-maximum ballots in gftt_eig_kernel's layout, so
//                         gftt_select_kernel runs unchanged on the result.
// These ROIs are rare (the TBD loop and the sample use blockSize 3, min
// eigenvalue); the launches are correct-first: HBM traffic 36 B/px of scratch
// (cov 12 + row sums 24) on top of the eigenvalue plane.
#include "tbdk_internal.hpp"

namespace tbdk {

namespace {

__device__ __forceinline__ int rrefl(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ int rfkey(float f)
{
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7FFFFFFF;
}

__device__ __forceinline__ float lane_left(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_right(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, false));
}

__device__ __forceinline__ int roi_of_strip(const GfttRoi* rois, int nroi, int b)
{
    int lo = 0, hi = nroi - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (rois[mid].cblk <= b) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

}  // namespace

__global__ __launch_bounds__(256) void gftt_resp_cov_kernel(GfttRespArgs a)
{
    const GfttRoi R = a.rois[blockIdx.y];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= R.w * R.h) return;
    const int y = i / R.w, x = i - y * R.w;
    const uint8_t* base = a.img + (size_t)R.y * a.pitch + R.x;
    const uint8_t* rr[3] = {base + (size_t)rrefl(y - 1, R.h) * a.pitch, base + (size_t)y * a.pitch,
                            base + (size_t)rrefl(y + 1, R.h) * a.pitch};
    const int xl = rrefl(x - 1, R.w), xr = rrefl(x + 1, R.w);
    const float k = a.k, k2 = a.k2;
    float rx[3], ry[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // Sobel rows in the filter engine's order (gftt_oracle.c)
        const float s0 = rr[j][xl], s1 = rr[j][x], s2 = rr[j][xr];
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
    float* c = a.cov + 3 * ((size_t)R.off + i);
    c[0] = dx * dx;
    c[1] = dx * dy;
    c[2] = dy * dy;
}

// ksize 3 / 5: (((S0 + S1) + S2) ...) per pixel
__global__ __launch_bounds__(256) void gftt_resp_rowsum_px_kernel(GfttRespArgs a)
{
    const GfttRoi R = a.rois[blockIdx.y];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= R.w * R.h) return;
    const int y = i / R.w, x = i - y * R.w;
    const float* c = a.cov + 3 * ((size_t)R.off + (size_t)y * R.w);
    const int anc = a.block / 2;
    double* d = a.rs + 3 * ((size_t)R.off + i);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        double s = (double)c[3 * rrefl(x - anc, R.w) + ch] + (double)c[3 * rrefl(x + 1 - anc, R.w) + ch];
        for (int t = 2; t < a.block; ++t) s = s + (double)c[3 * rrefl(x + t - anc, R.w) + ch];
        d[ch] = s;
    }
}

// other sizes: the running sum along the bordered row, one thread per row
__global__ __launch_bounds__(64) void gftt_resp_rowsum_run_kernel(GfttRespArgs a)
{
    const GfttRoi R = a.rois[blockIdx.y];
    const int y = blockIdx.x * 64 + threadIdx.x;
    if (y >= R.h) return;
    const float* c = a.cov + 3 * ((size_t)R.off + (size_t)y * R.w);
    double* d = a.rs + 3 * ((size_t)R.off + (size_t)y * R.w);
    const int anc = a.block / 2, B = a.block;
    double s[3] = {0.0, 0.0, 0.0};
    for (int t = 0; t < B; ++t) {
        const float* q = c + 3 * rrefl(t - anc, R.w);
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) s[ch] += (double)q[ch];
    }
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) d[ch] = s[ch];
    for (int x = 0; x + 1 < R.w; ++x) {
        const float* qa = c + 3 * rrefl(x + B - anc, R.w);
        const float* qs = c + 3 * rrefl(x - anc, R.w);
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            s[ch] += (double)qa[ch] - (double)qs[ch];
            d[3 * (x + 1) + ch] = s[ch];
        }
    }
}

// ColumnSum down each column, then the response at flat index j = y * w + x
__global__ __launch_bounds__(64) void gftt_resp_colsum_kernel(GfttRespArgs a)
{
    const GfttRoi R = a.rois[blockIdx.y];
    const int x = blockIdx.x * 64 + threadIdx.x;
    if (x >= R.w) return;
    const int B = a.block, anc = B / 2, W = R.w, H = R.h;
    const double* rs = a.rs + 3 * ((size_t)R.off + x);
    double S[3] = {0.0, 0.0, 0.0};
    for (int r = 0; r < B - 1; ++r) {
        const double* sp = rs + 3 * (size_t)rrefl(r - anc, H) * W;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) S[ch] += sp[ch];
    }
    const int64_t N = (int64_t)W * H;
    const int64_t avx_end = N & ~(int64_t)7, sse_end = avx_end + (N - avx_end >= 4 ? 4 : 0);
    float* E = a.eig + R.off + x;
    for (int y = 0; y < H; ++y) {
        const double* sp = rs + 3 * (size_t)rrefl(y - anc + B - 1, H) * W;  // entering
        const double* sm = rs + 3 * (size_t)rrefl(y - anc, H) * W;          // leaving
        float box[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const double s0 = S[ch] + sp[ch];
            box[ch] = (float)s0;
            S[ch] = s0 - sm[ch];
        }
        float e;
        if (!a.harris) {
            const float aa = box[0] * 0.5f, bb = box[1], cc = box[2] * 0.5f;
            const float t = aa - cc;
            e = (aa + cc) - sqrtf(bb * bb + t * t);
        } else {
            // calcHarris over the continuous map (corner.cpp:104-152): the AVX
            // lines, one SSE2 block, then the scalar double expression
            const float aa = box[0], bb = box[1], cc = box[2];
            const float acbb = aa * cc - bb * bb, ac = aa + cc;
            const int64_t j = (int64_t)y * W + x;
            if (j < avx_end) e = acbb - a.kf * (ac * ac);
            else if (j < sse_end) e = acbb - (a.kf * ac) * ac;
            else e = (float)((double)acbb - a.hk * (double)ac * (double)ac);
        }
        E[(size_t)y * gftt_epitch(W)] = e;
    }
}

// per strip: max key and the local-maximum ballots (gftt_eig_kernel's layout)
__global__ __launch_bounds__(64) void gftt_resp_lmax_kernel(GfttRespArgs a)
{
    const int r = roi_of_strip(a.rois, a.nroi, blockIdx.x);
    const GfttRoi R = a.rois[r];
    const int lane = threadIdx.x;
    const int strip = blockIdx.x - R.cblk;
    const int xc = strip * kGfttStrip - kGfttHalo + lane;
    const bool out_lane = lane >= kGfttHalo && lane < kGfttHalo + kGfttStrip && xc < R.w;
    const int gx = xc < 0 ? 0 : (xc >= R.w ? R.w - 1 : xc);
    const bool x_in = out_lane && gx >= 1 && gx <= R.w - 2;
    const int H = R.h;
    const float* E = a.eig + R.off + gx;
    uint64_t* lm = a.lmax + R.moff + (size_t)strip * H;
    const bool has_lm = R.w >= 3 && H >= 3;
    int best = INT_MIN;
    float e1 = 0.f, e2 = 0.f;
    for (int y = 0; y < H; ++y) {
        const float e = E[(size_t)y * gftt_epitch(R.w)];
        if (out_lane) best = rfkey(e) > best ? rfkey(e) : best;
        const int yc = y - 1;
        if (has_lm && yc >= 1 && yc <= H - 2) {  // uniform
            float m = fmaxf(e2, e);
            m = fmaxf(m, fmaxf(lane_left(e2), lane_right(e2)));
            m = fmaxf(m, fmaxf(lane_left(e1), lane_right(e1)));
            m = fmaxf(m, fmaxf(lane_left(e), lane_right(e)));
            const unsigned long long bal = __ballot(x_in && e1 >= m);
            if (lane == 0) lm[yc] = bal;
        }
        e2 = e1;
        e1 = e;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int v = __shfl_xor(best, o);
        best = v > best ? v : best;
    }
    if (lane == 0) a.blk_max[blockIdx.x] = best;
}

hipError_t launch_gftt_resp(const GfttRespArgs& a, int ncblk, int max_w, int max_h, int max_area, hipStream_t s)
{
    if (a.nroi <= 0) return hipSuccess;
    const dim3 gpx((max_area + 255) / 256, a.nroi);
    hipLaunchKernelGGL(gftt_resp_cov_kernel, gpx, dim3(256), 0, s, a);
    if (a.block == 3 || a.block == 5)
        hipLaunchKernelGGL(gftt_resp_rowsum_px_kernel, gpx, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(gftt_resp_rowsum_run_kernel, dim3((max_h + 63) / 64, a.nroi), dim3(64), 0, s, a);
    hipLaunchKernelGGL(gftt_resp_colsum_kernel, dim3((max_w + 63) / 64, a.nroi), dim3(64), 0, s, a);
    hipLaunchKernelGGL(gftt_resp_lmax_kernel, dim3(ncblk), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace tbdk
