// box_fit.hip — tbdk_box_propagate: per-box similarity fit from tracked
// corner pairs + box-centre propagation (the KLT motion model of the TBD loop
// as a standalone batched call).  One wave per box: tracked pairs are
// compacted in point order into LDS 256 at a time (ballot + mbcnt), the
// getRTMatrix sums (box_fit.hpp) are accumulated wave-parallel and solved.
#include "box_fit.hpp"
#include "tbdk_internal.hpp"

namespace tbdk {

namespace {

__global__ __launch_bounds__(64) void box_propagate_kernel(const float2* __restrict__ prev, const float2* __restrict__ next,
                                                           const uint8_t* __restrict__ status,
                                                           const int32_t* __restrict__ offsets,
                                                           const tbdk_roi* __restrict__ boxes, int nboxes,
                                                           int min_points, tbdk_box_fit* __restrict__ out)
{
    constexpr int CH = 256;
    __shared__ float2 sa[CH], sb[CH];
    const int e = blockIdx.x;
    if (e >= nboxes) return;
    const int lane = threadIdx.x;
    const int beg = offsets[e], end = offsets[e + 1];
    // tracked pairs of the box, compacted in point order, summed wave-parallel
    SimilaritySums part;
    int used = 0;
    for (int c0 = beg; c0 < end; c0 += CH) {
        int m = 0;
        for (int j0 = c0; j0 < c0 + CH && j0 < end; j0 += 64) {
            const int j = j0 + lane;
            const bool ok = j < end && (status == nullptr || status[j]);
            const unsigned long long bal = __ballot(ok);
            if (ok) {
                const int pos = m + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
                sa[pos] = prev[j];
                sb[pos] = next[j];
            }
            m += __popcll(bal);
        }
        __syncthreads();
        for (int i = lane; i < m; i += 64) part.add(sa + i, sb + i, 1);
        used += m;
        __syncthreads();
    }
    SimilaritySums sums;
    sums.s00 = wave_sum_f64(part.s00);
    sums.s02 = wave_sum_f64(part.s02);
    sums.s03 = wave_sum_f64(part.s03);
    sums.b0 = wave_sum_f64(part.b0);
    sums.b1 = wave_sum_f64(part.b1);
    sums.b2 = wave_sum_f64(part.b2);
    sums.b3 = wave_sum_f64(part.b3);
    sums.m = used;
    if (lane == 0) {
        tbdk_box_fit o;
        const SimilarityFit f = sums.solve();
        o.m[0] = f.p;
        o.m[1] = -f.q;
        o.m[2] = f.tx;
        o.m[3] = f.q;
        o.m[4] = f.p;
        o.m[5] = f.ty;
        const tbdk_roi B = boxes[e];
        const double cx0 = B.x + B.width / 2, cy0 = B.y + B.height / 2;  // integer centre, as the loop
        o.cx = f.p * cx0 - f.q * cy0 + f.tx;
        o.cy = f.q * cx0 + f.p * cy0 + f.ty;
        o.npoints = sums.m;
        const double scale = sqrt(f.p * f.p + f.q * f.q);
        o.valid = (f.ok && sums.m >= min_points && scale > 0.5 && scale < 2.0 && isfinite(o.cx) && isfinite(o.cy))
                      ? 1
                      : 0;
        out[e] = o;
    }
}

}  // namespace

hipError_t launch_box_propagate(const float* prev, const float* next, const uint8_t* status, const int32_t* offsets,
                                const tbdk_roi* boxes, int nboxes, int min_points, tbdk_box_fit* out, hipStream_t s)
{
    hipLaunchKernelGGL(box_propagate_kernel, dim3(nboxes), dim3(64), 0, s, reinterpret_cast<const float2*>(prev),
                       reinterpret_cast<const float2*>(next), status, offsets, boxes, nboxes, min_points, out);
    return hipGetLastError();
}

}  // namespace tbdk
