// box_fit.hpp — 4-DOF similarity fit of point correspondences, the non-full-
// affine branch of getRTMatrix (video/src/lkpyramid.cpp:1398-1470), used by
// the KLT box propagation.  The sums follow the reference exactly (float
// products of Point2f, accumulated in double, in point order); the 4x4 normal
// system is solved in closed form (the reference calls cv::solve(DECOMP_EIG):
// the two agree to double rounding, see tests/test_gpu_box_fit.py).
#pragma once

#include <hip/hip_runtime.h>

namespace tbdk {

struct SimilarityFit {
    double p, q, tx, ty;  // M = [p -q tx; q p ty]
    int ok;               // normal matrix not singular
};

struct SimilaritySums {
    double s00 = 0, s02 = 0, s03 = 0, b0 = 0, b1 = 0, b2 = 0, b3 = 0;
    int m = 0;

    // a[i] -> b[i], i in [0, k), appended in order (lkpyramid.cpp:1445-1454)
    template <class P>
    __host__ __device__ void add(P a, P b, int k)
    {
        for (int i = 0; i < k; ++i) {
            const float ax = a[i].x, ay = a[i].y, bx = b[i].x, by = b[i].y;
            s00 += ax * ax + ay * ay;
            s02 += ax;
            s03 += ay;
            b0 += ax * bx + ay * by;
            b1 += ax * by - ay * bx;
            b2 += bx;
            b3 += by;
        }
        m += k;
    }

    // [s00 0 s02 s03; 0 s00 -s03 s02; s02 -s03 n 0; s03 s02 0 n] [p q tx ty]^T = [b0 b1 b2 b3]^T
    __host__ __device__ SimilarityFit solve() const
    {
        SimilarityFit f{1.0, 0.0, 0.0, 0.0, 0};
        if (m <= 0) return f;
        const double n = (double)m;
        const double den = s00 - (s02 * s02 + s03 * s03) / n;
        if (!(den > 1e-9)) return f;
        f.p = (b0 - (s02 * b2 + s03 * b3) / n) / den;
        f.q = (b1 + (s03 * b2 - s02 * b3) / n) / den;
        f.tx = (b2 - s02 * f.p + s03 * f.q) / n;
        f.ty = (b3 - s03 * f.p - s02 * f.q) / n;
        f.ok = 1;
        return f;
    }
};

#if defined(__HIPCC__)
__device__ __forceinline__ double wave_sum_f64(double v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Wave-parallel form: lane l sums pairs l, l+64, ... in order, then a fixed
// xor-butterfly combines the 64 partial sums (deterministic; differs from the
// sequential order only by double rounding, like the reference's own solve).
__device__ inline SimilarityFit wave_fit_similarity(const float2* a, const float2* b, int m, int lane)
{
    SimilaritySums p;
    for (int i = lane; i < m; i += 64) p.add(a + i, b + i, 1);
    SimilaritySums s;
    s.s00 = wave_sum_f64(p.s00);
    s.s02 = wave_sum_f64(p.s02);
    s.s03 = wave_sum_f64(p.s03);
    s.b0 = wave_sum_f64(p.b0);
    s.b1 = wave_sum_f64(p.b1);
    s.b2 = wave_sum_f64(p.b2);
    s.b3 = wave_sum_f64(p.b3);
    s.m = m;
    return s.solve();
}
#endif

template <class P>
__host__ __device__ inline SimilarityFit fit_similarity(P a, P b, int m)
{
    SimilaritySums s;
    s.add(a, b, m);
    return s.solve();
}

}  // namespace tbdk
