/*
 * farneback_oracle.c — CPU restatement of the reference's dense Farneback
 * optical flow (cv::calcOpticalFlowFarneback / FarnebackOpticalFlowImpl::calc,
 * modules/video/src/optflowgf.cpp:57-578, 1096-1190).
 *
 * TEST INFRASTRUCTURE ONLY: tests/ use it as the checker of libtbdk's
 * farneback.hip; the product never links it.
 *
 * Restated, with the reference's float/double operation order:
 *   FarnebackPrepareGaussian   optflowgf.cpp:60-114 (6x6 G, inverse by
 *                              hal::Cholesky64f, core/src/matrix_decomp.cpp:95-170)
 *   FarnebackPolyExp           optflowgf.cpp:116-202
 *   FarnebackUpdateMatrices    optflowgf.cpp:217-312
 *   FarnebackUpdateFlow_Blur   optflowgf.cpp:314-405
 *   FarnebackUpdateFlow_GaussianBlur  optflowgf.cpp:407-578
 *   calc (level loop)          optflowgf.cpp:1096-1190
 * and the imgproc pieces calc uses on float images:
 *   getGaussianKernel          imgproc/src/smooth.dispatch.cpp:70-122
 *   GaussianBlur -> sepFilter2D (REFLECT_101): SymmRowSmallFilter (ksize <= 5) /
 *                              RowFilter, SymmColumnSmallFilter (ksize 3) /
 *                              SymmColumnFilter (imgproc/src/filter.simd.hpp:2330-2450, 2590-2790)
 *   resize INTER_LINEAR        imgproc/src/resize.cpp:3483-3700 (+ the exact-2x
 *                              INTER_AREA fast path, :3519-3550, 2479-2500, 2600-2640)
 *
 * The optflowgf.cpp functions are restated literally (running sums, stripe
 * updates).  orc_fb_calc_mode(..., box_direct=1) swaps the box blur's
 * image-long running sums for the fixed-order window sums of
 * orc_fb_update_flow_blur_direct (restarted every 4 rows / columns), the order
 * the GPU kernel uses, so that the GPU is checked bit for bit against it and
 * this mode against the reference's within a tolerance.
 * Known deviation: the imgproc SIMD paths (GaussianBlur's filter engine,
 * resize) may be built with FMA under AVX2 dispatch on the reference's host;
 * their scalar/SSE orders are restated here.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define FB_GAUSSIAN 256
#define FB_USE_INITIAL_FLOW 4

static int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* getGaussianKernel(n, sigma, CV_32F) */
void orc_fb_gaussian_kernel(int n, double sigma, float* cf)
{
    static const float tab[4][7] = {{1.f},
                                    {0.25f, 0.5f, 0.25f},
                                    {0.0625f, 0.25f, 0.375f, 0.25f, 0.0625f},
                                    {0.03125f, 0.109375f, 0.21875f, 0.28125f, 0.21875f, 0.109375f, 0.03125f}};
    const float* fixed = (n % 2 == 1 && n <= 7 && sigma <= 0) ? tab[n >> 1] : 0;
    double sigmaX = sigma > 0 ? sigma : ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
    double scale2X = -0.5 / (sigmaX * sigmaX);
    double sum = 0;
    for (int i = 0; i < n; i++) {
        double x = i - (n - 1) * 0.5;
        double t = fixed ? (double)fixed[i] : exp(scale2X * x * x);
        cf[i] = (float)t;
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; i++) cf[i] = (float)(cf[i] * sum);
}

/* GaussianBlur(src, dst, Size(ksize, ksize), sigma, sigma) on a float image,
 * BORDER_REFLECT_101: row filter into a buffer, then the column filter. */
void orc_fb_gauss_blur(const float* src, int w, int h, float* dst, int ksize, double sigma)
{
    float* k = malloc(sizeof(float) * (size_t)ksize);
    orc_fb_gaussian_kernel(ksize, sigma, k);
    const int r = ksize / 2;
    float* buf = malloc(sizeof(float) * (size_t)w * h);
    for (int y = 0; y < h; y++) {
        const float* S = src + (size_t)y * w;
        float* D = buf + (size_t)y * w;
        for (int x = 0; x < w; x++) {
#define SX(o) S[reflect101(x + (o), w)]
            float s;
            if (ksize == 3)
                s = SX(0) * k[1] + (SX(-1) + SX(1)) * k[0];
            else if (ksize == 5)
                s = SX(0) * k[2] + (SX(-1) + SX(1)) * k[1] + (SX(-2) + SX(2)) * k[0];
            else {
                s = k[0] * SX(-r);
                for (int j = 1; j < ksize; j++) s += k[j] * SX(j - r);
            }
#undef SX
            D[x] = s;
        }
    }
    for (int y = 0; y < h; y++) {
        float* D = dst + (size_t)y * w;
        for (int x = 0; x < w; x++) {
#define SY(o) buf[(size_t)reflect101(y + (o), h) * w + x]
            float s;
            if (ksize == 3) {
                s = (SY(-1) + SY(1)) * k[0] + SY(0) * k[1] + 0.0f;
            } else {
                s = k[r] * SY(0) + 0.0f;
                for (int j = 1; j <= r; j++) s += k[r + j] * (SY(j) + SY(-j));
            }
#undef SY
            D[x] = s;
        }
    }
    free(buf);
    free(k);
}

/* resize(src, dst, Size(dw, dh), 0, 0, INTER_LINEAR) for float, cn channels */
void orc_fb_resize_linear(const float* src, int sw, int sh, int cn, float* dst, int dw, int dh)
{
    const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
    const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    const int isx = (int)lrint(scale_x), isy = (int)lrint(scale_y);
    const int area_fast = fabs(scale_x - isx) < DBL_EPSILON && fabs(scale_y - isy) < DBL_EPSILON;
    if (area_fast && isx == 2 && isy == 2 && cn == 1) {
        const int vec = dw & ~3;  /* 4-lane SIMD part, scalar tail */
        for (int dy = 0; dy < dh; dy++) {
            const float* S0 = src + (size_t)(2 * dy) * sw;
            const float* S1 = S0 + sw;
            float* D = dst + (size_t)dy * dw;
            for (int dx = 0; dx < dw; dx++) {
                const float a = S0[2 * dx], b = S0[2 * dx + 1], c = S1[2 * dx], d = S1[2 * dx + 1];
                if (dx < vec) {
                    D[dx] = ((a + b) + (c + d)) * 0.25f;
                } else {
                    float sum = 0;
                    sum += a + b + c + d;
                    D[dx] = sum * 0.25f;
                }
            }
        }
        return;
    }
    int* xofs = malloc(sizeof(int) * (size_t)dw);
    float* alpha = malloc(sizeof(float) * 2 * (size_t)dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        alpha[2 * dx] = 1.f - fx;
        alpha[2 * dx + 1] = fx;
    }
    float* row0 = malloc(sizeof(float) * (size_t)dw * cn);
    float* row1 = malloc(sizeof(float) * (size_t)dw * cn);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)floorf(fy);
        fy -= sy;
        const float b0 = 1.f - fy, b1 = fy;
        for (int k = 0; k < 2; k++) {
            const float* S = src + (size_t)clampi(sy + k, 0, sh - 1) * sw * cn;
            float* R = k ? row1 : row0;
            for (int dx = 0; dx < dw; dx++)
                for (int c = 0; c < cn; c++) {
                    const int s = xofs[dx] * cn + c;
                    R[dx * cn + c] = dx < xmax ? S[s] * alpha[2 * dx] + S[s + cn] * alpha[2 * dx + 1] : S[s];
                }
        }
        float* D = dst + (size_t)dy * dw * cn;
        for (int x = 0; x < dw * cn; x++) D[x] = row0[x] * b0 + row1[x] * b1;
    }
    free(row0);
    free(row1);
    free(xofs);
    free(alpha);
}

/* resize(src, dst, Size(dw, dh), 0, 0, INTER_AREA) for a float image of cn
 * channels, downscaling only (imgproc/src/resize.cpp):
 *   same size          -> copy (cv::resize, :3745-3750)
 *   integer factors    -> resizeAreaFast_ (:3530-3553, invoker :2600-2666): the
 *                         SIMD hook only serves cn 1/4 at 2x2 (:2476), so cn 2 takes
 *                         the scalar loop, summed in unrolled groups of 4
 *                         (sum += ((a+b)+c)+d) then * (1.f/area).  The partial-cell
 *                         branch cannot run: an integer factor means dw*isx == sw.
 *   otherwise          -> computeResizeAreaTab (:2853-2892) + ResizeArea_Invoker
 *                         (:2710-2814): per source row, buf += S*alpha over the x
 *                         table; per output row, sum of beta*buf in table order.
 * inv_sx/inv_sy are cv::resize's inv_scale (dsize/ssize, or fx/fy when dsize is
 * empty). */
void orc_fb_resize_area_fx(const float* src, int sw, int sh, int cn, float* dst, int dw, int dh, double inv_sx,
                           double inv_sy)
{
    if (dw == sw && dh == sh) {
        if (dst != src) memcpy(dst, src, sizeof(float) * (size_t)sw * sh * cn);
        return;
    }
    const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    const int isx = (int)lrint(scale_x), isy = (int)lrint(scale_y);
    if (fabs(scale_x - isx) < DBL_EPSILON && fabs(scale_y - isy) < DBL_EPSILON) {
        const int area = isx * isy;
        const float sc = 1.f / area;
        int* ofs = malloc(sizeof(int) * (size_t)area);
        for (int sy = 0, k = 0; sy < isy; sy++)
            for (int sx = 0; sx < isx; sx++) ofs[k++] = sy * sw * cn + sx * cn;
        for (int dy = 0; dy < dh; dy++)
            for (int dx = 0; dx < dw * cn; dx++) {
                const float* S = src + (size_t)dy * isy * sw * cn + (dx / cn) * isx * cn + dx % cn;
                float sum = 0;
                int k = 0;
                for (; k <= area - 4; k += 4) sum += S[ofs[k]] + S[ofs[k + 1]] + S[ofs[k + 2]] + S[ofs[k + 3]];
                for (; k < area; k++) sum += S[ofs[k]];
                dst[(size_t)dy * dw * cn + dx] = sum * sc;
            }
        free(ofs);
        return;
    }
    /* tables: (si, di, alpha) triples in the reference's order */
    int* xsi = malloc(sizeof(int) * 2 * (size_t)sw);
    int* xdi = malloc(sizeof(int) * 2 * (size_t)sw);
    float* xal = malloc(sizeof(float) * 2 * (size_t)sw);
    int* ysi = malloc(sizeof(int) * 2 * (size_t)sh);
    int* ydi = malloc(sizeof(int) * 2 * (size_t)sh);
    float* yal = malloc(sizeof(float) * 2 * (size_t)sh);
    int nt[2];
    for (int t = 0; t < 2; t++) {
        const int ss = t ? sh : sw, ds = t ? dh : dw, c = t ? 1 : cn;
        const double scale = t ? scale_y : scale_x;
        int *si = t ? ysi : xsi, *di = t ? ydi : xdi;
        float* al = t ? yal : xal;
        int k = 0;
        for (int d = 0; d < ds; d++) {
            const double f1 = d * scale, f2 = f1 + scale;
            const double cell = scale < ss - f1 ? scale : ss - f1;
            int s1 = (int)ceil(f1), s2 = (int)floor(f2);
            s2 = s2 < ss - 1 ? s2 : ss - 1;
            s1 = s1 < s2 ? s1 : s2;
            if (s1 - f1 > 1e-3) {
                di[k] = d * c, si[k] = (s1 - 1) * c, al[k++] = (float)((s1 - f1) / cell);
            }
            for (int x = s1; x < s2; x++) di[k] = d * c, si[k] = x * c, al[k++] = (float)(1.0 / cell);
            if (f2 - s2 > 1e-3) {
                double r = f2 - s2 < 1. ? f2 - s2 : 1.;
                r = r < cell ? r : cell;
                di[k] = d * c, si[k] = s2 * c, al[k++] = (float)(r / cell);
            }
        }
        nt[t] = k;
    }
    const int W = dw * cn;
    float* buf = malloc(sizeof(float) * (size_t)W);
    float* sum = malloc(sizeof(float) * (size_t)W);
    for (int x = 0; x < W; x++) sum[x] = 0;
    int prev_dy = ydi[0];
    for (int j = 0; j < nt[1]; j++) {
        const float beta = yal[j];
        const int dy = ydi[j];
        const float* S = src + (size_t)ysi[j] * sw * cn;
        for (int x = 0; x < W; x++) buf[x] = 0;
        for (int k = 0; k < nt[0]; k++)
            for (int c = 0; c < cn; c++) buf[xdi[k] + c] = buf[xdi[k] + c] + S[xsi[k] + c] * xal[k];
        if (dy != prev_dy) {
            float* D = dst + (size_t)prev_dy * W;
            for (int x = 0; x < W; x++) {
                D[x] = sum[x];
                sum[x] = beta * buf[x];
            }
            prev_dy = dy;
        } else {
            for (int x = 0; x < W; x++) sum[x] += beta * buf[x];
        }
    }
    memcpy(dst + (size_t)prev_dy * W, sum, sizeof(float) * (size_t)W);
    free(buf);
    free(sum);
    free(xsi);
    free(xdi);
    free(xal);
    free(ysi);
    free(ydi);
    free(yal);
}

/* resize with an explicit dsize: inv_scale = dsize / ssize (cv::resize) */
void orc_fb_resize_area(const float* src, int sw, int sh, int cn, float* dst, int dw, int dh)
{
    orc_fb_resize_area_fx(src, sw, sh, cn, dst, dw, dh, (double)dw / sw, (double)dh / sh);
}

/* FarnebackPrepareGaussian: g, xg, xxg (length 2n+1, centred) and ig11/03/33/55 */
void orc_fb_prepare_gaussian(int n, double sigma, float* g_, float* xg_, float* xxg_, double* ig)
{
    float* g = g_ + n;
    float* xg = xg_ + n;
    float* xxg = xxg_ + n;
    if (sigma < FLT_EPSILON) sigma = n * 0.3;
    double s = 0.;
    for (int x = -n; x <= n; x++) {
        g[x] = (float)exp(-x * x / (2 * sigma * sigma));
        s += g[x];
    }
    s = 1. / s;
    for (int x = -n; x <= n; x++) {
        g[x] = (float)(g[x] * s);
        xg[x] = (float)(x * g[x]);
        xxg[x] = (float)(x * x * g[x]);
    }
    double G[36] = {0};
#define GG(i, j) G[(i)*6 + (j)]
    for (int y = -n; y <= n; y++)
        for (int x = -n; x <= n; x++) {
            GG(0, 0) += g[y] * g[x];
            GG(1, 1) += g[y] * g[x] * x * x;
            GG(3, 3) += g[y] * g[x] * x * x * x * x;
            GG(5, 5) += g[y] * g[x] * x * x * y * y;
        }
    GG(2, 2) = GG(0, 3) = GG(0, 4) = GG(3, 0) = GG(4, 0) = GG(1, 1);
    GG(4, 4) = GG(3, 3);
    GG(3, 4) = GG(4, 3) = GG(5, 5);
    /* invert(G, DECOMP_CHOLESKY): hal::Cholesky64f(A, m=6, b=I, n=6) */
    double* A = G;
    double b[36] = {0};
    for (int i = 0; i < 6; i++) b[i * 6 + i] = 1;
    int i, j, k;
    for (i = 0; i < 6; i++) {
        for (j = 0; j < i; j++) {
            s = A[i * 6 + j];
            for (k = 0; k < j; k++) s -= A[i * 6 + k] * A[j * 6 + k];
            A[i * 6 + j] = s * A[j * 6 + j];
        }
        s = A[i * 6 + i];
        for (k = 0; k < j; k++) {
            double t = A[i * 6 + k];
            s -= t * t;
        }
        A[i * 6 + i] = 1. / sqrt(s);
    }
    for (i = 0; i < 6; i++)
        for (j = 0; j < 6; j++) {
            s = b[i * 6 + j];
            for (k = 0; k < i; k++) s -= A[i * 6 + k] * b[k * 6 + j];
            b[i * 6 + j] = s * A[i * 6 + i];
        }
    for (i = 5; i >= 0; i--)
        for (j = 0; j < 6; j++) {
            s = b[i * 6 + j];
            for (k = 5; k > i; k--) s -= A[k * 6 + i] * b[k * 6 + j];
            b[i * 6 + j] = s * A[i * 6 + i];
        }
    ig[0] = b[1 * 6 + 1];
    ig[1] = b[0 * 6 + 3];
    ig[2] = b[3 * 6 + 3];
    ig[3] = b[5 * 6 + 5];
#undef GG
}

/* FarnebackPolyExp: dst = 5 floats per pixel (AoS, the reference's CV_32FC5) */
void orc_fb_poly_exp(const float* src, int width, int height, int n, double sigma, float* dst)
{
    float kbuf[64], xgb[64], xxgb[64];
    double ig[4];
    orc_fb_prepare_gaussian(n, sigma, kbuf, xgb, xxgb, ig);
    const float* g = kbuf + n;
    const float* xg = xgb + n;
    const float* xxg = xxgb + n;
    const double ig11 = ig[0], ig03 = ig[1], ig33 = ig[2], ig55 = ig[3];
    float* rowbuf = malloc(sizeof(float) * (size_t)(width + n * 2) * 3);
    float* row = rowbuf + n * 3;
    for (int y = 0; y < height; y++) {
        float g0 = g[0], g1, g2;
        const float* srow0 = src + (size_t)y * width;
        float* drow = dst + (size_t)y * width * 5;
        for (int x = 0; x < width; x++) {
            row[x * 3] = srow0[x] * g0;
            row[x * 3 + 1] = row[x * 3 + 2] = 0.f;
        }
        for (int k = 1; k <= n; k++) {
            g0 = g[k];
            g1 = xg[k];
            g2 = xxg[k];
            const float* s0 = src + (size_t)(y - k < 0 ? 0 : y - k) * width;
            const float* s1 = src + (size_t)(y + k > height - 1 ? height - 1 : y + k) * width;
            for (int x = 0; x < width; x++) {
                float p = s0[x] + s1[x];
                float t0 = row[x * 3] + g0 * p;
                float t1 = row[x * 3 + 1] + g1 * (s1[x] - s0[x]);
                float t2 = row[x * 3 + 2] + g2 * p;
                row[x * 3] = t0;
                row[x * 3 + 1] = t1;
                row[x * 3 + 2] = t2;
            }
        }
        for (int x = 0; x < n * 3; x++) {
            row[-1 - x] = row[2 - x];
            row[width * 3 + x] = row[width * 3 + x - 3];
        }
        for (int x = 0; x < width; x++) {
            g0 = g[0];
            double b1 = row[x * 3] * g0, b2 = 0, b3 = row[x * 3 + 1] * g0, b4 = 0, b5 = row[x * 3 + 2] * g0, b6 = 0;
            for (int k = 1; k <= n; k++) {
                double tg = row[(x + k) * 3] + row[(x - k) * 3];
                g0 = g[k];
                b1 += tg * g0;
                b4 += tg * xxg[k];
                b2 += (row[(x + k) * 3] - row[(x - k) * 3]) * xg[k];
                b3 += (row[(x + k) * 3 + 1] + row[(x - k) * 3 + 1]) * g0;
                b6 += (row[(x + k) * 3 + 1] - row[(x - k) * 3 + 1]) * xg[k];
                b5 += (row[(x + k) * 3 + 2] + row[(x - k) * 3 + 2]) * g0;
            }
            drow[x * 5 + 1] = (float)(b2 * ig11);
            drow[x * 5] = (float)(b3 * ig11);
            drow[x * 5 + 3] = (float)(b1 * ig03 + b4 * ig33);
            drow[x * 5 + 2] = (float)(b1 * ig03 + b5 * ig33);
            drow[x * 5 + 4] = (float)(b6 * ig55);
        }
    }
    free(rowbuf);
}

/* FarnebackUpdateMatrices over rows [y0, y1) */
void orc_fb_update_matrices(const float* R0_, const float* R1, const float* flow_, int width, int height, float* M_,
                            int y0, int y1)
{
    static const float border[5] = {0.14f, 0.14f, 0.4472f, 0.4472f, 0.4472f};
    const size_t step1 = (size_t)width * 5;
    for (int y = y0; y < y1; y++) {
        const float* flow = flow_ + (size_t)y * width * 2;
        const float* R0 = R0_ + (size_t)y * step1;
        float* M = M_ + (size_t)y * step1;
        for (int x = 0; x < width; x++) {
            float dx = flow[x * 2], dy = flow[x * 2 + 1];
            float fx = x + dx, fy = y + dy;
            int x1 = (int)floorf(fx), y1_ = (int)floorf(fy);
            float r2, r3, r4, r5, r6;
            fx -= x1;
            fy -= y1_;
            if ((unsigned)x1 < (unsigned)(width - 1) && (unsigned)y1_ < (unsigned)(height - 1)) {
                const float* ptr = R1 + (size_t)y1_ * step1 + (size_t)x1 * 5;
                float a00 = (1.f - fx) * (1.f - fy), a01 = fx * (1.f - fy), a10 = (1.f - fx) * fy, a11 = fx * fy;
                r2 = a00 * ptr[0] + a01 * ptr[5] + a10 * ptr[step1] + a11 * ptr[step1 + 5];
                r3 = a00 * ptr[1] + a01 * ptr[6] + a10 * ptr[step1 + 1] + a11 * ptr[step1 + 6];
                r4 = a00 * ptr[2] + a01 * ptr[7] + a10 * ptr[step1 + 2] + a11 * ptr[step1 + 7];
                r5 = a00 * ptr[3] + a01 * ptr[8] + a10 * ptr[step1 + 3] + a11 * ptr[step1 + 8];
                r6 = a00 * ptr[4] + a01 * ptr[9] + a10 * ptr[step1 + 4] + a11 * ptr[step1 + 9];
                r4 = (R0[x * 5 + 2] + r4) * 0.5f;
                r5 = (R0[x * 5 + 3] + r5) * 0.5f;
                r6 = (R0[x * 5 + 4] + r6) * 0.25f;
            } else {
                r2 = r3 = 0.f;
                r4 = R0[x * 5 + 2];
                r5 = R0[x * 5 + 3];
                r6 = R0[x * 5 + 4] * 0.5f;
            }
            r2 = (R0[x * 5] - r2) * 0.5f;
            r3 = (R0[x * 5 + 1] - r3) * 0.5f;
            r2 += r4 * dy + r6 * dx;
            r3 += r6 * dy + r5 * dx;
            if ((unsigned)(x - 5) >= (unsigned)(width - 10) || (unsigned)(y - 5) >= (unsigned)(height - 10)) {
                float scale = (x < 5 ? border[x] : 1.f) * (x >= width - 5 ? border[width - x - 1] : 1.f) *
                              (y < 5 ? border[y] : 1.f) * (y >= height - 5 ? border[height - y - 1] : 1.f);
                r2 *= scale;
                r3 *= scale;
                r4 *= scale;
                r5 *= scale;
                r6 *= scale;
            }
            M[x * 5] = r4 * r4 + r6 * r6;
            M[x * 5 + 1] = (r4 + r5) * r6;
            M[x * 5 + 2] = r5 * r5 + r6 * r6;
            M[x * 5 + 3] = r4 * r2 + r6 * r3;
            M[x * 5 + 4] = r6 * r2 + r5 * r3;
        }
    }
}

/* FarnebackUpdateFlow_Blur, literally: double running sums (vertical over
 * clamped rows, horizontal over replicated columns), the solve, and the
 * matrices updated in stripes behind the box filter */
void orc_fb_update_flow_blur(const float* R0, const float* R1, float* flow_, float* M, int width, int height,
                             int block_size, int update)
{
    int x, y, m = block_size / 2;
    int y0 = 0, y1;
    int min_update_stripe = (1 << 10) / width > block_size ? (1 << 10) / width : block_size;
    double scale = 1. / (block_size * block_size);
    double* vsum_ = malloc(sizeof(double) * (size_t)(width + m * 2 + 2) * 5);
    double* vsum = vsum_ + (m + 1) * 5;
    const size_t step = (size_t)width * 5;
    const float* srow0 = M;
    for (x = 0; x < width * 5; x++) vsum[x] = srow0[x] * (m + 2);
    for (y = 1; y < m; y++) {
        srow0 = M + (size_t)(y < height - 1 ? y : height - 1) * step;
        for (x = 0; x < width * 5; x++) vsum[x] += srow0[x];
    }
    for (y = 0; y < height; y++) {
        double g11, g12, g22, h1, h2;
        float* flow = flow_ + (size_t)y * width * 2;
        srow0 = M + (size_t)(y - m - 1 > 0 ? y - m - 1 : 0) * step;
        const float* srow1 = M + (size_t)(y + m < height - 1 ? y + m : height - 1) * step;
        for (x = 0; x < width * 5; x++) vsum[x] += srow1[x] - srow0[x];
        for (x = 0; x < (m + 1) * 5; x++) {
            vsum[-1 - x] = vsum[4 - x];
            vsum[width * 5 + x] = vsum[width * 5 + x - 5];
        }
        g11 = vsum[0] * (m + 2);
        g12 = vsum[1] * (m + 2);
        g22 = vsum[2] * (m + 2);
        h1 = vsum[3] * (m + 2);
        h2 = vsum[4] * (m + 2);
        for (x = 1; x < m; x++) {
            g11 += vsum[x * 5];
            g12 += vsum[x * 5 + 1];
            g22 += vsum[x * 5 + 2];
            h1 += vsum[x * 5 + 3];
            h2 += vsum[x * 5 + 4];
        }
        for (x = 0; x < width; x++) {
            g11 += vsum[(x + m) * 5] - vsum[(x - m) * 5 - 5];
            g12 += vsum[(x + m) * 5 + 1] - vsum[(x - m) * 5 - 4];
            g22 += vsum[(x + m) * 5 + 2] - vsum[(x - m) * 5 - 3];
            h1 += vsum[(x + m) * 5 + 3] - vsum[(x - m) * 5 - 2];
            h2 += vsum[(x + m) * 5 + 4] - vsum[(x - m) * 5 - 1];
            double g11_ = g11 * scale, g12_ = g12 * scale, g22_ = g22 * scale, h1_ = h1 * scale, h2_ = h2 * scale;
            double idet = 1. / (g11_ * g22_ - g12_ * g12_ + 1e-3);
            flow[x * 2] = (float)((g11_ * h2_ - g12_ * h1_) * idet);
            flow[x * 2 + 1] = (float)((g22_ * h1_ - g12_ * h2_) * idet);
        }
        y1 = y == height - 1 ? height : y - block_size;
        if (update && (y1 == height || y1 >= y0 + min_update_stripe)) {
            orc_fb_update_matrices(R0, R1, flow_, width, height, M, y0, y1);
            y0 = y1;
        }
    }
    free(vsum_);
}

/* The box blur in the fixed order libtbdk's fb_iter uses (NOT the
 * reference's): per column, the vertical window sum of rows c-m..c+m
 * (clamped) is summed in float from the top at every row c divisible by 4 and
 * slid from the previous row otherwise, V(c) = (V(c-1) + M(c+m)) - M(c-m-1);
 * the same along each row of V for the horizontal window (restart at columns
 * divisible by 4); then the reference's double scale and solve.  The
 * reference's running double sums (orc_fb_update_flow_blur) slide over the
 * whole image instead, with float-rounded row differences. */
void orc_fb_update_flow_blur_direct(const float* R0, const float* R1, float* flow, float* M, int width, int height,
                                    int block_size, int update)
{
    const int m = block_size / 2;
    const double scale = 1. / (block_size * block_size);
    float* V = malloc(sizeof(float) * (size_t)width * 5);
    float* Vp = malloc(sizeof(float) * (size_t)width * 5);
#define MROW(r) (M + (size_t)clampi((r), 0, height - 1) * width * 5)
    for (int y = 0; y < height; y++) {
        for (int x = 0; x < width * 5; x++) {
            float s;
            if (y % 4 == 0) {
                s = MROW(y - m)[x];
                for (int i = -m + 1; i <= m; i++) s += MROW(y + i)[x];
            } else {
                s = (Vp[x] + MROW(y + m)[x]) - MROW(y - m - 1)[x];
            }
            V[x] = s;
        }
        float* f = flow + (size_t)y * width * 2;
        float h[5];
        for (int x = 0; x < width; x++) {
            double g[5];
            for (int c = 0; c < 5; c++) {
#define VCOL(cc) V[clampi((cc), 0, width - 1) * 5 + c]
                if (x % 4 == 0) {
                    h[c] = VCOL(x - m);
                    for (int j = -m + 1; j <= m; j++) h[c] += VCOL(x + j);
                } else {
                    h[c] = (h[c] + VCOL(x + m)) - VCOL(x - m - 1);
                }
#undef VCOL
                g[c] = h[c] * scale;
            }
            const double idet = 1. / (g[0] * g[2] - g[1] * g[1] + 1e-3);
            f[x * 2] = (float)((g[0] * g[4] - g[1] * g[3]) * idet);
            f[x * 2 + 1] = (float)((g[2] * g[3] - g[1] * g[4]) * idet);
        }
        float* t = Vp;
        Vp = V;
        V = t;
    }
#undef MROW
    free(V);
    free(Vp);
    if (update) orc_fb_update_matrices(R0, R1, flow, width, height, M, 0, height);
}

/* FarnebackUpdateFlow_GaussianBlur: float Gaussian (sigma m*0.3) of M with
 * replicated borders, solve, update */
void orc_fb_update_flow_gauss(const float* R0, const float* R1, float* flow, float* M, int width, int height,
                              int block_size, int update)
{
    const int m = block_size / 2;
    double sigma = m * 0.3, s = 1;
    float kernel[64];
    kernel[0] = (float)s;
    for (int i = 1; i <= m; i++) {
        float t = (float)exp(-i * i / (2 * sigma * sigma));
        kernel[i] = t;
        s += t * 2;
    }
    s = 1. / s;
    for (int i = 0; i <= m; i++) kernel[i] = (float)(kernel[i] * s);
    float* vsum_ = malloc(sizeof(float) * (size_t)(width + m * 2 + 2) * 5);
    float* vsum = vsum_ + (m + 1) * 5;
    float* hsum = malloc(sizeof(float) * (size_t)width * 5);
    for (int y = 0; y < height; y++) {
        for (int x = 0; x < width * 5; x++) {
            float s0 = M[(size_t)y * width * 5 + x] * kernel[0];
            for (int i = 1; i <= m; i++)
                s0 += (M[(size_t)clampi(y + i, 0, height - 1) * width * 5 + x] +
                       M[(size_t)clampi(y - i, 0, height - 1) * width * 5 + x]) *
                      kernel[i];
            vsum[x] = s0;
        }
        for (int x = 0; x < m * 5; x++) {
            vsum[-1 - x] = vsum[4 - x];
            vsum[width * 5 + x] = vsum[width * 5 + x - 5];
        }
        for (int x = 0; x < width * 5; x++) {
            float sum = vsum[x] * kernel[0];
            for (int i = 1; i <= m; i++) sum += kernel[i] * (vsum[x - i * 5] + vsum[x + i * 5]);
            hsum[x] = sum;
        }
        float* f = flow + (size_t)y * width * 2;
        for (int x = 0; x < width; x++) {
            double g11 = hsum[x * 5], g12 = hsum[x * 5 + 1], g22 = hsum[x * 5 + 2], h1 = hsum[x * 5 + 3],
                   h2 = hsum[x * 5 + 4];
            double idet = 1. / (g11 * g22 - g12 * g12 + 1e-3);
            f[x * 2] = (float)((g11 * h2 - g12 * h1) * idet);
            f[x * 2 + 1] = (float)((g22 * h1 - g12 * h2) * idet);
        }
    }
    free(vsum_);
    free(hsum);
    if (update) orc_fb_update_matrices(R0, R1, flow, width, height, M, 0, height);
}

static int cv_round(double v) { return (int)lrint(v); }

/* FarnebackOpticalFlowImpl::calc.  prev/next: u8 (pitch bytes); flow0: w*h*2
 * floats, the output, and with FB_USE_INITIAL_FLOW also the input: the coarsest
 * level starts from resize(flow0, INTER_AREA) *= scale (optflowgf.cpp:1151-1160;
 * `*=` is convertTo(flow, -1, scale), a plain copy when scale == 1). */
int orc_fb_calc_mode(const uint8_t* prev, const uint8_t* next, int W, int H, int pitch, float* flow0, int num_levels,
                     double pyr_scale, int win_size, int num_iters, int poly_n, double poly_sigma, int flags,
                     int box_direct)
{
    if (pyr_scale >= 1) return -1;
    const int min_size = 32;
    int k;
    double scale = 1;
    for (k = 0; k < num_levels; k++) {
        scale *= pyr_scale;
        if (W * scale < min_size || H * scale < min_size) break;
    }
    const int levels = k;
    float* fimg = malloc(sizeof(float) * (size_t)W * H);
    float* fblur = malloc(sizeof(float) * (size_t)W * H);
    float* prevFlow = NULL;
    int pw = 0, ph = 0;
    for (k = levels; k >= 0; k--) {
        scale = 1;
        for (int i = 0; i < k; i++) scale *= pyr_scale;
        double sigma = (1. / scale - 1) * 0.5;
        int smooth_sz = cv_round(sigma * 5) | 1;
        if (smooth_sz < 3) smooth_sz = 3;
        const int width = cv_round(W * scale), height = cv_round(H * scale);
        float* flow = k > 0 ? malloc(sizeof(float) * 2 * (size_t)width * height) : flow0;
        if (!prevFlow && (flags & FB_USE_INITIAL_FLOW)) {
            orc_fb_resize_area(flow0, W, H, 2, flow, width, height);
            if (!(fabs(scale - 1) < DBL_EPSILON)) {
                const float a = (float)scale;
                for (size_t i = 0; i < (size_t)width * height * 2; i++) flow[i] = flow[i] * a + 0.0f;
            }
        } else if (!prevFlow) {
            memset(flow, 0, sizeof(float) * 2 * (size_t)width * height);
        } else {
            orc_fb_resize_linear(prevFlow, pw, ph, 2, flow, width, height);
            const float a = (float)(1. / pyr_scale);
            for (size_t i = 0; i < (size_t)width * height * 2; i++) flow[i] = flow[i] * a + 0.0f;
            free(prevFlow);
        }
        float* R[2];
        float* I = malloc(sizeof(float) * (size_t)width * height);
        for (int i = 0; i < 2; i++) {
            const uint8_t* img = i ? next : prev;
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++) fimg[(size_t)y * W + x] = (float)img[(size_t)y * pitch + x];
            orc_fb_gauss_blur(fimg, W, H, fblur, smooth_sz, sigma);
            orc_fb_resize_linear(fblur, W, H, 1, I, width, height);
            R[i] = malloc(sizeof(float) * 5 * (size_t)width * height);
            orc_fb_poly_exp(I, width, height, poly_n, poly_sigma, R[i]);
        }
        free(I);
        float* M = malloc(sizeof(float) * 5 * (size_t)width * height);
        orc_fb_update_matrices(R[0], R[1], flow, width, height, M, 0, height);
        for (int i = 0; i < num_iters; i++) {
            if (flags & FB_GAUSSIAN)
                orc_fb_update_flow_gauss(R[0], R[1], flow, M, width, height, win_size, i < num_iters - 1);
            else if (box_direct)
                orc_fb_update_flow_blur_direct(R[0], R[1], flow, M, width, height, win_size, i < num_iters - 1);
            else
                orc_fb_update_flow_blur(R[0], R[1], flow, M, width, height, win_size, i < num_iters - 1);
        }
        free(M);
        free(R[0]);
        free(R[1]);
        if (k > 0) {
            prevFlow = flow;
            pw = width;
            ph = height;
        }
    }
    free(fimg);
    free(fblur);
    return 0;
}

/* the reference: running-sum box blur */
int orc_fb_calc(const uint8_t* prev, const uint8_t* next, int W, int H, int pitch, float* flow0, int num_levels,
                double pyr_scale, int win_size, int num_iters, int poly_n, double poly_sigma, int flags)
{
    return orc_fb_calc_mode(prev, next, W, H, pitch, flow0, num_levels, pyr_scale, win_size, num_iters, poly_n,
                            poly_sigma, flags, 0);
}
