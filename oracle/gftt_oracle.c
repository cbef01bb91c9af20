/*
 * gftt_oracle.c — CPU restatement of cv::goodFeaturesToTrack (min-eigenvalue
 * variant) for one isolated u8 image.  TEST INFRASTRUCTURE ONLY.
 *
 * Float evaluation order (compiled with -ffp-contract=off) follows the
 * reference's non-FMA code paths:
 *   Sobel ksize 3, CV_32F, scale 1/(4*blockSize*255)  (corner.cpp:248-263, deriv.cpp:414-465)
 *     Dx: row [-1 0 1] (exact), column [k 2k k]: (S0+S2)*k + (S1*2k + 0)
 *         (filter.simd.hpp:2025-2027, SymmColumnSmallVec_32f)
 *     Dy: row [k 2k k]: ((k*S0) + 2k*S1) + k*S2 (RowFilter, filter.simd.hpp:2357-2366),
 *         column [-1 0 1]: (S2 - S0) + 0          (filter.simd.hpp:2032-2037)
 *   cov = (Dx*Dx, Dx*Dy, Dy*Dy)                         (corner.cpp:283-311)
 *   boxFilter 3x3 unnormalised, sums in double: RowSum ksize 3
 *     ((S0 + S1) + S2) (box_filter.simd.hpp:84-89) and the running ColumnSum
 *     (box_filter.simd.hpp:176-273) started at the top border row.
 *   minEig = (a + c) - sqrt((a - c)^2 + b^2), a, c halved     (corner.cpp:52-101)
 *   borders: BORDER_REFLECT_101 on the isolated image.
 * Selection: max (no mask), threshold-to-zero at (float)(max*q), 3x3 dilate,
 * interior local maxima, sort by value desc then address desc
 * (featureselect.cpp:56-64), greedy min-distance grid (:421-503).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "klt_oracle.h"

void orc_min_eig(const uint8_t* img, int w, int h, int pitch, float* eig)
{
    const double scale = 1.0 / ((double)(1 << 2) * 3 * 255.0);
    const float k = (float)(1.0 * scale), k2 = (float)(2.0 * scale);
    /* Sobel with reflect-101 borders */
    float* dx = (float*)malloc(sizeof(float) * (size_t)w * h);
    float* dy = (float*)malloc(sizeof(float) * (size_t)w * h);
    float* rx = (float*)malloc(sizeof(float) * (size_t)w * 3);
    float* ry = (float*)malloc(sizeof(float) * (size_t)w * 3);
    for (int y = 0; y < h; ++y) {
        for (int j = 0; j < 3; ++j) {
            const uint8_t* s = img + (size_t)orc_reflect101(y + j - 1, h) * pitch;
            for (int x = 0; x < w; ++x) {
                const float s0 = s[orc_reflect101(x - 1, w)], s1 = s[x], s2 = s[orc_reflect101(x + 1, w)];
                float t = -1.f * s0;
                t = t + 0.f * s1;
                t = t + 1.f * s2;
                rx[j * w + x] = t;
                float u = k * s0;
                u = u + k2 * s1;
                u = u + k * s2;
                ry[j * w + x] = u;
            }
        }
        for (int x = 0; x < w; ++x) {
            dx[(size_t)y * w + x] = (rx[x] + rx[2 * w + x]) * k + (rx[w + x] * k2 + 0.f);
            dy[(size_t)y * w + x] = (ry[2 * w + x] - ry[x]) + 0.f;
        }
    }
    /* cov */
    float* cov = (float*)malloc(sizeof(float) * 3 * (size_t)w * h);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        cov[3 * i] = dx[i] * dx[i];
        cov[3 * i + 1] = dx[i] * dy[i];
        cov[3 * i + 2] = dy[i] * dy[i];
    }
    /* boxFilter: row sums (double) of every (bordered) row, running column sums */
    double* rs = (double*)malloc(sizeof(double) * 3 * (size_t)w * (h + 2));
    for (int yy = -1; yy <= h; ++yy) {
        const float* c = cov + (size_t)orc_reflect101(yy, h) * w * 3;
        double* d = rs + (size_t)(yy + 1) * w * 3;
        for (int x = 0; x < w; ++x) {
            const int xl = orc_reflect101(x - 1, w), xr = orc_reflect101(x + 1, w);
            for (int ch = 0; ch < 3; ++ch)
                d[3 * x + ch] = (double)c[3 * xl + ch] + (double)c[3 * x + ch] + (double)c[3 * xr + ch];
        }
    }
    double* sum = (double*)calloc(3 * (size_t)w, sizeof(double));
    for (int i = 0; i < 3 * w; ++i) sum[i] = 0.0 + rs[i];          /* row -1 */
    for (int i = 0; i < 3 * w; ++i) sum[i] = sum[i] + rs[3 * w + i]; /* row 0 */
    for (int y = 0; y < h; ++y) {
        const double* sp = rs + (size_t)(y + 2) * w * 3;  /* entering row y+1 */
        const double* sm = rs + (size_t)y * w * 3;        /* leaving row y-1  */
        for (int x = 0; x < w; ++x) {
            float box[3];
            for (int ch = 0; ch < 3; ++ch) {
                const int i = 3 * x + ch;
                const double s0 = sum[i] + sp[i];
                box[ch] = (float)s0;
                sum[i] = s0 - sm[i];
            }
            const float a = box[0] * 0.5f, b = box[1], c = box[2] * 0.5f;
            const float t = a - c;
            eig[(size_t)y * w + x] = (a + c) - sqrtf(b * b + t * t);
        }
    }
    free(dx); free(dy); free(rx); free(ry); free(cov); free(rs); free(sum);
}

/* cornerMinEigenVal / cornerHarris for any blockSize (ksize 3, u8 source,
 * BORDER_REFLECT_101), restating cornerEigenValsVecs (corner.cpp:237-326):
 *   scale = 1 / (4 * blockSize * 255); the ksize-3 Sobel rows as above
 *   boxFilter(cov, blockSize, anchor blockSize/2, unnormalised, CV_64F sums):
 *     RowSum (box_filter.simd.hpp:64-170, cn = 3): ksize 3 and 5 add the taps
 *       left to right; other sizes run s = 0 + taps, then s += (S[i+k] - S[i])
 *       along the bordered row
 *     ColumnSum<double,float> (:175-273): SUM = 0 + the first ksize-1 rows,
 *       then per row s = SUM + Sp; out = (float)s; SUM = s - Sm
 *   calcMinEigenVal (:52-101): (a + c) - sqrt(t*t + b*b), a, c halved (all
 *     three code paths round alike)
 *   calcHarris (:104-152) over the continuous (flattened) map, index j: the
 *     AVX lines (corner.avx.cpp:144-160: acbb - k*(ac*ac), k as float) for
 *     j < N & ~7, one SSE2 block ((acbb) - (k*ac)*ac) if 4 more remain, the
 *     scalar double expression for the rest: the code an AVX x86-64 host runs. */
void orc_corner_response(const uint8_t* img, int w, int h, int pitch, int block, int harris, double hk, float* out)
{
    const double scale = 1.0 / ((double)(1 << 2) * block * 255.0);
    const float k = (float)(1.0 * scale), k2 = (float)(2.0 * scale);
    const size_t n = (size_t)w * h;
    float* cov = (float*)malloc(sizeof(float) * 3 * (n ? n : 1));
    for (int y = 0; y < h; ++y) {
        const uint8_t* r0 = img + (size_t)orc_reflect101(y - 1, h) * pitch;
        const uint8_t* r1 = img + (size_t)y * pitch;
        const uint8_t* r2 = img + (size_t)orc_reflect101(y + 1, h) * pitch;
        for (int x = 0; x < w; ++x) {
            const int xl = orc_reflect101(x - 1, w), xr = orc_reflect101(x + 1, w);
            float rx[3], ry[3];
            const uint8_t* rr[3] = {r0, r1, r2};
            for (int j = 0; j < 3; ++j) {
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
            float* c = cov + 3 * ((size_t)y * w + x);
            c[0] = dx * dx;
            c[1] = dx * dy;
            c[2] = dy * dy;
        }
    }
    const int anc = block / 2;
    double* rs = (double*)malloc(sizeof(double) * 3 * (n ? n : 1));
    for (int y = 0; y < h; ++y) {
        const float* c = cov + 3 * (size_t)y * w;
        double* d = rs + 3 * (size_t)y * w;
        for (int ch = 0; ch < 3; ++ch) {
#define TAP(i) ((double)c[3 * orc_reflect101((i) - anc, w) + ch]) /* bordered-row element i */
            if (block == 3 || block == 5) {
                for (int x = 0; x < w; ++x) {
                    double s = TAP(x) + TAP(x + 1);
                    for (int t = 2; t < block; ++t) s = s + TAP(x + t);
                    d[3 * x + ch] = s;
                }
            } else {
                double s = 0;
                for (int t = 0; t < block; ++t) s += TAP(t);
                d[ch] = s;
                for (int x = 0; x + 1 < w; ++x) {
                    s += TAP(x + block) - TAP(x);
                    d[3 * (x + 1) + ch] = s;
                }
            }
#undef TAP
        }
    }
    double* sum = (double*)malloc(sizeof(double) * 3 * (size_t)(w ? w : 1));
    for (int i = 0; i < 3 * w; ++i) sum[i] = 0.0;
    for (int r = 0; r < block - 1; ++r) {
        const double* sp = rs + 3 * (size_t)orc_reflect101(r - anc, h) * w;
        for (int i = 0; i < 3 * w; ++i) sum[i] += sp[i];
    }
    const size_t avx_end = n & ~(size_t)7, sse_end = avx_end + (n - avx_end >= 4 ? 4 : 0);
    const float kf = (float)hk;
    for (int y = 0; y < h; ++y) {
        const double* sp = rs + 3 * (size_t)orc_reflect101(y - anc + block - 1, h) * w; /* entering */
        const double* sm = rs + 3 * (size_t)orc_reflect101(y - anc, h) * w;             /* leaving */
        for (int x = 0; x < w; ++x) {
            float box[3];
            for (int ch = 0; ch < 3; ++ch) {
                const int i = 3 * x + ch;
                const double s0 = sum[i] + sp[i];
                box[ch] = (float)s0;
                sum[i] = s0 - sm[i];
            }
            const size_t j = (size_t)y * w + x;
            if (!harris) {
                const float a = box[0] * 0.5f, b = box[1], c = box[2] * 0.5f;
                const float t = a - c;
                out[j] = (a + c) - sqrtf(b * b + t * t);
            } else {
                const float a = box[0], b = box[1], c = box[2];
                const float acbb = a * c - b * b, ac = a + c;
                if (j < avx_end) out[j] = acbb - kf * (ac * ac);
                else if (j < sse_end) out[j] = acbb - (kf * ac) * ac;
                else out[j] = (float)((double)acbb - hk * (double)ac * (double)ac);
            }
        }
    }
    free(cov); free(rs); free(sum);
}

typedef struct { float v; int idx; } orc_cand;

static int orc_cand_cmp(const void* pa, const void* pb)
{
    const orc_cand* a = (const orc_cand*)pa;
    const orc_cand* b = (const orc_cand*)pb;
    if (a->v > b->v) return -1;
    if (a->v < b->v) return 1;
    return (a->idx > b->idx) ? -1 : (a->idx < b->idx ? 1 : 0);  /* higher address first */
}

/* goodFeaturesToTrack (featureselect.cpp:361-516) with blockSize and the
 * Harris response (useHarrisDetector, harrisK) */
int orc_gftt_ex(const uint8_t* img, int w, int h, int pitch, int maxCorners, double qualityLevel,
                double minDistance, int block, int harris, double hk, float* corners)
{
    if (w <= 0 || h <= 0) return 0;
    float* eig = (float*)malloc(sizeof(float) * (size_t)w * h);
    if (block == 3 && !harris) orc_min_eig(img, w, h, pitch, eig);
    else orc_corner_response(img, w, h, pitch, block, harris, hk, eig);
    double maxVal = 0;
    int first = 1;
    for (size_t i = 0; i < (size_t)w * h; ++i)
        if (first || eig[i] > maxVal) { maxVal = eig[i]; first = 0; }
    const float thr = (float)(maxVal * qualityLevel);
    for (size_t i = 0; i < (size_t)w * h; ++i)
        if (!(eig[i] > thr)) eig[i] = 0.f;  /* THRESH_TOZERO */
    orc_cand* cand = (orc_cand*)malloc(sizeof(orc_cand) * (size_t)w * h);
    int total = 0;
    for (int y = 1; y < h - 1; ++y)
        for (int x = 1; x < w - 1; ++x) {
            const float v = eig[(size_t)y * w + x];
            if (v == 0.f) continue;
            float m = v;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    const float q = eig[(size_t)(y + dy) * w + x + dx];
                    if (q > m) m = q;
                }
            if (v == m) { cand[total].v = v; cand[total].idx = y * w + x; total++; }
        }
    qsort(cand, (size_t)total, sizeof(orc_cand), orc_cand_cmp);
    int n = 0;
    if (minDistance >= 1) {
        const int cell = (int)lrint(minDistance);
        const int gw = (w + cell - 1) / cell, gh = (h + cell - 1) / cell;
        int* gcount = (int*)calloc((size_t)gw * gh, sizeof(int));
        int* gfirst = (int*)malloc(sizeof(int) * (size_t)gw * gh);
        int* next = (int*)malloc(sizeof(int) * (size_t)(total > 0 ? total : 1));
        float* px = (float*)malloc(sizeof(float) * (size_t)(total > 0 ? total : 1));
        float* py = (float*)malloc(sizeof(float) * (size_t)(total > 0 ? total : 1));
        const double md2 = minDistance * minDistance;
        int nacc = 0;
        for (int i = 0; i < total; ++i) {
            const int y = cand[i].idx / w, x = cand[i].idx % w;
            const int xc = x / cell, yc = y / cell;
            int x1 = xc - 1 < 0 ? 0 : xc - 1, y1 = yc - 1 < 0 ? 0 : yc - 1;
            int x2 = xc + 1 > gw - 1 ? gw - 1 : xc + 1, y2 = yc + 1 > gh - 1 ? gh - 1 : yc + 1;
            int good = 1;
            for (int yy = y1; yy <= y2 && good; ++yy)
                for (int xx = x1; xx <= x2 && good; ++xx) {
                    int g = yy * gw + xx;
                    int it = gcount[g] ? gfirst[g] : -1;
                    while (it >= 0) {
                        const float ddx = (float)x - px[it], ddy = (float)y - py[it];
                        if ((double)(ddx * ddx + ddy * ddy) < md2) { good = 0; break; }
                        it = next[it];
                    }
                }
            if (good) {
                const int g = yc * gw + xc;
                px[nacc] = (float)x; py[nacc] = (float)y;
                next[nacc] = gcount[g] ? gfirst[g] : -1;  /* order within a cell does not matter */
                gfirst[g] = nacc; gcount[g]++;
                nacc++;
                corners[2 * n] = (float)x; corners[2 * n + 1] = (float)y;
                n++;
                if (maxCorners > 0 && n == maxCorners) break;
            }
        }
        free(gcount); free(gfirst); free(next); free(px); free(py);
    } else {
        for (int i = 0; i < total; ++i) {
            corners[2 * n] = (float)(cand[i].idx % w);
            corners[2 * n + 1] = (float)(cand[i].idx / w);
            n++;
            if (maxCorners > 0 && n == maxCorners) break;
        }
    }
    free(eig); free(cand);
    return n;
}

int orc_gftt(const uint8_t* img, int w, int h, int pitch, int maxCorners, double qualityLevel,
             double minDistance, float* corners)
{
    return orc_gftt_ex(img, w, h, pitch, maxCorners, qualityLevel, minDistance, 3, 0, 0.04, corners);
}
