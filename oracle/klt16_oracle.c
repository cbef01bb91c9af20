/* klt16_oracle.c — CPU restatement of the fp16 and fp32 pixel paths of sparse
 * PyrLK (TEST INFRASTRUCTURE ONLY; loaded by tests/ and bench.py's cpu_baseline).
 * The fp32 path (16U and 32F frames, the other depths cv::cuda::SparsePyrLK-
 * OpticalFlow takes, cudaoptflow/src/pyrlk.cpp:189-205) is the same algorithm
 * with fp32 levels and derivative pairs (no rounding to fp16).
 *
 * The reference has no fp16/fp32 CPU PyrLK (calcSharrDeriv and LKTrackerInvoker
 * take 8-bit levels, video/src/lkpyramid.cpp:57,1272-1276), so this file is the
 * definition the GPU path (opencv_amd/csrc/klt_f16.hip) is checked against:
 * LKTrackerInvoker's algorithm (lkpyramid.cpp:178-695) with its fixed-point
 * steps replaced by fp32 on fp16 pixels, in one fixed operation order:
 *   - pyrDown: pyrDown_<FltCast<float,8>>'s scalar expression order
 *     (imgproc/src/pyramids.cpp:775-777, 856), result rounded to fp16 (RNE);
 *   - derivatives: calcSharrDeriv's formula (lkpyramid.cpp:86-131) in fp32 from
 *     fp16 pixels, rounded to fp16; zero outside the level;
 *   - window values: fmaf chains over the four bilinear taps; per window column
 *     the rows accumulated by fmaf in row order; the column partials summed left
 *     to right.
 * Parity is therefore bit-exact by construction, and "parity unpinned" against
 * the reference itself (there is no reference fp16 path to pin it to); the
 * tests also compare it with the 8-bit path on the same frames. */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "klt_oracle.h"

/* IEEE binary16 <-> binary32, round to nearest even */
float orc16_h2f(uint16_t h)
{
    uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu, x;
    if (e == 0) {
        float f = (float)m * (1.f / 16777216.f); /* subnormal: m * 2^-24, exact */
        memcpy(&x, &f, 4);
        x |= s;
    } else if (e == 31) {
        x = s | 0x7F800000u | (m << 13);
    } else {
        x = s | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

uint16_t orc16_f2h(float f)
{
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint16_t s = (uint16_t)((x >> 16) & 0x8000u);
    const uint32_t a = x & 0x7FFFFFFFu;
    if (a >= 0x7F800000u) return (uint16_t)(s | (a > 0x7F800000u ? 0x7E00u : 0x7C00u));
    if (a < 0x38800000u) /* below the smallest normal half: m * 2^-24 rounded to even */
        return (uint16_t)(s | (uint16_t)nearbyintf(fabsf(f) * 16777216.f));
    uint32_t h = (a - 0x38000000u) >> 13;
    const uint32_t rem = a & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    if (h >= 0x7C00u) h = 0x7C00u;
    return (uint16_t)(s | h);
}

/* one pyrDown level, fp16 in / fp16 out (pitches in elements) */
void orc16_pyr_down(const uint16_t* src, int sw, int sh, int spitch, uint16_t* dst, int dw, int dh, int dpitch)
{
    for (int y = 0; y < dh; ++y)
        for (int x = 0; x < dw; ++x) {
            float r[5];
            for (int j = 0; j < 5; ++j) {
                const uint16_t* row = src + (size_t)orc_reflect101(2 * y + j - 2, sh) * spitch;
                float s0 = orc16_h2f(row[orc_reflect101(2 * x - 2, sw)]);
                float s1 = orc16_h2f(row[orc_reflect101(2 * x - 1, sw)]);
                float s2 = orc16_h2f(row[orc_reflect101(2 * x, sw)]);
                float s3 = orc16_h2f(row[orc_reflect101(2 * x + 1, sw)]);
                float s4 = orc16_h2f(row[orc_reflect101(2 * x + 2, sw)]);
                r[j] = s2 * 6.f + (s1 + s3) * 4.f + s0 + s4;
            }
            dst[(size_t)y * dpitch + x] = orc16_f2h((r[2] * 6.f + (r[1] + r[3]) * 4.f + r[0] + r[4]) * (1.f / 256.f));
        }
}

/* calcSharrDeriv's formula on an fp16 level: dst (h x w x 2) fp16 (Ix, Iy) */
void orc16_scharr(const uint16_t* src, int w, int h, int pitch, uint16_t* dst)
{
    for (int y = 0; y < h; ++y) {
        const uint16_t* r0 = src + (size_t)orc_reflect101(y - 1, h) * pitch;
        const uint16_t* r1 = src + (size_t)y * pitch;
        const uint16_t* r2 = src + (size_t)orc_reflect101(y + 1, h) * pitch;
        for (int x = 0; x < w; ++x) {
            float t0[3], t1[3];
            for (int k = 0; k < 3; ++k) {
                const int c = orc_reflect101(x + k - 1, w);
                t0[k] = (orc16_h2f(r0[c]) + orc16_h2f(r2[c])) * 3.f + orc16_h2f(r1[c]) * 10.f;
                t1[k] = orc16_h2f(r2[c]) - orc16_h2f(r0[c]);
            }
            const float ix = t0[2] - t0[0];
            const float iy = (t1[2] + t1[0]) * 3.f + t1[1] * 10.f;
            dst[((size_t)y * w + x) * 2] = orc16_f2h(ix);
            dst[((size_t)y * w + x) * 2 + 1] = orc16_f2h(iy);
        }
    }
}

/* one pyrDown level of the fp32 pixel path (the same order, no rounding), cn
 * interleaved channels (pitches in elements): every channel filtered on its
 * own, the 5 taps cn elements apart (pyrDown_ on CV_32FC(cn), pyramids.cpp:722-857) */
void orc32_pyr_down_cn(const float* src, int sw, int sh, int spitch, int cn, float* dst, int dw, int dh, int dpitch)
{
    for (int y = 0; y < dh; ++y)
        for (int x = 0; x < dw; ++x)
            for (int c = 0; c < cn; ++c) {
                float r[5];
                for (int j = 0; j < 5; ++j) {
                    const float* row = src + (size_t)orc_reflect101(2 * y + j - 2, sh) * spitch;
                    float s0 = row[orc_reflect101(2 * x - 2, sw) * cn + c];
                    float s1 = row[orc_reflect101(2 * x - 1, sw) * cn + c];
                    float s2 = row[orc_reflect101(2 * x, sw) * cn + c];
                    float s3 = row[orc_reflect101(2 * x + 1, sw) * cn + c];
                    float s4 = row[orc_reflect101(2 * x + 2, sw) * cn + c];
                    r[j] = s2 * 6.f + (s1 + s3) * 4.f + s0 + s4;
                }
                dst[(size_t)y * dpitch + (size_t)x * cn + c] =
                    (r[2] * 6.f + (r[1] + r[3]) * 4.f + r[0] + r[4]) * (1.f / 256.f);
            }
}

void orc32_pyr_down(const float* src, int sw, int sh, int spitch, float* dst, int dw, int dh, int dpitch)
{
    orc32_pyr_down_cn(src, sw, sh, spitch, 1, dst, dw, dh, dpitch);
}

/* calcSharrDeriv's formula on an fp32 level of cn interleaved channels
 * (lkpyramid.cpp:55-144: neighbours cn elements apart, rows / columns
 * reflect-101): dst (h x w x cn x 2) fp32 (Ix, Iy) per element */
void orc32_scharr_cn(const float* src, int w, int h, int pitch, int cn, float* dst)
{
    for (int y = 0; y < h; ++y) {
        const float* r0 = src + (size_t)orc_reflect101(y - 1, h) * pitch;
        const float* r1 = src + (size_t)y * pitch;
        const float* r2 = src + (size_t)orc_reflect101(y + 1, h) * pitch;
        for (int x = 0; x < w; ++x)
            for (int ch = 0; ch < cn; ++ch) {
                float t0[3], t1[3];
                for (int k = 0; k < 3; ++k) {
                    const int c = orc_reflect101(x + k - 1, w) * cn + ch;
                    t0[k] = (r0[c] + r2[c]) * 3.f + r1[c] * 10.f;
                    t1[k] = r2[c] - r0[c];
                }
                const size_t o = (((size_t)y * w + x) * cn + ch) * 2;
                dst[o] = t0[2] - t0[0];
                dst[o + 1] = (t1[2] + t1[0]) * 3.f + t1[1] * 10.f;
            }
    }
}

void orc32_scharr(const float* src, int w, int h, int pitch, float* dst)
{
    orc32_scharr_cn(src, w, h, pitch, 1, dst);
}

typedef struct orc16_level {
    const void* px;     /* h x w (x cn) fp16 (or fp32 with f32) */
    const void* d;      /* h x w (x cn) x 2 fp16 / fp32 (Ix, Iy), or NULL for a J-only level */
    int w, h;
    int f32;            /* the fp32 pixel path: the same algorithm on fp32 levels */
    int cn;             /* interleaved channels (0 or 1: one); fp32 only */
} orc16_level;

typedef struct orc16_pyr {
    int nlevels;
    orc16_level lv[8];
} orc16_pyr;

static inline int lcn(const orc16_level* L) { return L->cn > 1 ? L->cn : 1; }

/* channel ch of pixel (x, y), coordinates reflect-101 (the padded level's frame) */
static inline float px16(const orc16_level* L, int x, int y, int ch)
{
    const int cn = lcn(L);
    const size_t k = ((size_t)orc_reflect101(y, L->h) * L->w + orc_reflect101(x, L->w)) * cn + ch;
    return L->f32 ? ((const float*)L->px)[k] : orc16_h2f(((const uint16_t*)L->px)[k]);
}

/* derivative c (0: Ix, 1: Iy) of channel ch at (x, y); zero outside the level */
static inline float dv16(const orc16_level* L, int x, int y, int ch, int c)
{
    if (x < 0 || y < 0 || x >= L->w || y >= L->h) return 0.f; /* BORDER_CONSTANT 0 frame */
    const size_t k = (((size_t)y * L->w + x) * lcn(L) + ch) * 2 + c;
    return L->f32 ? ((const float*)L->d)[k] : orc16_h2f(((const uint16_t*)L->d)[k]);
}

static inline void weights16(float a, float b, float* w)
{
    w[0] = (1.f - a) * (1.f - b);
    w[1] = a * (1.f - b);
    w[2] = (1.f - a) * b;
    w[3] = a * b;
}

/* fma(w11, v11, fma(w10, v10, fma(w01, v01, fma(w00, v00, c)))) */
static inline float bil(const float* w, float v00, float v01, float v10, float v11, float c)
{
    float t = fmaf(w[0], v00, c);
    t = fmaf(w[1], v01, t);
    t = fmaf(w[2], v10, t);
    return fmaf(w[3], v11, t);
}

typedef struct orc16_job {
    const orc16_pyr *prev, *next;
    const float* prevPts;
    float* nextPts;
    uint8_t* status;
    float* err;
    int32_t* iters;
    const orc_lk_params* prm;
    int maxLevel, maxCount;
    double eps2;
    int begin, end;
} orc16_job;

static void lk16_point(const orc16_job* jb, int i, float* buf)
{
    const int WW = jb->prm->winW, WH = jb->prm->winH, flags = jb->prm->flags;
    /* cn channels: a window row is WW * cn elements (column e = pixel e / cn,
     * channel e % cn), G and b sum over all of them, as the CPU path does
     * (lkpyramid.cpp:233-252, 268-420: winSize.width * cn per row) */
    const int cn = lcn(&jb->prev->lv[0]), WE = WW * cn;
    float* iv = buf;
    float* gx = iv + WE * WH;
    float* gy = gx + WE * WH;
    float* col = gy + WE * WH;
    const float FLT_SCALE = 1.f / (1 << 20);
    const float halfx = (WW - 1) * 0.5f, halfy = (WH - 1) * 0.5f;
    const float p0x = jb->prevPts[2 * i], p0y = jb->prevPts[2 * i + 1];
    float outx = 0.f, outy = 0.f;
    if (flags & ORC_OPTFLOW_USE_INITIAL_FLOW) {
        outx = jb->nextPts[2 * i];
        outy = jb->nextPts[2 * i + 1];
    }
    int status = 1, nit = 0;
    float errv = 0.f;
    for (int level = jb->maxLevel; level >= 0; --level) {
        const orc16_level* I = &jb->prev->lv[level];
        const orc16_level* J = &jb->next->lv[level];
        const float sc = (float)(1. / (1 << level));
        float prevx = p0x * sc, prevy = p0y * sc, nextx, nexty;
        if (level == jb->maxLevel) {
            if (flags & ORC_OPTFLOW_USE_INITIAL_FLOW) {
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
        if (ipx < -WW || ipx >= I->w || ipy < -WH || ipy >= I->h) {
            if (level == 0) {
                status = 0;
                errv = 0.f;
            }
            continue;
        }
        float w[4];
        weights16(prevx - ipx, prevy - ipy, w);
        float s[3];
        for (int v = 0; v < 3; ++v) {
            for (int e = 0; e < WE; ++e) {
                const int x = e / cn, ch = e - x * cn;
                float acc = 0.f;
                for (int r = 0; r < WH; ++r) {
                    const int X = ipx + x, Y = ipy + r;
                    const size_t k = (size_t)r * WE + e;
                    if (v == 0) {
                        iv[k] = bil(w, px16(I, X, Y, ch), px16(I, X + 1, Y, ch), px16(I, X, Y + 1, ch),
                                    px16(I, X + 1, Y + 1, ch), 0.f);
                        gx[k] = bil(w, dv16(I, X, Y, ch, 0), dv16(I, X + 1, Y, ch, 0), dv16(I, X, Y + 1, ch, 0),
                                    dv16(I, X + 1, Y + 1, ch, 0), 0.f);
                        gy[k] = bil(w, dv16(I, X, Y, ch, 1), dv16(I, X + 1, Y, ch, 1), dv16(I, X, Y + 1, ch, 1),
                                    dv16(I, X + 1, Y + 1, ch, 1), 0.f);
                    }
                    const float a = v == 2 ? gy[k] : gx[k], b = v == 0 ? gx[k] : gy[k];
                    acc = fmaf(a, b, acc);
                }
                col[e] = acc;
            }
            float t = col[0];
            for (int e = 1; e < WE; ++e) t += col[e];
            s[v] = t;
        }
        const float A11 = s[0] * FLT_SCALE, A12 = s[1] * FLT_SCALE, A22 = s[2] * FLT_SCALE;
        float D = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * WW * WH);
        if (flags & ORC_OPTFLOW_LK_GET_MIN_EIGENVALS) errv = minEig;
        if (minEig < jb->prm->minEigThreshold || D < 1.19209290e-07F) {
            if (level == 0) status = 0;
            continue;
        }
        D = 1.f / D;
        nextx -= halfx;
        nexty -= halfy;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < jb->maxCount; ++j) {
            const int inx = (int)floorf(nextx), iny = (int)floorf(nexty);
            if (inx < -WW || inx >= J->w || iny < -WH || iny >= J->h) {
                if (level == 0) status = 0;
                break;
            }
            ++nit;
            weights16(nextx - inx, nexty - iny, w);
            float b[2];
            for (int v = 0; v < 2; ++v) {
                for (int e = 0; e < WE; ++e) {
                    const int x = e / cn, ch = e - x * cn;
                    float acc = 0.f;
                    for (int r = 0; r < WH; ++r) {
                        const int X = inx + x, Y = iny + r;
                        const size_t k = (size_t)r * WE + e;
                        const float d = bil(w, px16(J, X, Y, ch), px16(J, X + 1, Y, ch), px16(J, X, Y + 1, ch),
                                            px16(J, X + 1, Y + 1, ch), -iv[k]);
                        acc = fmaf(d, v == 0 ? gx[k] : gy[k], acc);
                    }
                    col[e] = acc;
                }
                float t = col[0];
                for (int e = 1; e < WE; ++e) t += col[e];
                b[v] = t * (32.f * FLT_SCALE);
            }
            const float ddx = (A12 * b[1] - A22 * b[0]) * D;
            const float ddy = (A12 * b[0] - A11 * b[1]) * D;
            nextx += ddx;
            nexty += ddy;
            outx = nextx + halfx;
            outy = nexty + halfy;
            if ((double)ddx * ddx + (double)ddy * ddy <= jb->eps2) break;
            if (j > 0 && (double)fabsf(ddx + pdx) < 0.01 && (double)fabsf(ddy + pdy) < 0.01) {
                outx -= ddx * 0.5f;
                outy -= ddy * 0.5f;
                break;
            }
            pdx = ddx;
            pdy = ddy;
        }
        if (level == 0 && jb->err && (flags & ORC_OPTFLOW_LK_GET_MIN_EIGENVALS) == 0 && status) {
            const float npx = outx - halfx, npy = outy - halfy;
            const int inx = (int)floorf(npx), iny = (int)floorf(npy);
            if (inx < -WW || inx >= J->w || iny < -WH || iny >= J->h) {
                status = 0;
            } else {
                weights16(npx - inx, npy - iny, w);
                for (int e = 0; e < WE; ++e) {
                    const int x = e / cn, ch = e - x * cn;
                    float ev = 0.f;
                    for (int r = 0; r < WH; ++r) {
                        const int X = inx + x, Y = iny + r;
                        ev += fabsf(bil(w, px16(J, X, Y, ch), px16(J, X + 1, Y, ch), px16(J, X, Y + 1, ch),
                                        px16(J, X + 1, Y + 1, ch), -iv[(size_t)r * WE + e]));
                    }
                    col[e] = ev;
                }
                float t = col[0];
                for (int e = 1; e < WE; ++e) t += col[e];
                /* lkpyramid.cpp:690: errval / (32 * winSize.width * cn * winSize.height) */
                errv = (t * 32.f) * (1.f / (float)(32 * WW * cn * WH));
            }
        }
    }
    jb->nextPts[2 * i] = outx;
    jb->nextPts[2 * i + 1] = outy;
    jb->status[i] = (uint8_t)status;
    if (jb->err) jb->err[i] = errv;
    if (jb->iters) jb->iters[i] = nit;
}

static void* lk16_worker(void* arg)
{
    const orc16_job* jb = (const orc16_job*)arg;
    const int cn = lcn(&jb->prev->lv[0]);
    const int area = jb->prm->winW * cn * jb->prm->winH;
    float* buf = (float*)malloc(sizeof(float) * ((size_t)area * 3 + (size_t)jb->prm->winW * cn));
    for (int i = jb->begin; i < jb->end; ++i) lk16_point(jb, i, buf);
    free(buf);
    return NULL;
}

/* sparse LK on two fp16 pyramids (levels px + derivative planes d of prev) */
int orc16_lk(const orc16_pyr* prev, const orc16_pyr* next, const float* prevPts, float* nextPts, uint8_t* status,
             float* err, int npoints, const orc_lk_params* prm, int32_t* iters)
{
    if (npoints <= 0) return 0;
    if (prm->winW < 3 || prm->winH < 3 || prm->winW > 64 || prm->winH > 64) return -1;
    int maxLevel = prm->maxLevel;
    if (prev->nlevels - 1 < maxLevel) maxLevel = prev->nlevels - 1;
    if (next->nlevels - 1 < maxLevel) maxLevel = next->nlevels - 1;
    for (int l = 0; l <= maxLevel; ++l)
        if (prev->lv[l].w != next->lv[l].w || prev->lv[l].h != next->lv[l].h || !prev->lv[l].d ||
            prev->lv[l].f32 != next->lv[l].f32 || lcn(&prev->lv[l]) != lcn(&next->lv[l]) ||
            (lcn(&prev->lv[l]) > 1 && !prev->lv[l].f32))
            return -2;
    const double eps = prm->epsilon < 0. ? 0. : (prm->epsilon > 10. ? 10. : prm->epsilon);
    int nth = prm->nthreads > 0 ? prm->nthreads : 1;
    if (nth > npoints) nth = npoints;
    orc16_job* jobs = (orc16_job*)malloc(sizeof(orc16_job) * (size_t)nth);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nth);
    for (int t = 0; t < nth; ++t) {
        orc16_job* jb = &jobs[t];
        jb->prev = prev;
        jb->next = next;
        jb->prevPts = prevPts;
        jb->nextPts = nextPts;
        jb->status = status;
        jb->err = err;
        jb->iters = iters;
        jb->prm = prm;
        jb->maxLevel = maxLevel;
        jb->maxCount = prm->maxCount < 0 ? 0 : (prm->maxCount > 100 ? 100 : prm->maxCount);
        jb->eps2 = eps * eps;
        jb->begin = (int)((int64_t)npoints * t / nth);
        jb->end = (int)((int64_t)npoints * (t + 1) / nth);
    }
    if (nth == 1) {
        lk16_worker(&jobs[0]);
    } else {
        for (int t = 0; t < nth; ++t) pthread_create(&th[t], NULL, lk16_worker, &jobs[t]);
        for (int t = 0; t < nth; ++t) pthread_join(th[t], NULL);
    }
    free(jobs);
    free(th);
    return 0;
}
