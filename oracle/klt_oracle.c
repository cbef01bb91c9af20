/*
 * klt_oracle.c — CPU restatement of the reference KLT path (TEST INFRASTRUCTURE).
 * See klt_oracle.h for scope and parity status.  Compiled with
 * -ffp-contract=off so every float/double expression rounds exactly as the
 * reference's SSE2 build does (no FMA contraction).
 */
#include "klt_oracle.h"
#include "../opencv_amd/csrc/synth_spec.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* CV_DESCALE (lkpyramid.cpp:51) */
#define ORC_DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

double orc_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* cv::borderInterpolate for BORDER_REFLECT_101
 * (modules/core/src/copy.cpp borderInterpolate; BORDER_DEFAULT == REFLECT_101) */
int orc_reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

/* cvRound(float) == round-half-even (core/include/opencv2/core/fast_math.hpp:101-106) */
static int orc_round(float v)
{
    return (int)lrintf(v);
}

static int orc_floor(float v)
{
    return (int)floorf(v);
}

/* ------------------------------------------------------------------ pyramid */

/* pyrDown_<FixPtCast<uchar,8>> (imgproc/src/pyramids.cpp:722-857): 5x5
 * [1 4 6 4 1]^2 in integers, (s + 128) >> 8, reflect-101 on the isolated
 * source plane, dst size given by the caller ((w+1)/2, (h+1)/2). */
void orc_pyr_down_cn(const uint8_t* src, int sw, int sh, int spitch, int cn,
                     uint8_t* dst, int dw, int dh, int dpitch)
{
    /* element x*cn + c of a row: taps of channel c at the reflected pixel columns
     * (pyramids.cpp:746-790 builds tabL / tabR the same way per channel) */
    const int dwn = dw * cn;
    int* row = (int*)malloc(sizeof(int) * 5 * (size_t)dwn);
    int* tab = (int*)malloc(sizeof(int) * 5 * (size_t)dwn);
    for (int x = 0; x < dw; ++x)
        for (int c = 0; c < cn; ++c)
            for (int i = 0; i < 5; ++i) tab[(x * cn + c) * 5 + i] = orc_reflect101(2 * x + i - 2, sw) * cn + c;
    for (int y = 0; y < dh; ++y) {
        for (int j = 0; j < 5; ++j) {
            const uint8_t* s = src + (size_t)orc_reflect101(2 * y + j - 2, sh) * spitch;
            int* r = row + j * dwn;
            for (int x = 0; x < dwn; ++x) {
                const int* t = tab + x * 5;
                r[x] = s[t[2]] * 6 + (s[t[1]] + s[t[3]]) * 4 + s[t[0]] + s[t[4]];
            }
        }
        uint8_t* d = dst + (size_t)y * dpitch;
        for (int x = 0; x < dwn; ++x) {
            int v = row[2 * dwn + x] * 6 + (row[dwn + x] + row[3 * dwn + x]) * 4 + row[x] + row[4 * dwn + x];
            d[x] = (uint8_t)((v + 128) >> 8);
        }
    }
    free(row);
    free(tab);
}

void orc_pyr_down(const uint8_t* src, int sw, int sh, int spitch,
                  uint8_t* dst, int dw, int dh, int dpitch)
{
    orc_pyr_down_cn(src, sw, sh, spitch, 1, dst, dw, dh, dpitch);
}

/* copyMakeBorder(..., BORDER_REFLECT_101) of the interior into the border */
static void orc_fill_border(orc_plane* p)
{
    const int cn = p->cn > 0 ? p->cn : 1;
    for (int y = -p->pad; y < p->h + p->pad; ++y) {
        int ry = orc_reflect101(y, p->h);
        uint8_t* drow = p->data + (size_t)(y + p->pad) * p->pitch + (size_t)p->pad * cn;
        const uint8_t* srow = p->data + (size_t)(ry + p->pad) * p->pitch + (size_t)p->pad * cn;
        for (int x = -p->pad; x < p->w + p->pad; ++x) {
            if (y >= 0 && y < p->h && x >= 0 && x < p->w) continue;
            const int rx = orc_reflect101(x, p->w);
            for (int c = 0; c < cn; ++c) drow[x * cn + c] = srow[rx * cn + c];
        }
    }
}

static void orc_plane_alloc(orc_plane* p, int w, int h, int pad, int cn)
{
    p->w = w;
    p->h = h;
    p->pad = pad;
    p->cn = cn;
    p->pitch = (w + 2 * pad) * cn;
    p->data = (uint8_t*)calloc((size_t)p->pitch * (h + 2 * pad), 1);
}

/* cv::buildOpticalFlowPyramid(withDerivatives=false, pyrBorder=REFLECT_101)
 * (video/src/lkpyramid.cpp:697-793) */
int orc_build_pyramid(const uint8_t* img, int w, int h, int pitch,
                      int winW, int winH, int maxLevel, int pad, orc_pyr* pyr)
{
    return orc_build_pyramid_cn(img, w, h, pitch, 1, winW, winH, maxLevel, pad, pyr);
}

int orc_build_pyramid_cn(const uint8_t* img, int w, int h, int pitch, int cn,
                         int winW, int winH, int maxLevel, int pad, orc_pyr* pyr)
{
    if (maxLevel >= ORC_MAX_LEVELS) maxLevel = ORC_MAX_LEVELS - 1;
    memset(pyr, 0, sizeof(*pyr));
    orc_plane_alloc(&pyr->lv[0], w, h, pad, cn);
    for (int y = 0; y < h; ++y)
        memcpy(pyr->lv[0].data + (size_t)(y + pad) * pyr->lv[0].pitch + (size_t)pad * cn, img + (size_t)y * pitch,
               (size_t)w * cn);
    orc_fill_border(&pyr->lv[0]);
    int sw = w, sh = h;
    for (int level = 0; level <= maxLevel; ++level) {
        if (level != 0) {
            orc_plane* s = &pyr->lv[level - 1];
            orc_plane* d = &pyr->lv[level];
            orc_plane_alloc(d, sw, sh, pad, cn);
            orc_pyr_down_cn(s->data + (size_t)s->pad * s->pitch + (size_t)s->pad * cn, s->w, s->h, s->pitch, cn,
                            d->data + (size_t)d->pad * d->pitch + (size_t)d->pad * cn, d->w, d->h, d->pitch);
            orc_fill_border(d);
        }
        pyr->nlevels = level + 1;
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= winW || sh <= winH) return pyr->nlevels;
    }
    return pyr->nlevels;
}

void orc_free_pyramid(orc_pyr* pyr)
{
    for (int i = 0; i < ORC_MAX_LEVELS; ++i) free(pyr->lv[i].data);
    memset(pyr, 0, sizeof(*pyr));
}

/* ------------------------------------------------------------------ Scharr */

/* calcSharrDeriv (video/src/lkpyramid.cpp:55-144) */
void orc_scharr(const uint8_t* src, int w, int h, int pitch, int16_t* dst, int dstride)
{
    orc_scharr_cn(src, w, h, pitch, 1, dst, dstride);
}

/* rows of colsn = w*cn elements, neighbours cn elements apart; the column
 * border copies element x0 = cn / x1 = (w-2)*cn per channel (lkpyramid.cpp:111-116) */
void orc_scharr_cn(const uint8_t* src, int w, int h, int pitch, int cn, int16_t* dst, int dstride)
{
    const int wn = w * cn;
    int16_t* t0 = (int16_t*)malloc(sizeof(int16_t) * (size_t)(wn + 2 * cn)) + cn;
    int16_t* t1 = (int16_t*)malloc(sizeof(int16_t) * (size_t)(wn + 2 * cn)) + cn;
    for (int y = 0; y < h; ++y) {
        const uint8_t* s0 = src + (size_t)(y > 0 ? y - 1 : (h > 1 ? 1 : 0)) * pitch;
        const uint8_t* s1 = src + (size_t)y * pitch;
        const uint8_t* s2 = src + (size_t)(y < h - 1 ? y + 1 : (h > 1 ? h - 2 : 0)) * pitch;
        for (int x = 0; x < wn; ++x) {
            t0[x] = (int16_t)((s0[x] + s2[x]) * 3 + s1[x] * 10);
            t1[x] = (int16_t)(s2[x] - s0[x]);
        }
        int x0 = (w > 1 ? 1 : 0) * cn, x1 = (w > 1 ? w - 2 : 0) * cn;
        for (int k = 0; k < cn; ++k) {
            t0[-cn + k] = t0[x0 + k]; t0[wn + k] = t0[x1 + k];
            t1[-cn + k] = t1[x0 + k]; t1[wn + k] = t1[x1 + k];
        }
        int16_t* d = dst + (size_t)y * dstride;
        for (int x = 0; x < wn; ++x) {
            d[2 * x] = (int16_t)(t0[x + cn] - t0[x - cn]);
            d[2 * x + 1] = (int16_t)((t1[x + cn] + t1[x - cn]) * 3 + t1[x] * 10);
        }
    }
    free(t0 - cn);
    free(t1 - cn);
}

/* --------------------------------------------------------------------- LK */

typedef struct orc_level_ctx {
    const orc_plane* I;
    const orc_plane* J;
    const int16_t* dI;   /* derivative plane incl. zero border of dpad */
    int dpad, dstride;   /* dstride in int16 elements */
} orc_level_ctx;

typedef struct orc_job {
    const orc_level_ctx* lv;
    const float* prevPts;
    float* nextPts;
    uint8_t* status;
    float* err;
    int32_t* iters;
    float* gate;         /* optional: per point, the smallest relative margin of any gate evaluated */
    const orc_lk_params* prm;
    int level, maxLevel, maxCount;
    double eps2;
    int begin, end;
} orc_job;

/* Diagnostics for the tolerance clause of SURVEY.md §8(c) ("any status
 * disagreement must lie within 1e-3 (relative) of the minEig/bounds
 * thresholds"): how close a gate's operand came to its threshold, relative to
 * the threshold.  The bounds gates floor(x) < -win / floor(x) >= cols are
 * x < -win / x >= cols on the float coordinate. */
static void orc_gate_note(const orc_job* jb, int ptidx, float m)
{
    if (jb->gate && m < jb->gate[ptidx]) jb->gate[ptidx] = m;
}

static void orc_gate_bounds(const orc_job* jb, int ptidx, float x, float y, int winW, int winH, int cols, int rows)
{
    if (!jb->gate) return;
    float m = fabsf(x + (float)winW) / (float)winW;
    float t = fabsf(x - (float)cols) / (float)cols;
    if (t < m) m = t;
    t = fabsf(y + (float)winH) / (float)winH;
    if (t < m) m = t;
    t = fabsf(y - (float)rows) / (float)rows;
    if (t < m) m = t;
    orc_gate_note(jb, ptidx, m);
}

static const uint8_t* orc_px(const orc_plane* p, int x, int y, int cn)
{
    return p->data + (size_t)(y + p->pad) * p->pitch + (size_t)(x + p->pad) * cn;
}

/* LKTrackerInvoker::operator() for one point at one level
 * (video/src/lkpyramid.cpp:194-694); accumulation per ORC_ACCUM_* */
static void orc_lk_point(const orc_job* jb, int ptidx, int16_t* Iwin, int16_t* dIwin)
{
    const orc_lk_params* prm = jb->prm;
    const orc_level_ctx* L = jb->lv;
    const int winW = prm->winW, winH = prm->winH;
    const int level = jb->level;
    const float halfx = (winW - 1) * 0.5f, halfy = (winH - 1) * 0.5f;
    const int W_BITS = 14, W_BITS1 = 14;
    const float FLT_SCALE = 1.f / (1 << 20);
    const int exact = prm->accum == ORC_ACCUM_EXACT;
    const int Icols = L->I->w, Irows = L->I->h, Jcols = L->J->w, Jrows = L->J->h;
    const int cn = L->I->cn > 0 ? L->I->cn : 1, wcn = winW * cn; /* window row: winW*cn elements */

    float sc = (float)(1. / (1 << level));
    float prevx = jb->prevPts[2 * ptidx] * sc, prevy = jb->prevPts[2 * ptidx + 1] * sc;
    float nextx, nexty;
    if (level == jb->maxLevel) {
        if (prm->flags & ORC_OPTFLOW_USE_INITIAL_FLOW) {
            nextx = jb->nextPts[2 * ptidx] * sc;
            nexty = jb->nextPts[2 * ptidx + 1] * sc;
        } else {
            nextx = prevx;
            nexty = prevy;
        }
    } else {
        nextx = jb->nextPts[2 * ptidx] * 2.f;
        nexty = jb->nextPts[2 * ptidx + 1] * 2.f;
    }
    jb->nextPts[2 * ptidx] = nextx;
    jb->nextPts[2 * ptidx + 1] = nexty;

    prevx -= halfx;
    prevy -= halfy;
    int ipx = orc_floor(prevx), ipy = orc_floor(prevy);
    orc_gate_bounds(jb, ptidx, prevx, prevy, winW, winH, Icols, Irows);
    if (ipx < -winW || ipx >= Icols || ipy < -winH || ipy >= Irows) {
        if (level == 0) {
            jb->status[ptidx] = 0;
            if (jb->err) jb->err[ptidx] = 0;
        }
        return;
    }

    float a = prevx - ipx, b = prevy - ipy;
    int iw00 = orc_round((1.f - a) * (1.f - b) * (1 << W_BITS));
    int iw01 = orc_round(a * (1.f - b) * (1 << W_BITS));
    int iw10 = orc_round((1.f - a) * b * (1 << W_BITS));
    int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

    /* patch extraction + G (lkpyramid.cpp:268-420) */
    float q11[4] = {0, 0, 0, 0}, q12[4] = {0, 0, 0, 0}, q22[4] = {0, 0, 0, 0};
    float t11 = 0, t12 = 0, t22 = 0;
    int64_t e11 = 0, e12 = 0, e22 = 0;
    const int dstep = L->dstride;
    const int cn2 = 2 * cn;
    for (int y = 0; y < winH; ++y) {
        const uint8_t* src = orc_px(L->I, ipx, ipy + y, cn);
        const int stepI = L->I->pitch;
        const int16_t* dsrc = L->dI + (size_t)(ipy + y + L->dpad) * dstep + (size_t)cn2 * (ipx + L->dpad);
        int16_t* Iptr = Iwin + y * wcn;
        int16_t* dIptr = dIwin + 2 * y * wcn;
        for (int x = 0; x < wcn; ++x) {
            int ival = ORC_DESCALE(src[x] * iw00 + src[x + cn] * iw01 + src[x + stepI] * iw10 +
                                   src[x + stepI + cn] * iw11, W_BITS1 - 5);
            int ixval = ORC_DESCALE(dsrc[2 * x] * iw00 + dsrc[2 * x + cn2] * iw01 + dsrc[2 * x + dstep] * iw10 +
                                    dsrc[2 * x + dstep + cn2] * iw11, W_BITS1);
            int iyval = ORC_DESCALE(dsrc[2 * x + 1] * iw00 + dsrc[2 * x + cn2 + 1] * iw01 +
                                    dsrc[2 * x + dstep + 1] * iw10 + dsrc[2 * x + dstep + cn2 + 1] * iw11, W_BITS1);
            Iptr[x] = (int16_t)ival;
            dIptr[2 * x] = (int16_t)ixval;
            dIptr[2 * x + 1] = (int16_t)iyval;
        }
        if (exact) {
            for (int x = 0; x < wcn; ++x) {
                int ix = dIptr[2 * x], iy = dIptr[2 * x + 1];
                e11 += (int64_t)(ix * ix);
                e12 += (int64_t)(ix * iy);
                e22 += (int64_t)(iy * iy);
            }
        } else {
            /* SSE2 lanes: x in chunks of 4 (lkpyramid.cpp:279-316), scalar tail (:403-419) */
            int x = 0;
            for (; x <= wcn - 4; x += 4) {
                for (int k = 0; k < 4; ++k) {
                    float fx = (float)dIptr[2 * (x + k)], fy = (float)dIptr[2 * (x + k) + 1];
                    q22[k] = q22[k] + fy * fy;
                    q12[k] = q12[k] + fx * fy;
                    q11[k] = q11[k] + fx * fx;
                }
            }
            for (; x < wcn; ++x) {
                int ix = dIptr[2 * x], iy = dIptr[2 * x + 1];
                t11 += (float)(ix * ix);
                t12 += (float)(ix * iy);
                t22 += (float)(iy * iy);
            }
        }
    }
    float A11, A12, A22;
    if (exact) {
        A11 = (float)e11 * FLT_SCALE;
        A12 = (float)e12 * FLT_SCALE;
        A22 = (float)e22 * FLT_SCALE;
    } else {
        /* lkpyramid.cpp:422-440 */
        t11 += q11[0] + q11[1] + q11[2] + q11[3];
        t12 += q12[0] + q12[1] + q12[2] + q12[3];
        t22 += q22[0] + q22[1] + q22[2] + q22[3];
        A11 = t11 * FLT_SCALE;
        A12 = t12 * FLT_SCALE;
        A22 = t22 * FLT_SCALE;
    }

    float D = A11 * A22 - A12 * A12;
    float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                   (float)(2 * winW * winH);
    if (jb->err && (prm->flags & ORC_OPTFLOW_LK_GET_MIN_EIGENVALS) != 0) jb->err[ptidx] = minEig;
    if (prm->minEigThreshold > 0) orc_gate_note(jb, ptidx, fabsf(minEig - prm->minEigThreshold) / prm->minEigThreshold);
    orc_gate_note(jb, ptidx, fabsf(D - FLT_EPSILON) / FLT_EPSILON);
    if (minEig < prm->minEigThreshold || D < FLT_EPSILON) {
        if (level == 0) jb->status[ptidx] = 0;
        return;
    }
    D = 1.f / D;

    nextx -= halfx;
    nexty -= halfy;
    float pdx = 0, pdy = 0;
    int nit = 0;
    for (int j = 0; j < jb->maxCount; ++j) {
        int inx = orc_floor(nextx), iny = orc_floor(nexty);
        orc_gate_bounds(jb, ptidx, nextx, nexty, winW, winH, Jcols, Jrows);
        if (inx < -winW || inx >= Jcols || iny < -winH || iny >= Jrows) {
            if (level == 0) jb->status[ptidx] = 0;
            break;
        }
        nit++;
        a = nextx - inx;
        b = nexty - iny;
        iw00 = orc_round((1.f - a) * (1.f - b) * (1 << W_BITS));
        iw01 = orc_round(a * (1.f - b) * (1 << W_BITS));
        iw10 = orc_round((1.f - a) * b * (1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

        float qb0[4] = {0, 0, 0, 0}, qb1[4] = {0, 0, 0, 0};
        float tb1 = 0, tb2 = 0;
        int64_t eb1 = 0, eb2 = 0;
        const int stepJ = L->J->pitch;
        for (int y = 0; y < winH; ++y) {
            const uint8_t* Jptr = orc_px(L->J, inx, iny + y, cn);
            const int16_t* Iptr = Iwin + y * wcn;
            const int16_t* dIptr = dIwin + 2 * y * wcn;
            int d[64 * 4];
            for (int x = 0; x < wcn; ++x)
                d[x] = ORC_DESCALE(Jptr[x] * iw00 + Jptr[x + cn] * iw01 + Jptr[x + stepJ] * iw10 +
                                   Jptr[x + stepJ + cn] * iw11, W_BITS1 - 5) - Iptr[x];
            if (exact) {
                for (int x = 0; x < wcn; ++x) {
                    eb1 += (int64_t)(d[x] * dIptr[2 * x]);
                    eb2 += (int64_t)(d[x] * dIptr[2 * x + 1]);
                }
            } else {
                /* SSE2 lanes: chunks of 8, _mm_madd_epi16 pairs (x, x+4) (lkpyramid.cpp:507-534) */
                int x = 0;
                for (; x <= wcn - 8; x += 8) {
                    const int* dd = d + x;
                    const int16_t* g = dIptr + 2 * x;
                    qb0[0] = qb0[0] + (float)(dd[0] * g[0] + dd[4] * g[8]);
                    qb0[1] = qb0[1] + (float)(dd[0] * g[1] + dd[4] * g[9]);
                    qb0[2] = qb0[2] + (float)(dd[1] * g[2] + dd[5] * g[10]);
                    qb0[3] = qb0[3] + (float)(dd[1] * g[3] + dd[5] * g[11]);
                    qb1[0] = qb1[0] + (float)(dd[2] * g[4] + dd[6] * g[12]);
                    qb1[1] = qb1[1] + (float)(dd[2] * g[5] + dd[6] * g[13]);
                    qb1[2] = qb1[2] + (float)(dd[3] * g[6] + dd[7] * g[14]);
                    qb1[3] = qb1[3] + (float)(dd[3] * g[7] + dd[7] * g[15]);
                }
                for (; x < wcn; ++x) {
                    tb1 += (float)(d[x] * dIptr[2 * x]);
                    tb2 += (float)(d[x] * dIptr[2 * x + 1]);
                }
            }
        }
        float b1, b2;
        if (exact) {
            b1 = (float)eb1 * FLT_SCALE;
            b2 = (float)eb2 * FLT_SCALE;
        } else {
            /* lkpyramid.cpp:619-633 */
            float bb0 = qb0[0] + qb1[0], bb1 = qb0[1] + qb1[1], bb2 = qb0[2] + qb1[2], bb3 = qb0[3] + qb1[3];
            tb1 += bb0 + bb2;
            tb2 += bb1 + bb3;
            b1 = tb1 * FLT_SCALE;
            b2 = tb2 * FLT_SCALE;
        }
        float dx = (A12 * b2 - A22 * b1) * D;
        float dy = (A12 * b1 - A11 * b2) * D;
        nextx += dx;
        nexty += dy;
        jb->nextPts[2 * ptidx] = nextx + halfx;
        jb->nextPts[2 * ptidx + 1] = nexty + halfy;
        if ((double)dx * dx + (double)dy * dy <= jb->eps2) break;
        if (j > 0 && fabs((double)fabsf(dx + pdx)) < 0.01 && fabs((double)fabsf(dy + pdy)) < 0.01) {
            jb->nextPts[2 * ptidx] -= dx * 0.5f;
            jb->nextPts[2 * ptidx + 1] -= dy * 0.5f;
            break;
        }
        pdx = dx;
        pdy = dy;
    }
    if (jb->iters) jb->iters[ptidx] += nit;

    /* error at level 0 (lkpyramid.cpp:654-693) */
    if (jb->status[ptidx] && jb->err && level == 0 && (prm->flags & ORC_OPTFLOW_LK_GET_MIN_EIGENVALS) == 0) {
        float npx = jb->nextPts[2 * ptidx] - halfx, npy = jb->nextPts[2 * ptidx + 1] - halfy;
        int inx = orc_floor(npx), iny = orc_floor(npy);
        orc_gate_bounds(jb, ptidx, npx, npy, winW, winH, Jcols, Jrows);
        if (inx < -winW || inx >= Jcols || iny < -winH || iny >= Jrows) {
            jb->status[ptidx] = 0;
            return;
        }
        float aa = npx - inx, bb = npy - iny;
        iw00 = orc_round((1.f - aa) * (1.f - bb) * (1 << W_BITS));
        iw01 = orc_round(aa * (1.f - bb) * (1 << W_BITS));
        iw10 = orc_round((1.f - aa) * bb * (1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        float errval = 0.f;
        const int stepJ = L->J->pitch;
        for (int y = 0; y < winH; ++y) {
            const uint8_t* Jptr = orc_px(L->J, inx, iny + y, cn);
            const int16_t* Iptr = Iwin + y * wcn;
            for (int x = 0; x < wcn; ++x) {
                int diff = ORC_DESCALE(Jptr[x] * iw00 + Jptr[x + cn] * iw01 + Jptr[x + stepJ] * iw10 +
                                       Jptr[x + stepJ + cn] * iw11, W_BITS1 - 5) - Iptr[x];
                errval += fabsf((float)diff);
            }
        }
        jb->err[ptidx] = errval * 1.f / (float)(32 * winW * cn * winH);
    }
}

static void* orc_lk_worker(void* arg)
{
    const orc_job* jb = (const orc_job*)arg;
    const int cn = jb->lv->I->cn > 0 ? jb->lv->I->cn : 1;
    int area = jb->prm->winW * jb->prm->winH * cn;
    int16_t* Iwin = (int16_t*)malloc(sizeof(int16_t) * (size_t)area * 3);
    for (int i = jb->begin; i < jb->end; ++i) orc_lk_point(jb, i, Iwin, Iwin + area);
    free(Iwin);
    return NULL;
}

int orc_lk(const orc_pyr* prev, const orc_pyr* next,
           const float* prevPts, float* nextPts, uint8_t* status, float* err,
           int npoints, const orc_lk_params* prm, int32_t* iters)
{
    return orc_lk_gate(prev, next, prevPts, nextPts, status, err, npoints, prm, iters, NULL);
}

int orc_lk_gate(const orc_pyr* prev, const orc_pyr* next,
                const float* prevPts, float* nextPts, uint8_t* status, float* err,
                int npoints, const orc_lk_params* prm, int32_t* iters, float* gate)
{
    if (npoints <= 0) return 0;
    if (prm->winW < 3 || prm->winH < 3 || prm->winW > 64 || prm->winH > 64) return -1;
    if (prev->lv[0].cn > 4) return -1;
    int maxLevel = prm->maxLevel;
    if (prev->nlevels - 1 < maxLevel) maxLevel = prev->nlevels - 1;
    if (next->nlevels - 1 < maxLevel) maxLevel = next->nlevels - 1;
    int maxCount = prm->maxCount < 0 ? 0 : (prm->maxCount > 100 ? 100 : prm->maxCount);
    double eps = prm->epsilon < 0. ? 0. : (prm->epsilon > 10. ? 10. : prm->epsilon);
    for (int i = 0; i < npoints; ++i) status[i] = 1;
    if (iters) memset(iters, 0, sizeof(int32_t) * (size_t)npoints);
    if (gate)
        for (int i = 0; i < npoints; ++i) gate[i] = FLT_MAX;
    int nth = prm->nthreads > 0 ? prm->nthreads : 1;
    if (nth > npoints) nth = npoints;

    for (int level = maxLevel; level >= 0; --level) {
        const orc_plane* I = &prev->lv[level];
        const orc_plane* J = &next->lv[level];
        const int cn = I->cn > 0 ? I->cn : 1;
        if (I->w != J->w || I->h != J->h || cn != (J->cn > 0 ? J->cn : 1)) return -2;
        int dpad = prm->winW > prm->winH ? prm->winW + 1 : prm->winH + 1;
        int dstride = 2 * cn * (I->w + 2 * dpad);
        int16_t* dI = (int16_t*)calloc((size_t)dstride * (I->h + 2 * dpad), sizeof(int16_t));
        orc_scharr_cn(I->data + (size_t)I->pad * I->pitch + (size_t)I->pad * cn, I->w, I->h, I->pitch, cn,
                      dI + (size_t)dpad * dstride + 2 * cn * dpad, dstride);
        orc_level_ctx lctx = {I, J, dI, dpad, dstride};
        orc_job* jobs = (orc_job*)malloc(sizeof(orc_job) * (size_t)nth);
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nth);
        for (int t = 0; t < nth; ++t) {
            orc_job* jb = &jobs[t];
            jb->lv = &lctx;
            jb->prevPts = prevPts;
            jb->nextPts = nextPts;
            jb->status = status;
            jb->err = err;
            jb->iters = iters;
            jb->gate = gate;
            jb->prm = prm;
            jb->level = level;
            jb->maxLevel = maxLevel;
            jb->maxCount = maxCount;
            jb->eps2 = eps * eps;
            jb->begin = (int)((int64_t)npoints * t / nth);
            jb->end = (int)((int64_t)npoints * (t + 1) / nth);
        }
        if (nth == 1) {
            orc_lk_worker(&jobs[0]);
        } else {
            for (int t = 0; t < nth; ++t) pthread_create(&th[t], NULL, orc_lk_worker, &jobs[t]);
            for (int t = 0; t < nth; ++t) pthread_join(th[t], NULL);
        }
        free(th);
        free(jobs);
        free(dI);
    }
    return maxLevel;
}

/* ------------------------------------------------------------------ synth */

int orc_synth_frames(uint32_t seed, int W, int H, int nobj, int t0, int nframes,
                     uint8_t* out, int pitch, int32_t* gt_boxes)
{
    if (nobj > SYN_MAX_OBJECTS) return -1;
    syn_object* objs = (syn_object*)malloc(sizeof(syn_object) * (size_t)(nobj > 0 ? nobj : 1));
    syn_pose* poses = (syn_pose*)malloc(sizeof(syn_pose) * (size_t)(nobj > 0 ? nobj : 1));
    syn_make_objects(seed, W, H, nobj, objs);
    uint32_t bgseed = syn_hash(seed ^ 0xB6A5EEDU);
    for (int f = 0; f < nframes; ++f) {
        int t = t0 + f;
        for (int o = 0; o < nobj; ++o) {
            syn_pose_at(&objs[o], W, H, t, &poses[o]);
            if (gt_boxes) {
                int32_t* g = gt_boxes + ((size_t)f * nobj + o) * 5;
                g[0] = syn_gt_box(&poses[o], W, H, g + 1);
                if (!g[0]) g[1] = g[2] = g[3] = g[4] = 0;
            }
        }
        if (!out) continue; /* ground truth only */
        uint8_t* img = out + (size_t)f * pitch * H;
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) img[(size_t)y * pitch + x] = (uint8_t)syn_background(x, y, bgseed);
        /* draw objects in order over their boxes (last hit wins) */
        for (int o = 0; o < nobj; ++o) {
            const syn_pose* p = &poses[o];
            int x0 = p->bx0 < 0 ? 0 : p->bx0, y0 = p->by0 < 0 ? 0 : p->by0;
            int x1 = p->bx1 > W ? W : p->bx1, y1 = p->by1 > H ? H : p->by1;
            for (int y = y0; y < y1; ++y)
                for (int x = x0; x < x1; ++x) {
                    int v;
                    if (syn_object_texel(p, x, y, &v)) img[(size_t)y * pitch + x] = (uint8_t)v;
                }
        }
    }
    free(objs);
    free(poses);
    return 0;
}
