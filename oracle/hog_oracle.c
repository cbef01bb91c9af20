/*
 * hog_oracle.c — CPU restatement of the reference's HOG people detector
 * (cv::HOGDescriptor, modules/objdetect/src/hog.cpp), which the sample's
 * detection step calls (samples/gpu/tbd.cpp:596-606; cv::cuda::HOG in GPU mode).
 *
 * TEST INFRASTRUCTURE ONLY: tests/ use it as the checker of libtbdk's hog.hip;
 * the product never links it.
 *
 * Restated with the reference's operation order:
 *   resize INTER_LINEAR_EXACT (u8)  imgproc/src/resize.cpp:732-891 (interpolationLinear
 *                                  coefficients in 8.8 fixed point, ufixedpoint16/32
 *                                  arithmetic of imgproc/src/fixedpoint.inl.hpp:309-380)
 *   computeGradient                hog.cpp:239-550 (gamma LUT, REFLECT_101 borders, the
 *                                  3-channel max-magnitude pick with the SSE2 body's and
 *                                  the scalar tail's different tie rules, bin split)
 *   cartToPolar -> magnitude32f / fastAtan32f  core/src/mathfuncs_core.simd.hpp:76-225,
 *                                  the AVX2 dispatch (8 lanes, FMA) the reference selects at
 *                                  run time on an x86-64 host; scalar for rows < 16 pixels
 *   HOGCache::init / getBlock      hog.cpp:619-1117 (Gaussian block weights, pixData
 *                                  tables in count1/count2/count4 order, SSE2 weights)
 *   normalizeBlockHistogram        hog.cpp:1119-1248 (4-lane partial sums, L2-Hys)
 *   detect                         hog.cpp:1655-1767 (4-lane float block dot, double sum)
 *   detectMultiScale / HOGInvoker  hog.cpp:1799-1839, 2051-2105
 *   groupRectangles                hog.cpp:3783-3861 with partition() and SimilarRects
 *                                  (core/include/opencv2/core/operations.hpp,
 *                                  objdetect.hpp) and clipObjects (cascadedetect.cpp:1683)
 * Parity against the reference binaries is unpinned: the reference's HOG tests
 * read images from opencv_extra, which is not vendored.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct orc_hog_params {
    int win_w, win_h, block_w, block_h, bstride_x, bstride_y, cell_w, cell_h, nbins;
    double win_sigma;       /* <= 0: (block_w + block_h) / 8 */
    double l2hys;           /* 0.2 */
    int gamma;              /* gammaCorrection */
    int signed_grad;
    int wstride_x, wstride_y;
} orc_hog_params;

static int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

/* ---- resize(src, dst, size, 0, 0, INTER_LINEAR_EXACT), u8, cn channels ---- */

static void lin_coeffs(double inv_scale, int ssize, int dsize, int* ofs, int* c0, int* c1, int* mn, int* mx)
{
    const double scale = 1. / inv_scale;
    *mn = 0;
    *mx = dsize;
    for (int d = 0; d < dsize; d++) {
        const double f = scale * ((double)d + 0.5) - 0.5;
        const int iv = (int)floor(f);
        ofs[d] = 0, c0[d] = 256, c1[d] = 0;
        if (iv >= 0 && ssize > 1) {
            if (iv < ssize - 1) {
                ofs[d] = iv;
                const double fr = f - iv;
                c1[d] = fr < 0 ? 0 : (int)lrint(fr * 256.0);
                c0[d] = 256 - c1[d];
            } else {
                ofs[d] = ssize - 1;
                if (d < *mx) *mx = d;
            }
        } else if (d + 1 > *mn) {
            *mn = d + 1;
        }
    }
}

void orc_hog_resize_exact(const uint8_t* src, int sw, int sh, int spitch, int cn, uint8_t* dst, int dw, int dh,
                          int dpitch)
{
    int *xo = malloc(sizeof(int) * dw * 3), *yo = malloc(sizeof(int) * dh * 3);
    int minx, maxx, miny, maxy;
    lin_coeffs((double)dw / sw, sw, dw, xo, xo + dw, xo + 2 * dw, &minx, &maxx);
    lin_coeffs((double)dh / sh, sh, dh, yo, yo + dh, yo + 2 * dh, &miny, &maxy);
    uint32_t* line = malloc(sizeof(uint32_t) * dw * cn * 2);
    /* hline: ufixedpoint16 (8 fractional bits) per output column */
#define HLINE(row, out)                                                                      \
    do {                                                                                     \
        const uint8_t* S = src + (size_t)(row)*spitch;                                       \
        for (int dx = 0; dx < dw; dx++)                                                      \
            for (int c = 0; c < cn; c++) {                                                   \
                uint32_t v;                                                                  \
                if (dx < minx) v = (uint32_t)S[c] << 8;                                      \
                else if (dx >= maxx) v = (uint32_t)S[(sw - 1) * cn + c] << 8;                \
                else v = (uint32_t)xo[dw + dx] * S[xo[dx] * cn + c] +                        \
                         (uint32_t)xo[2 * dw + dx] * S[(xo[dx] + 1) * cn + c];               \
                (out)[dx * cn + c] = v;                                                      \
            }                                                                                \
    } while (0)
    for (int dy = 0; dy < dh; dy++) {
        uint8_t* D = dst + (size_t)dy * dpitch;
        if (dy < miny || dy >= maxy) {
            HLINE(dy < miny ? 0 : sh - 1, line);
            for (int x = 0; x < dw * cn; x++) D[x] = (uint8_t)((line[x] + 128) >> 8);
            continue;
        }
        HLINE(yo[dy], line);
        HLINE(yo[dy] + 1, line + dw * cn);
        for (int x = 0; x < dw * cn; x++) {
            const uint32_t v = line[x] * (uint32_t)yo[dh + dy] + line[dw * cn + x] * (uint32_t)yo[2 * dh + dy];
            D[x] = (uint8_t)((v + 32768) >> 16);
        }
    }
#undef HLINE
    free(line);
    free(xo);
    free(yo);
}

/* ---- computeGradient (padding 0) ---- */

static const float kAtanP1 = 0.9997878412794807f * (float)(180 / M_PI);
static const float kAtanP3 = -0.3258083974640975f * (float)(180 / M_PI);
static const float kAtanP5 = 0.1555786518463281f * (float)(180 / M_PI);
static const float kAtanP7 = -0.04432655554792128f * (float)(180 / M_PI);

/* fastAtan32f element: vector form (v_atan_f32::compute, FMA) or scalar atan_f32 */
static float fast_atan(float y, float x, int vec)
{
    const float ax = fabsf(x), ay = fabsf(y);
    float a;
    if (vec) {
        const float c = fminf(ax, ay) / (fmaxf(ax, ay) + (float)DBL_EPSILON);
        const float cc = c * c;
        a = fmaf(fmaf(fmaf(cc, kAtanP7, kAtanP5), cc, kAtanP3), cc, kAtanP1) * c;
        if (!(ax >= ay)) a = 90.f - a;
        if (x < 0) a = 180.f - a;
        if (y < 0) a = 360.f - a;
    } else {
        float c, c2;
        if (ax >= ay) {
            c = ay / (ax + (float)DBL_EPSILON);
            c2 = c * c;
            a = (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
        } else {
            c = ax / (ay + (float)DBL_EPSILON);
            c2 = c * c;
            a = 90.f - (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
        }
        if (x < 0) a = 180.f - a;
        if (y < 0) a = 360.f - a;
    }
    return a * (float)(M_PI / 180);
}

/* img: u8, cn 1 or 3 (BGR; cn 4 = BGRA read as BGR), pitch bytes.
 * grad: w*h*2 floats; qangle: w*h*2 bytes. */
void orc_hog_gradient(const uint8_t* img, int w, int h, int pitch, int cn, int nbins, int gamma, int signed_grad,
                      float* grad, uint8_t* qangle)
{
    float lut[256];
    for (int i = 0; i < 256; i++) lut[i] = gamma ? sqrtf((float)i) : (float)i;
    const float angle_scale = signed_grad ? (float)(nbins / (2.0 * M_PI)) : (float)(nbins / M_PI);
    /* cartToPolar feeds magnitude32f/fastAtan32f 1024-element chunks of the row
     * (core/src/mathfuncs.cpp:285-298, BLOCK_SIZE precomp.hpp:269); a chunk shorter
     * than 2 x 8 AVX2 lanes runs the scalar forms (mathfuncs_core.simd.hpp:131-138,202-207) */
    const int simd_w = w & ~3;   /* the SSE2 3-channel body */
    for (int y = 0; y < h; y++) {
        const uint8_t* P = img + (size_t)y * pitch;
        const uint8_t* Pp = img + (size_t)reflect101(y - 1, h) * pitch;
        const uint8_t* Pn = img + (size_t)reflect101(y + 1, h) * pitch;
        for (int x = 0; x < w; x++) {
            const int xl = reflect101(x - 1, w), xr = reflect101(x + 1, w);
            float dx, dy;
            if (cn == 1) {
                dx = lut[P[xr]] - lut[P[xl]];
                dy = lut[Pn[x]] - lut[Pp[x]];
            } else {
                float ddx[3], ddy[3], mag[3];
                for (int c = 0; c < 3; c++) {
                    ddx[c] = lut[P[xr * cn + c]] - lut[P[xl * cn + c]];
                    ddy[c] = lut[Pn[x * cn + c]] - lut[Pp[x * cn + c]];
                    mag[c] = ddx[c] * ddx[c] + ddy[c] * ddy[c];
                }
                if (x < simd_w) { /* mask = m2 > m1 ? 2 : 1; then max(m2, m1) > m0 ? that : 0 */
                    int k = mag[2] > mag[1] ? 2 : 1;
                    if (!(fmaxf(mag[2], mag[1]) > mag[0])) k = 0;
                    dx = ddx[k], dy = ddy[k];
                } else { /* start at 2; replace when strictly smaller */
                    int k = 2;
                    if (mag[k] < mag[1]) k = 1;
                    if (mag[k] < mag[0]) k = 0;
                    dx = ddx[k], dy = ddy[k];
                }
            }
            const int chunk = w - (x / 1024) * 1024, vec_mag = (chunk < 1024 ? chunk : 1024) >= 16;
            const float m = vec_mag ? sqrtf(fmaf(dx, dx, dy * dy)) : sqrtf(dx * dx + dy * dy);
            float ang = fast_atan(dy, dx, vec_mag) * angle_scale - 0.5f;
            int hidx = (int)floorf(ang);
            ang -= hidx;
            float* G = grad + ((size_t)y * w + x) * 2;
            G[0] = m * (1.f - ang);
            G[1] = m * ang;
            if (hidx < 0) hidx += nbins;
            else if (hidx >= nbins) hidx -= nbins;
            uint8_t* Q = qangle + ((size_t)y * w + x) * 2;
            Q[0] = (uint8_t)hidx;
            hidx++;
            Q[1] = (uint8_t)(hidx < nbins ? hidx : 0);
        }
    }
}

/* ---- HOGCache tables ---- */

typedef struct {
    int di, dj;      /* pixel inside the block */
    int n;           /* entries used (1, 2 or 4) */
    int hofs[4];
    float hw[4];     /* histWeights */
    float gw;        /* gradWeight */
} PixData;

static double win_sigma(const orc_hog_params* p)
{
    return p->win_sigma > 0 ? p->win_sigma : (p->block_w + p->block_h) / 8.;
}

/* HOGCache::init's pixData in its final (count1, count2, count4) order */
int orc_hog_pixdata(const orc_hog_params* p, PixData* out)
{
    const int bw = p->block_w, bh = p->block_h, ncx = bw / p->cell_w, ncy = bh / p->cell_h, nb = p->nbins;
    const int raw = bw * bh;
    PixData* tmp = malloc(sizeof(PixData) * raw * 3);
    float* di = malloc(sizeof(float) * bh);
    float* dj = malloc(sizeof(float) * bw);
    const float sigma = (float)win_sigma(p);
    const float scale = 1.f / (sigma * sigma * 2);
    const float fbh = bh * 0.5f, fbw = bw * 0.5f;
    for (int i = 0; i < bh; i++) {
        di[i] = i - fbh;
        di[i] *= di[i];
    }
    for (int j = 0; j < bw; j++) {
        dj[j] = j - fbw;
        dj[j] *= dj[j];
    }
    int c1 = 0, c2 = 0, c4 = 0;
    for (int j = 0; j < bw; j++)
        for (int i = 0; i < bh; i++) {
            PixData* d;
            float cellX = (j + 0.5f) / p->cell_w - 0.5f;
            float cellY = (i + 0.5f) / p->cell_h - 0.5f;
            int icx0 = (int)floorf(cellX), icy0 = (int)floorf(cellY);
            int icx1 = icx0 + 1, icy1 = icy0 + 1;
            cellX -= icx0;
            cellY -= icy0;
            const int x0ok = (unsigned)icx0 < (unsigned)ncx, x1ok = (unsigned)icx1 < (unsigned)ncx;
            const int y0ok = (unsigned)icy0 < (unsigned)ncy, y1ok = (unsigned)icy1 < (unsigned)ncy;
            if (x0ok && x1ok) {
                if (y0ok && y1ok) {
                    d = &tmp[raw * 2 + c4++];
                    d->n = 4;
                    d->hofs[0] = (icx0 * ncy + icy0) * nb, d->hw[0] = (1.f - cellX) * (1.f - cellY);
                    d->hofs[1] = (icx1 * ncy + icy0) * nb, d->hw[1] = cellX * (1.f - cellY);
                    d->hofs[2] = (icx0 * ncy + icy1) * nb, d->hw[2] = (1.f - cellX) * cellY;
                    d->hofs[3] = (icx1 * ncy + icy1) * nb, d->hw[3] = cellX * cellY;
                } else {
                    d = &tmp[raw + c2++];
                    d->n = 2;
                    if (y0ok) {
                        icy1 = icy0;
                        cellY = 1.f - cellY;
                    }
                    d->hofs[0] = (icx0 * ncy + icy1) * nb, d->hw[0] = (1.f - cellX) * cellY;
                    d->hofs[1] = (icx1 * ncy + icy1) * nb, d->hw[1] = cellX * cellY;
                }
            } else {
                if (x0ok) {
                    icx1 = icx0;
                    cellX = 1.f - cellX;
                }
                if (y0ok && y1ok) {
                    d = &tmp[raw + c2++];
                    d->n = 2;
                    d->hofs[0] = (icx1 * ncy + icy0) * nb, d->hw[0] = cellX * (1.f - cellY);
                    d->hofs[1] = (icx1 * ncy + icy1) * nb, d->hw[1] = cellX * cellY;
                } else {
                    d = &tmp[c1++];
                    d->n = 1;
                    if (y0ok) {
                        icy1 = icy0;
                        cellY = 1.f - cellY;
                    }
                    d->hofs[0] = (icx1 * ncy + icy1) * nb, d->hw[0] = cellX * cellY;
                }
            }
            d->di = i, d->dj = j;
            d->gw = expf(-(di[i] + dj[j]) * scale);
        }
    int k = 0;
    for (int t = 0; t < c1; t++) out[k++] = tmp[t];
    for (int t = 0; t < c2; t++) out[k++] = tmp[raw + t];
    for (int t = 0; t < c4; t++) out[k++] = tmp[raw * 2 + t];
    free(tmp);
    free(di);
    free(dj);
    return k;
}

static void normalize_block(float* hist, int sz, float thresh)
{
    float ps[4], sum;
    int i;
    for (int l = 0; l < 4; l++) ps[l] = hist[l] * hist[l];
    for (i = 4; i <= sz - 4; i += 4)
        for (int l = 0; l < 4; l++) ps[l] = ps[l] + hist[i + l] * hist[i + l];
    sum = (ps[0] + ps[1]) + (ps[2] + ps[3]);
    for (; i < sz; ++i) sum += hist[i] * hist[i];
    float scale = 1.f / (sqrtf(sum) + sz * 0.1f);
    for (int l = 0; l < 4; l++) {
        hist[l] = fminf(scale * hist[l], thresh);
        ps[l] = hist[l] * hist[l];
    }
    for (i = 4; i <= sz - 4; i += 4)
        for (int l = 0; l < 4; l++) {
            hist[i + l] = fminf(hist[i + l] * scale, thresh);
            ps[l] = ps[l] + hist[i + l] * hist[i + l];
        }
    sum = (ps[0] + ps[1]) + (ps[2] + ps[3]);
    for (; i < sz; ++i) {
        hist[i] = fminf(hist[i] * scale, thresh);
        sum += hist[i] * hist[i];
    }
    scale = 1.f / (sqrtf(sum) + 1e-3f);
    for (i = 0; i < sz; i++) hist[i] = scale * hist[i];
}

/* getBlock at (x, y) of a w-wide gradient image: out = blockHistogramSize floats */
static void get_block(const float* grad, const uint8_t* qangle, int w, int x, int y, const PixData* pd, int npd,
                      int sz, float thresh, float* out)
{
    memset(out, 0, sizeof(float) * sz);
    for (int k = 0; k < npd; k++) {
        const PixData* q = &pd[k];
        const size_t o = ((size_t)(y + q->di) * w + x + q->dj) * 2;
        const float a0 = grad[o], a1 = grad[o + 1];
        const int h0 = qangle[o], h1 = qangle[o + 1];
        for (int e = 0; e < q->n; e++) {
            const float wgt = q->gw * q->hw[e];
            float* hist = out + q->hofs[e];
            const float t0 = hist[h0] + a0 * wgt;
            const float t1 = hist[h1] + a1 * wgt;
            hist[h0] = t0;
            hist[h1] = t1;
        }
    }
    normalize_block(out, sz, thresh);
}

static int gcd_(int a, int b)
{
    while (b) {
        const int t = a % b;
        a = b;
        b = t;
    }
    return a;
}

/* every block of the cache grid (stride gcd(winStride, blockStride)) of a
 * gradient image: blocks[(by * nbx + bx) * sz] */
void orc_hog_blocks(const float* grad, const uint8_t* qangle, int w, int h, const orc_hog_params* p, float* blocks,
                    int* nbx_out, int* nby_out)
{
    const int csx = gcd_(p->wstride_x, p->bstride_x), csy = gcd_(p->wstride_y, p->bstride_y);
    const int nbx = (w - p->block_w) / csx + 1, nby = (h - p->block_h) / csy + 1;
    const int sz = (p->block_w / p->cell_w) * (p->block_h / p->cell_h) * p->nbins;
    PixData* pd = malloc(sizeof(PixData) * p->block_w * p->block_h);
    const int npd = orc_hog_pixdata(p, pd);
    for (int by = 0; by < nby; by++)
        for (int bx = 0; bx < nbx; bx++)
            get_block(grad, qangle, w, bx * csx, by * csy, pd, npd, sz, (float)p->l2hys,
                      blocks + ((size_t)by * nbx + bx) * sz);
    free(pd);
    *nbx_out = nbx;
    *nby_out = nby;
}

/* HOGDescriptor::detect on one image (padding 0): hits in window order.
 * xs/ys/scores have room for every window; returns the hit count. */
int orc_hog_detect(const uint8_t* img, int w, int h, int pitch, int cn, const orc_hog_params* p, const float* svm,
                   int svm_len, double hit_threshold, int* xs, int* ys, double* scores)
{
    if (w < p->win_w || h < p->win_h) return 0;
    float* grad = malloc(sizeof(float) * 2 * (size_t)w * h);
    uint8_t* qa = malloc(2 * (size_t)w * h);
    orc_hog_gradient(img, w, h, pitch, cn, p->nbins, p->gamma, p->signed_grad, grad, qa);
    const int csx = gcd_(p->wstride_x, p->bstride_x), csy = gcd_(p->wstride_y, p->bstride_y);
    const int sz = (p->block_w / p->cell_w) * (p->block_h / p->cell_h) * p->nbins;
    const int nbx = (w - p->block_w) / csx + 1, nby = (h - p->block_h) / csy + 1;
    float* blocks = malloc(sizeof(float) * (size_t)nbx * nby * sz);
    int gx, gy;
    orc_hog_blocks(grad, qa, w, h, p, blocks, &gx, &gy);
    const int wbx = (p->win_w - p->block_w) / p->bstride_x + 1, wby = (p->win_h - p->block_h) / p->bstride_y + 1;
    const int dsize = wbx * wby * sz;
    const double rho = svm_len > dsize ? svm[dsize] : 0;
    const int nwx = (w - p->win_w) / p->wstride_x + 1, nwy = (h - p->win_h) / p->wstride_y + 1;
    int nhit = 0;
    for (int wy = 0; wy < nwy; wy++)
        for (int wx = 0; wx < nwx; wx++) {
            const int x0 = wx * p->wstride_x, y0 = wy * p->wstride_y;
            double s = rho;
            const float* sv = svm;
            for (int j = 0; j < wbx; j++)
                for (int i = 0; i < wby; i++, sv += sz) { /* blockData: x-major */
                    const int bx = (x0 + j * p->bstride_x) / csx, by = (y0 + i * p->bstride_y) / csy;
                    const float* v = blocks + ((size_t)by * nbx + bx) * sz;
                    float ps[4];
                    int k;
                    for (int l = 0; l < 4; l++) ps[l] = sv[l] * v[l];
                    for (k = 4; k <= sz - 4; k += 4)
                        for (int l = 0; l < 4; l++) ps[l] = ps[l] + v[k + l] * sv[k + l];
                    const double t0 = ps[0] + ps[1], t1 = ps[2] + ps[3];
                    s += t0 + t1;
                    for (; k < sz; k++) s += v[k] * sv[k];
                }
            if (s >= hit_threshold) {
                xs[nhit] = x0, ys[nhit] = y0, scores[nhit] = s;
                nhit++;
            }
        }
    free(grad);
    free(qa);
    free(blocks);
    return nhit;
}

/* ---- groupRectangles (weights version) + clipObjects ---- */

static int similar(const int* a, const int* b, double eps)
{
    const double delta = eps * ((a[2] < b[2] ? a[2] : b[2]) + (a[3] < b[3] ? a[3] : b[3])) * 0.5;
    return fabs((double)(a[0] - b[0])) <= delta && fabs((double)(a[1] - b[1])) <= delta &&
           fabs((double)(a[0] + a[2] - b[0] - b[2])) <= delta && fabs((double)(a[1] + a[3] - b[1] - b[3])) <= delta;
}

static int find_root(int* parent, int i)
{
    while (parent[i] != i) i = parent[i];
    return i;
}

/* rects: n x (x, y, w, h) in/out; weights in/out.  Returns the new count. */
int orc_hog_group(int* rects, double* weights, int n, int group_threshold, double eps, int img_w, int img_h)
{
    if (group_threshold > 0 && n > 0) {
        /* connected components of the similarity graph (partition()'s classes) */
        int* parent = malloc(sizeof(int) * n);
        for (int i = 0; i < n; i++) parent[i] = i;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < i; j++)
                if (similar(rects + 4 * i, rects + 4 * j, eps)) {
                    const int a = find_root(parent, i), b = find_root(parent, j);
                    if (a != b) parent[a] = b;
                }
        int* label = malloc(sizeof(int) * n);
        int ncls = 0;
        int* root_cls = malloc(sizeof(int) * n);
        for (int i = 0; i < n; i++) root_cls[i] = -1;
        for (int i = 0; i < n; i++) {
            const int r = find_root(parent, i);
            if (root_cls[r] < 0) root_cls[r] = ncls++;
            label[i] = root_cls[r];
        }
        double* rr = calloc((size_t)ncls * 4, sizeof(double));
        int* cnt = calloc(ncls, sizeof(int));
        double* fw = malloc(sizeof(double) * ncls);
        for (int c = 0; c < ncls; c++) fw[c] = -DBL_MAX;
        for (int i = 0; i < n; i++) {
            const int c = label[i];
            for (int t = 0; t < 4; t++) rr[4 * c + t] += rects[4 * i + t];
            if (weights[i] > fw[c]) fw[c] = weights[i];
            cnt[c]++;
        }
        int* ri = malloc(sizeof(int) * 4 * ncls);
        for (int c = 0; c < ncls; c++) {
            const double s = 1.0 / cnt[c];
            for (int t = 0; t < 4; t++) ri[4 * c + t] = (int)lrint(rr[4 * c + t] * s); /* Rect_<double> -> Rect */
        }
        int m = 0;
        for (int i = 0; i < ncls; i++) {
            const int* r1 = ri + 4 * i;
            const int n1 = cnt[i];
            if (n1 <= group_threshold) continue;
            int j;
            for (j = 0; j < ncls; j++) {
                const int n2 = cnt[j];
                if (j == i || n2 <= group_threshold) continue;
                const int* r2 = ri + 4 * j;
                const int dx = (int)lrint(r2[2] * eps), dy = (int)lrint(r2[3] * eps);
                if (r1[0] >= r2[0] - dx && r1[1] >= r2[1] - dy && r1[0] + r1[2] <= r2[0] + r2[2] + dx &&
                    r1[1] + r1[3] <= r2[1] + r2[3] + dy && (n2 > (n1 > 3 ? n1 : 3) || n1 < 3))
                    break;
            }
            if (j == ncls) {
                memcpy(rects + 4 * m, r1, sizeof(int) * 4);
                weights[m] = fw[i];
                m++;
            }
        }
        n = m;
        free(parent);
        free(label);
        free(root_cls);
        free(rr);
        free(cnt);
        free(fw);
        free(ri);
    }
    /* clipObjects: intersect with the image, drop empty */
    int m = 0;
    for (int i = 0; i < n; i++) {
        int x0 = rects[4 * i], y0 = rects[4 * i + 1];
        int x1 = x0 + rects[4 * i + 2], y1 = y0 + rects[4 * i + 3];
        x0 = x0 > 0 ? x0 : 0, y0 = y0 > 0 ? y0 : 0;
        x1 = x1 < img_w ? x1 : img_w, y1 = y1 < img_h ? y1 : img_h;
        if (x1 <= x0 || y1 <= y0) continue;
        rects[4 * m] = x0, rects[4 * m + 1] = y0, rects[4 * m + 2] = x1 - x0, rects[4 * m + 3] = y1 - y0;
        weights[m] = weights[i];
        m++;
    }
    return m;
}

/* HOGDescriptor::detectMultiScale(img, rects, weights, hit_threshold, winStride,
 * padding 0, scale0, group_threshold, false).  rects: room for max_rects x 4. */
int orc_hog_detect_multiscale(const uint8_t* img, int w, int h, int pitch, int cn, const orc_hog_params* p,
                              const float* svm, int svm_len, double hit_threshold, int nlevels, double scale0,
                              int group_threshold, int* rects, double* weights, int max_rects)
{
    double scale = 1.;
    double lv[256];
    int levels;
    for (levels = 0; levels < nlevels && levels < 256; levels++) {
        lv[levels] = scale;
        if ((int)lrint(w / scale) < p->win_w || (int)lrint(h / scale) < p->win_h || scale0 <= 1) break;
        scale *= scale0;
    }
    if (levels < 1) levels = 1;
    int n = 0;
    uint8_t* small = malloc((size_t)w * h * cn);
    const int nwin = (w / p->wstride_x + 1) * (h / p->wstride_y + 1);
    int *xs = malloc(sizeof(int) * nwin), *ys = malloc(sizeof(int) * nwin);
    double* sc = malloc(sizeof(double) * nwin);
    for (int l = 0; l < levels; l++) {
        const double s = lv[l];
        const int sw = (int)lrint(w / s), sh = (int)lrint(h / s);
        const uint8_t* li = img;
        int lp = pitch;
        if (sw != w || sh != h) {
            orc_hog_resize_exact(img, w, h, pitch, cn, small, sw, sh, sw * cn);
            li = small;
            lp = sw * cn;
        }
        const int k = orc_hog_detect(li, sw, sh, lp, cn, p, svm, svm_len, hit_threshold, xs, ys, sc);
        const int ww = (int)lrint(p->win_w * s), wh = (int)lrint(p->win_h * s);
        for (int i = 0; i < k && n < max_rects; i++, n++) {
            rects[4 * n] = (int)lrint(xs[i] * s);
            rects[4 * n + 1] = (int)lrint(ys[i] * s);
            rects[4 * n + 2] = ww;
            rects[4 * n + 3] = wh;
            weights[n] = sc[i];
        }
    }
    free(small);
    free(xs);
    free(ys);
    free(sc);
    return orc_hog_group(rects, weights, n, group_threshold, 0.2, w, h);
}
