/*
 * synth_spec.h — deterministic synthetic TBD sequence specification.
 *
 * The reference has no vendored video for the TBD path;
 * BASELINE.md §3 asks for an in-repo generator that is bit-identical on host and
 * device.  This header is that specification.  It is included by
 *   - the HIP renderer (opencv_amd/csrc/synth.hip)            — bench/test input
 *   - the host pose/GT-box tables (opencv_amd/csrc/synth_host.cpp)
 *   - the CPU oracle (oracle/klt_oracle.c)                     — test checker
 * so that a frame generated on an MI355X equals the one the oracle renders.
 *
 * Model (modelled on the moving-rectangle scene of
 * modules/python/test/tst_scene_render.py:14-22 in the reference):
 *   background : two-octave integer value noise, static.
 *   objects    : N textured rectangles (64..200 px), each with a bouncing
 *                constant velocity (|v| <= 3 px/frame), a rotation of
 *                <= 1 deg/frame and a triangle-wave scale in [0.85, 1.15].
 *                Later objects occlude earlier ones.
 * Everything per pixel is integer arithmetic; the per-frame pose is computed once
 * on the host in IEEE double (no libm: own sin/cos) and quantised to Q16.
 */
#ifndef OPENCV_AMD_SYNTH_SPEC_H
#define OPENCV_AMD_SYNTH_SPEC_H

#include <stdint.h>

#if defined(__HIPCC__)
#define SYN_HD __host__ __device__ static inline
#else
#define SYN_HD static inline
#endif

#define SYN_MAX_OBJECTS 4096

/* lowbias32 integer hash */
SYN_HD uint32_t syn_hash(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

SYN_HD int syn_lattice(int32_t ix, int32_t iy, uint32_t seed)
{
    return (int)(syn_hash(((uint32_t)ix * 0x9E3779B1U) ^ syn_hash((uint32_t)iy ^ seed)) & 255U);
}

/* bilinear value noise; cell = 2^k px; coordinates in Q8 (arithmetic >> floors) */
SYN_HD int syn_vnoise(int32_t uq8, int32_t vq8, int k, uint32_t seed)
{
    int32_t cx = uq8 >> (8 + k), cy = vq8 >> (8 + k);
    int fx = (uq8 >> k) & 255, fy = (vq8 >> k) & 255;
    int v00 = syn_lattice(cx, cy, seed), v01 = syn_lattice(cx + 1, cy, seed);
    int v10 = syn_lattice(cx, cy + 1, seed), v11 = syn_lattice(cx + 1, cy + 1, seed);
    int top = v00 * (256 - fx) + v01 * fx;
    int bot = v10 * (256 - fx) + v11 * fx;
    return (top * (256 - fy) + bot * fy + 32768) >> 16;
}

SYN_HD int syn_background(int x, int y, uint32_t seed)
{
    int b1 = syn_vnoise(x << 8, y << 8, 4, seed);
    int b2 = syn_vnoise(x << 8, y << 8, 2, seed ^ 0xA511E9B3U);
    return (b1 * 3 + b2) >> 2;
}

/* per-frame quantised pose of one object (all Q16 fixed point) */
typedef struct syn_pose {
    int32_t cx, cy;          /* centre, Q16 px                         */
    int32_t ia, ib, ic, id;  /* inverse map (R(-theta)/s), Q16          */
    int32_t hw, hh;          /* half extents in object space, Q16      */
    int32_t bx0, by0, bx1, by1; /* integer bounding box [x0,x1) (unclipped) */
    uint32_t seed;           /* texture seed                            */
    int32_t bright;          /* brightness offset                       */
} syn_pose;

SYN_HD int syn_object_texel(const syn_pose* p, int x, int y, int* out)
{
    if (x < p->bx0 || x >= p->bx1 || y < p->by0 || y >= p->by1) return 0;
    int64_t dx = ((int64_t)x << 16) - p->cx;
    int64_t dy = ((int64_t)y << 16) - p->cy;
    int64_t u = ((int64_t)p->ia * dx + (int64_t)p->ib * dy) >> 16;
    int64_t v = ((int64_t)p->ic * dx + (int64_t)p->id * dy) >> 16;
    if (u < -(int64_t)p->hw || u >= (int64_t)p->hw || v < -(int64_t)p->hh || v >= (int64_t)p->hh)
        return 0;
    int32_t uq8 = (int32_t)((u + p->hw) >> 8), vq8 = (int32_t)((v + p->hh) >> 8);
    int t1 = syn_vnoise(uq8, vq8, 2, p->seed);
    int t2 = syn_vnoise(uq8, vq8, 3, p->seed ^ 0x5BD1E995U);
    int val = ((t1 * 5 + t2 * 3) >> 3) + p->bright;
    *out = val < 0 ? 0 : (val > 255 ? 255 : val);
    return 1;
}

/* full pixel: background, then objects in order (last hit wins) */
SYN_HD uint8_t syn_pixel(const syn_pose* poses, int nobj, int x, int y, uint32_t bgseed)
{
    int v = syn_background(x, y, bgseed);
    for (int o = 0; o < nobj; ++o) {
        int t;
        if (syn_object_texel(&poses[o], x, y, &t)) v = t;
    }
    return (uint8_t)v;
}

/* ---------------- host-side pose model (IEEE double, no libm) ---------------- */

typedef struct syn_object {
    int32_t w, h;
    double cx0, cy0, vx, vy;
    double omega;        /* rad / frame */
    double sphase, srate;/* triangle-wave scale phase / rate (cycles per frame) */
    uint32_t tex_seed;
    int32_t bright;
} syn_object;

static inline double syn_floor(double x)
{
    double t = (double)(int64_t)x;
    return (t > x) ? t - 1.0 : t;
}

/* sin / cos by range reduction to [-pi, pi] and a 24-term Taylor series */
static inline void syn_sincos(double a, double* s, double* c)
{
    const double TWO_PI = 6.283185307179586476925286766559;
    const double PI = 3.1415926535897932384626433832795;
    double k = syn_floor((a + PI) / TWO_PI);
    double x = a - k * TWO_PI;
    double x2 = x * x;
    double ts = x, tc = 1.0, ss = x, cc = 1.0;
    for (int n = 1; n <= 12; ++n) {
        ts = -ts * x2 / (double)((2 * n) * (2 * n + 1));
        tc = -tc * x2 / (double)((2 * n - 1) * (2 * n));
        ss += ts;
        cc += tc;
    }
    *s = ss;
    *c = cc;
}

static inline double syn_unit(uint32_t* state)
{
    *state = syn_hash(*state + 0x9E3779B9U);
    return (double)(*state >> 8) / 16777216.0;
}

static inline void syn_make_objects(uint32_t seed, int W, int H, int nobj, syn_object* objs)
{
    uint32_t st = syn_hash(seed ^ 0x1234567U);
    for (int o = 0; o < nobj; ++o) {
        syn_object* ob = &objs[o];
        ob->w = 64 + (int)(syn_unit(&st) * 137.0);
        ob->h = 64 + (int)(syn_unit(&st) * 137.0);
        ob->cx0 = 32.0 + syn_unit(&st) * (double)(W - 64);
        ob->cy0 = 32.0 + syn_unit(&st) * (double)(H - 64);
        ob->vx = (syn_unit(&st) * 2.0 - 1.0) * 3.0;
        ob->vy = (syn_unit(&st) * 2.0 - 1.0) * 3.0;
        ob->omega = (syn_unit(&st) * 2.0 - 1.0) * 0.017453292519943295;
        ob->sphase = syn_unit(&st);
        ob->srate = 0.002 + syn_unit(&st) * 0.003;
        ob->tex_seed = syn_hash(st ^ (uint32_t)o);
        ob->bright = (int)(syn_unit(&st) * 64.0) - 32;
    }
}

static inline double syn_bounce(double p0, double v, int t, double lo, double hi)
{
    double L = hi - lo;
    double p = p0 - lo + v * (double)t;
    double q = p - syn_floor(p / (2.0 * L)) * (2.0 * L);
    if (q > L) q = 2.0 * L - q;
    return lo + q;
}

static inline int32_t syn_q16(double x)
{
    return (int32_t)syn_floor(x * 65536.0 + 0.5);
}

/* pose of object `ob` at frame t on a W x H canvas */
static inline void syn_pose_at(const syn_object* ob, int W, int H, int t, syn_pose* p)
{
    double cx = syn_bounce(ob->cx0, ob->vx, t, 32.0, (double)(W - 32));
    double cy = syn_bounce(ob->cy0, ob->vy, t, 32.0, (double)(H - 32));
    double u = ob->sphase + ob->srate * (double)t;
    double fr = u - syn_floor(u);
    double tri = 1.0 - 4.0 * (fr < 0.5 ? 0.5 - fr : fr - 0.5); /* in [-1, 1] */
    double s = 1.0 + 0.15 * tri;
    double sn, cs;
    syn_sincos(ob->omega * (double)t, &sn, &cs);
    p->cx = syn_q16(cx);
    p->cy = syn_q16(cy);
    p->ia = syn_q16(cs / s);
    p->ib = syn_q16(sn / s);
    p->ic = syn_q16(-sn / s);
    p->id = syn_q16(cs / s);
    p->hw = ob->w << 15;
    p->hh = ob->h << 15;
    /* forward-mapped corners -> integer bounding box */
    double hw = 0.5 * ob->w * s, hh = 0.5 * ob->h * s;
    double ex = (cs < 0 ? -cs : cs) * hw + (sn < 0 ? -sn : sn) * hh;
    double ey = (sn < 0 ? -sn : sn) * hw + (cs < 0 ? -cs : cs) * hh;
    p->bx0 = (int32_t)syn_floor(cx - ex) - 1;
    p->by0 = (int32_t)syn_floor(cy - ey) - 1;
    p->bx1 = (int32_t)syn_floor(cx + ex) + 2;
    p->by1 = (int32_t)syn_floor(cy + ey) + 2;
    p->seed = ob->tex_seed;
    p->bright = ob->bright;
}

/* ground-truth detection box, clipped to the canvas: returns 0 if empty */
static inline int syn_gt_box(const syn_pose* p, int W, int H, int32_t box[4])
{
    int32_t x0 = p->bx0 + 1, y0 = p->by0 + 1, x1 = p->bx1 - 1, y1 = p->by1 - 1;
    if (x0 < 0) x0 = 0;
    if (y0 < 0) y0 = 0;
    if (x1 > W) x1 = W;
    if (y1 > H) y1 = H;
    if (x1 <= x0 || y1 <= y0) return 0;
    box[0] = x0; box[1] = y0; box[2] = x1 - x0; box[3] = y1 - y0;
    return 1;
}

#endif /* OPENCV_AMD_SYNTH_SPEC_H */
