/*
 * klt_oracle.h — CPU restatement of the reference's KLT hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the parity tests, smoke() and
 * bench.py's cpu_baseline leg compare the HIP path against.  The product path
 * (opencv_amd/) never links, imports or calls anything under oracle/.
 *
 * Parity status: the reference (OpenCV 3.4.7 fork) cannot be compiled from a
 * few of its own source files (core's headers need the CMake-generated
 * opencv2/opencv_modules.hpp / cvconfig.h), and its golden data for this path
 * lives in the non-vendored opencv_extra.  The restatement below is therefore
 * pinned only by the reference's in-tree known-answer checks
 * (modules/imgproc/test/test_filter.cpp:2298-2304) and by the reference tests'
 * own acceptance criteria, restated in tests/ — i.e. "parity unpinned" against
 * reference-produced vectors.
 *
 * Each function cites the reference file:line whose behaviour it restates.
 */
#ifndef TBD_KLT_ORACLE_H
#define TBD_KLT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A padded u8 plane: interior pixel (x,y) lives at
 * data[(y+pad)*pitch + x + pad]; the border holds BORDER_REFLECT_101 values. */
typedef struct orc_plane {
    uint8_t* data;
    int w, h, pitch, pad;
    int cn;          /* channels, interleaved (0 reads as 1) */
} orc_plane;

#define ORC_MAX_LEVELS 8

typedef struct orc_pyr {
    int nlevels;               /* maxLevel + 1 */
    orc_plane lv[ORC_MAX_LEVELS];
} orc_pyr;

/* accumulation order for the float sums of LKTrackerInvoker */
enum { ORC_ACCUM_SSE2 = 0, ORC_ACCUM_EXACT = 1 };

/* flags (video/include/opencv2/video/tracking.hpp:56-57) */
#define ORC_OPTFLOW_USE_INITIAL_FLOW 4
#define ORC_OPTFLOW_LK_GET_MIN_EIGENVALS 8

int  orc_reflect101(int p, int len);

/* cv::buildOpticalFlowPyramid without derivatives (lkpyramid.cpp:697-793);
 * returns the number of levels built (maxLevel actually used + 1). */
int  orc_build_pyramid(const uint8_t* img, int w, int h, int pitch,
                       int winW, int winH, int maxLevel, int pad, orc_pyr* pyr);
void orc_free_pyramid(orc_pyr* pyr);
/* the same for cn-channel interleaved u8 images (any cn; the CPU path's) */
int  orc_build_pyramid_cn(const uint8_t* img, int w, int h, int pitch, int cn,
                          int winW, int winH, int maxLevel, int pad, orc_pyr* pyr);

/* pyrDown_<FixPtCast<uchar,8>> of one isolated plane (imgproc/src/pyramids.cpp:722-857) */
void orc_pyr_down(const uint8_t* src, int sw, int sh, int spitch,
                  uint8_t* dst, int dw, int dh, int dpitch);
void orc_pyr_down_cn(const uint8_t* src, int sw, int sh, int spitch, int cn,
                     uint8_t* dst, int dw, int dh, int dpitch);

/* calcSharrDeriv (lkpyramid.cpp:55-144): dst is (h x w x 2) int16, interleaved */
void orc_scharr(const uint8_t* src, int w, int h, int pitch, int16_t* dst, int dstride);
/* cn channels: dst (h x w x 2cn) int16, per pixel (Ix_c, Iy_c) for c = 0..cn-1 */
void orc_scharr_cn(const uint8_t* src, int w, int h, int pitch, int cn, int16_t* dst, int dstride);

typedef struct orc_lk_params {
    int winW, winH;
    int maxLevel;        /* requested; clamped to the pyramids' depth */
    int maxCount;        /* TermCriteria COUNT (clamped to [0,100])   */
    double epsilon;      /* TermCriteria EPS  (clamped to [0,10])     */
    int flags;
    float minEigThreshold;
    int accum;           /* ORC_ACCUM_SSE2 | ORC_ACCUM_EXACT          */
    int nthreads;
} orc_lk_params;

/* cv::calcOpticalFlowPyrLK on prebuilt pyramids (lkpyramid.cpp:1207-1377 +
 * LKTrackerInvoker::operator() :178-695).  iters (optional) receives, per
 * point, the Newton iterations executed summed over levels. */
int  orc_lk(const orc_pyr* prev, const orc_pyr* next,
            const float* prevPts, float* nextPts, uint8_t* status, float* err,
            int npoints, const orc_lk_params* prm, int32_t* iters);
/* the same, and per point (gate, optional) the smallest relative margin of
 * any minEig / determinant / bounds gate it evaluated at any level:
 * |v - thr| / |thr| (test diagnostics for SURVEY.md §8(c)) */
int  orc_lk_gate(const orc_pyr* prev, const orc_pyr* next,
                 const float* prevPts, float* nextPts, uint8_t* status, float* err,
                 int npoints, const orc_lk_params* prm, int32_t* iters, float* gate);

/* synthetic sequence (opencv_amd/csrc/synth_spec.h) rendered on the CPU
 * (out NULL: the ground-truth boxes only) */
int  orc_synth_frames(uint32_t seed, int W, int H, int nobj, int t0, int nframes,
                      uint8_t* out, int pitch, int32_t* gt_boxes /* nframes*nobj*5 or NULL */);

/* wall-clock helper for the CPU baseline */
double orc_now(void);

#ifdef __cplusplus
}
#endif
#endif

#ifdef __cplusplus
extern "C" {
#endif
/* cv::goodFeaturesToTrack(image, corners, maxCorners, qualityLevel, minDistance,
 * noArray(), blockSize=3, gradientSize=3, useHarris=false) on an isolated u8
 * image (imgproc/src/featureselect.cpp:361-516, corner.cpp:52-101,237-326).
 * Returns the corner count; corners: maxCorners x float2 (x, y). */
int orc_gftt(const uint8_t* img, int w, int h, int pitch, int maxCorners, double qualityLevel,
             double minDistance, float* corners);
/* cornerMinEigenVal(blockSize=3, ksize=3, BORDER_REFLECT_101) -> eig (w x h float) */
void orc_min_eig(const uint8_t* img, int w, int h, int pitch, float* eig);
void orc_corner_response(const uint8_t* img, int w, int h, int pitch, int block, int harris, double hk, float* out);
int orc_gftt_ex(const uint8_t* img, int w, int h, int pitch, int maxCorners, double qualityLevel,
                double minDistance, int block, int harris, double hk, float* corners);
#ifdef __cplusplus
}
#endif

/* ---- warpAffine (oracle/warp_oracle.c) ---- */
#ifdef __cplusplus
extern "C" {
#endif
/* border modes / flags: same values as the reference (core/include/opencv2/core/base.hpp,
 * imgproc/include/opencv2/imgproc.hpp) */
#define ORC_BORDER_CONSTANT 0
#define ORC_BORDER_REPLICATE 1
#define ORC_BORDER_REFLECT 2
#define ORC_BORDER_WRAP 3
#define ORC_BORDER_REFLECT_101 4
#define ORC_BORDER_TRANSPARENT 5
#define ORC_WARP_INVERSE_MAP 16
int orc_border_interpolate(int p, int len, int border);
void orc_invert_affine(const double* M, double* out);
/* cv::warpAffine of a CV_8UC1 image; flags = INTER_NEAREST(0) / INTER_LINEAR(1) /
 * INTER_AREA(3, as LINEAR) | WARP_INVERSE_MAP(16); returns -1 for other modes */
void orc_bicubic_tab(int ay, int ax, short* w);
int orc_warp_affine_u8(const uint8_t* src, int sw, int sh, int spitch, uint8_t* dst, int dw, int dh, int dpitch,
                       const double* M, int flags, int border, int bval);
#ifdef __cplusplus
}
#endif
