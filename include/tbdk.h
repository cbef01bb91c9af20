/*
 * tbdk.h — C ABI of the MI355X-native TBD/KLT hot path (libtbdk.so).
 *
 * This is the drop-in boundary for the per-frame tracking-by-detection path of
 * the reference (tkortz/opencv, OpenCV 3.4.7 fork).  Each entry point names the
 * reference interface it replaces.  Conventions:
 *   - plain pointers and sizes; every image/point buffer is DEVICE memory owned
 *     by the caller (hipMalloc / torch), except where a parameter says "host";
 *   - every call is asynchronous on the given HIP stream (passed as void*,
 *     NULL = the legacy default stream); no hidden host sync, no device
 *     globals, so contexts on different devices/threads are independent;
 *   - every call returns an int status (TBDK_OK or a negative TBDK_E*);
 *     n == 0 is a no-op returning TBDK_OK (reference: pyrlk.cpp:221-227
 *     releases the outputs on empty input).
 */
#ifndef TBDK_H
#define TBDK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TBDK_OK 0
#define TBDK_EINVAL (-1)   /* bad argument (reference: CV_Assert -> cv::Exception)   */
#define TBDK_EHIP (-2)     /* HIP runtime error (reference: cudaSafeCall)             */
#define TBDK_ENOMEM (-3)   /* device allocation failed                                */
#define TBDK_ENODEV (-4)   /* no such device / no GPU (reference: throw_no_cuda())    */

#define TBDK_MAX_LEVELS 8

/* pixel depths of a pyramid (cv::Mat depth codes: CV_8U = 0; 7 is OpenCV 4's CV_16F) */
#define TBDK_DEPTH_8U 0
#define TBDK_DEPTH_16F 7
#define TBDK_DEPTH_32F 5

/* flags, same values as the reference (video/include/opencv2/video/tracking.hpp:56-57) */
#define TBDK_OPTFLOW_USE_INITIAL_FLOW 4
#define TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS 8

typedef struct tbdk_ctx tbdk_ctx;

/* One pyramid level in device memory.  Interior pixel (x, y) is at
 * data[(y + pad) * pitch + x + pad]; the `pad`-wide frame around it holds
 * BORDER_REFLECT_101 values, as cv::buildOpticalFlowPyramid's padded levels do
 * (video/src/lkpyramid.cpp:726-762). */
typedef struct tbdk_level {
    uint8_t* data;
    int32_t width, height, pitch, pad;
} tbdk_level;

/* A pyramid, the layout of cv::buildOpticalFlowPyramid (lkpyramid.cpp:697-793):
 * lv[i] are the u8 levels, each with a reflect-101 frame of `pad` pixels; with
 * derivatives (tbdk_pyr_create, withDerivatives=true, lkpyramid.cpp:765-780)
 * dv[i] are the Scharr planes of calcSharrDeriv (lkpyramid.cpp:55-144), CV_16SC2
 * interleaved (Ix, Iy) per pixel (4 bytes; pitch in bytes) with a zero
 * (BORDER_CONSTANT) frame of `pad` pixels; without (tbdk_pyr_create_levels)
 * dv[i].data is NULL and tbdk_lk_sparse derives the window's Scharr values
 * itself (same results).  A tbdk_pyr must come from tbdk_pyr_create* (which
 * fill every field); callers never fill one themselves.
 * ABI 2 (TBDK_ABI_VERSION): `depth` and `flags` follow `storage`, so every
 * field before them has its offset of the original (depth-less) layout. */
typedef struct tbdk_pyr {
    int32_t nlevels;                 /* levels built = maxLevel used + 1 */
    int32_t win_w, win_h;            /* window the level count was derived for */
    tbdk_level lv[TBDK_MAX_LEVELS];
    tbdk_level dv[TBDK_MAX_LEVELS];
    void* storage;                   /* owned by the library; free with tbdk_pyr_destroy */
    int32_t depth;                   /* TBDK_DEPTH_8U (tbdk_pyr_create*), TBDK_DEPTH_16F
                                        (tbdk_pyr_create_f16: fp16 levels, fp16 (Ix, Iy)
                                        derivative pairs) or TBDK_DEPTH_32F
                                        (tbdk_pyr_create_f32: fp32 levels and pairs) */
    int32_t flags;                   /* TBDK_PYR_NO_DERIVS: levels only */
    int32_t cn;                      /* channels per pixel, interleaved (1; 2..4 from
                                        tbdk_pyr_create_cn); level rows hold
                                        (width + 2*pad)*cn bytes, derivative rows
                                        (Ix_c, Iy_c) pairs for c = 0..cn-1 */
} tbdk_pyr;

#define TBDK_ABI_VERSION 2
#define TBDK_PYR_NO_DERIVS 1

/* cv::TermCriteria(COUNT+EPS, maxCount, epsilon) + flags + minEigThreshold of
 * cv::calcOpticalFlowPyrLK (video/include/opencv2/video/tracking.hpp:178-183) */
typedef struct tbdk_lk_params {
    int32_t win_w, win_h;            /* default 21, 21 */
    int32_t max_level;               /* default 3 (clamped to the pyramids) */
    int32_t max_count;               /* default 30, clamped to [0, 100] */
    double epsilon;                  /* default 0.01, clamped to [0, 10] then squared */
    int32_t flags;                   /* TBDK_OPTFLOW_* */
    float min_eig_threshold;         /* default 1e-4 */
    int32_t impl;                    /* 0 auto; 1 register-strip kernel; 2 generic LDS kernel;
                                        3 several points per wave (all bit-identical) */
} tbdk_lk_params;

/* ---- context ------------------------------------------------------------ */

/* Creates a context bound to HIP device `device` (one per thread x device).
 * It also creates the library's side streams (Farneback's level prep, the HOG
 * level lanes): HIP maps streams onto a few hardware queues in creation order,
 * so creating the context before the caller's own streams keeps those side
 * streams off the caller's queue (HOG "Side streams"). */
int tbdk_ctx_create(int device, tbdk_ctx** out);
int tbdk_ctx_destroy(tbdk_ctx* ctx);
/* Context options (test and tuning knobs; TBDK_EINVAL for unknown names):
 *   "gftt_eig_redo" (0/1): treat every row-segment boundary of the GFTT
 *       eigenvalue strips as a fresh-start mismatch, forcing the re-walk
 *       rounds taken when a segment's fresh start differs from the
 *       reference's running box-filter sum (results equal).
 *   "pyr_fuse" (0/1/2, default 1): tbdk_pyr_build of a u8 pyramid: 1
 *       computes level 0's padded copy and level 1 in one launch, then one
 *       launch per level; 2 computes levels 0, 1 and 2 in one tiled launch (the
 *       frame read once through LDS; pyramids whose level pads exceed size - 2
 *       take 1; measured slower, kept for A/B runs); 0: one launch per level
 *       (results equal).  fp16 / fp32 pyramids: >= 1 builds L levels in L
 *       role-split launches (level 0's copy, level 1 and level 0's Scharr
 *       plane from the frame, then level i and plane i-1 from level i-1);
 *       0 takes one launch per level and one for every plane (results equal).
 *   "pyr_xcd" (0/1, default 1): the u8 two-role and fp16 / fp32 role-split
 *       pyramid launches deal each role's blocks to the 8 XCDs in contiguous
 *       row bands, so rows a role reads twice share one XCD's L2 (results equal).
 *   "pyr_rows" (1/2/4, default 1): rows per thread of the u8 two-role
 *       launch (pyr_fuse 1: level 0's 16-byte copies of that many rows, level
 *       1 in row pairs sharing their 7 frame rows when > 1) and of the fp16 /
 *       fp32 role-split launches (copies and Scharr planes that many rows,
 *       levels in pairs at most); more than 1 measured slower (fewer waves
 *       to hide the loads' latency), kept for A/B runs (results equal).
 *   "lk_scharr_fly" (0/1, default 0): the several-points-per-wave PyrLK
 *       kernel derives the window's Scharr values from the u8 level even when
 *       the pyramid has derivative planes (it always does without them;
 *       results equal).
 *   "lk_solo" (0..100, default 4): the several-points-per-wave PyrLK kernel
 *       runs a wave's last stepping point on all the wave's lanes (its window
 *       rows split over the lane groups) once the wave's other points have
 *       stopped, from Newton step lk_solo of the level on (0: never; padded
 *       levels only; results equal).
 *   "lk_impl" (0..3): the PyrLK kernel taken when tbdk_lk_params.impl is 0
 *       (the TBD loop's setting): 0 auto, else as tbdk_lk_params.impl
 *       (results equal).
 *   "hog_block_tiled" (0..2, default 1): HOG block histograms of 2x2-cell,
 *       9-bin geometries by the LDS-tiled kernel, its histograms in LDS (1)
 *       or in registers (2); 0 forces the per-cell kernel of every other
 *       geometry (results equal).
 *   "hog_level_streams" (1..4, default 3): tbdk_hog_detect_multiscale runs
 *       the levels' resize/gradient/block chains on this many streams (the
 *       caller's and internal ones, joined back before the window pass;
 *       results equal).
 *   "hog_window_tiled" (0/1, default 1): tbdk_hog_detect_multiscale's window
 *       pass stages each row of 16 windows' blocks and the detector in LDS
 *       (36-float blocks); 0 reads them per window from L2 (results equal).
 *   "fb_prep_ahead" (0/1, default 1): tbdk_farneback computes every level's
 *       images and polynomial expansions on an internal stream, coarse to
 *       fine, while the coarser levels iterate on the caller's stream
 *       (results equal). */
int tbdk_ctx_set_option(tbdk_ctx* ctx, const char* name, int64_t value);
/*   "tbd_early_gftt" (0/1/2, default 2): the TBD loop runs GFTT over the
 *       detections that will start new tracks at the start of the step, off
 *       the critical path; 2 also over the box each existing track would get
 *       on a re-detection frame from the detection overlapping it most (a
 *       guess: boxes the tracker step does not confirm take the regular GFTT;
 *       results equal).
 *   "tbd_spec_lookahead" (0/1, default 1): with a look-ahead frame, the TBD
 *       loop starts the next frame's PyrLK of the point sets that stay
 *       unchanged unless their track is deleted before the host tracker step
 *       (results equal).
 *   "tbd_zero_copy" (0/1, default 1; taken by tbdk_tbd_create): the TBD loop's
 *       kernels read their host tables from, and the fit writes its results
 *       to, coherent pinned host memory directly instead of through copies
 *       (results equal).
 *   "tbd_early_la" (0/1/2, default 1): with a look-ahead frame, the TBD loop
 *       tracks this step's early GFTT rows into the next frame right after the
 *       fit (1: on re-detection frames, where no speculative PyrLK runs; 2:
 *       every frame); the next step's refreshed-set PyrLK skips them (results
 *       equal).
 *   "tbd_fit_flag" (0/1, default 1; taken by tbdk_tbd_create, with zero copy):
 *       the fit kernel's last wave publishes the frame's results by a
 *       system-scope flag in pinned memory that the host polls, instead of an
 *       event recorded behind the fit (whose marker held the next frame's
 *       pyramid back; results equal).
 *   "tbd_early_order" (0/1/2, default 0): where a step launches its early
 *       GFTT (and, tbd_gftt_ahead, the next frame's): 0 first, 1 after the
 *       critical refreshed-set PyrLK (its host setup no longer delays that
 *       launch, and the PyrLK waves are dispatched ahead of the GFTT's), 2 after
 *       the fit and the next frame's pyramid, before the host waits for the fit
 *       (results equal).
 *   "tbd_early_prio" (0/1, default 0; taken by tbdk_tbd_create): the early
 *       GFTT's stream at the lowest (0) or highest (1) priority (results equal).
 *   "tbd_pyr_derivs" (0/1, default 0; taken by tbdk_tbd_create): the loop's
 *       pyramids carry Scharr derivative planes and PyrLK reads them instead of
 *       deriving the window's values (results equal; A/B runs).
 *   "lk_seg_inline", "tbd_fit_inline", "gftt_inline" (0/1, default 1): the TBD
 *       loop's PyrLK segment lists (up to 256), the fit's per-track table (up
 *       to 256 tracks) and GFTT ROI tables (up to 128 ROIs, also in
 *       tbdk_gftt_rois) travel in the kernel arguments instead of being read
 *       from the staged tables (with zero copy: pinned host memory, one
 *       host-link round trip per first read); larger tables are read from
 *       memory (results equal).
 *   "tbd_fit_wgpub" (0/1, default 1): with the fit flag, each fit workgroup
 *       publishes its tracks' results with one system-scope release (wave 0
 *       stores them), not one release per wave (results equal).
 *   "tbd_la_pyr_side" (0/1/2, default 2): where the TBD loop builds the
 *       look-ahead pyramid: 0 on the caller's stream behind the fit; 1 on its
 *       look-ahead stream behind the step's PyrLK launches, beside the fit; 2 on
 *       the look-ahead stream right after the step's critical PyrLK launch,
 *       behind only the caller's work before the step (the loop keeps three
 *       pyramids, so the one it overwrites is two frames old and no longer
 *       read). The look-ahead PyrLK that follows it needs no cross-stream edge
 *       (results equal).
 *   "tbd_post_direct" (0/1, default 1): after a step that runs no post-tracker
 *       GFTT, the next step's refreshed-set PyrLK waits for the early GFTT's
 *       completion directly rather than through the post-tracker stream's
 *       event (results equal).
 *   "tbd_la_defer" (0/1, default 0): the look-ahead PyrLK of the unchanged
 *       sets is launched by the next step right after its critical PyrLK
 *       instead of at the end of its own step (results equal; A/B runs).
 *   "gftt_compact" (0/1, default 1): GFTT with quality <= 1 (blockSize 3,
 *       min-eigenvalue) writes no eigenvalue plane, only its local maxima's
 *       values per strip row (corner lists equal; quality > 1, Harris and other
 *       block sizes keep the plane).
 *   "tbd_gftt_ahead" (0/1, default 1): inside tbdk_tbd_run each step also
 *       launches the NEXT frame's early GFTT over its new-track ROIs (that
 *       frame's detections beyond the bounds filter), over the caller's next
 *       frame, so the refreshed-set PyrLK of the step after it does not wait for
 *       a GFTT launched only one step earlier; the step of that frame launches
 *       just the ROIs it misses (re-detection guesses).  The caller's stream
 *       waits for that work before the call returns (results equal).
 *   "tbd_ahead_at" (0/1/2, default 0): where a step launches that ahead GFTT:
 *       0 with its own early GFTT, 1 after its critical PyrLK, 2 just before
 *       the host waits for the fit (never before the step's own early GFTT;
 *       results equal).
 *   "tbd_borrow_l0" (0/1, default 0): inside tbdk_tbd_run the loop's pyramids
 *       take the caller's frames as level 0 (no padded copy; PyrLK reads
 *       windows across a frame's edge by reflect-101 coordinates, the values
 *       the copy holds); when the call returns the last frame's level 0 has
 *       been copied into the loop's own buffer and the caller's stream waits
 *       for the last read of a frame, so the frames may be reused once that
 *       stream is synchronised (results equal; PyrLK measured slower reading
 *       the frames than the loop's reused buffers, so off by default).
 *       tbdk_tbd_step / _step_ahead / _run_host always copy.
 *   "tbd_fit_gate" (0/1, default 1): the TBD loop's host waits (polling) for
 *       the look-ahead PyrLK's completion event and then launches the fit on
 *       the step's stream behind the step's own PyrLK, instead of enqueuing a
 *       cross-stream wait in front of the fit (results equal; A/B runs).
 *   "tbd_async_la" (0/1, default 0; taken by tbdk_tbd_create): the TBD loop's
 *       look-ahead PyrLK launches are issued by a worker thread of the loop
 *       (one more host thread per loop, spinning between frames; results equal;
 *       A/B runs).
 *   "timing_every" (>= 1, default 1): HIP events on a pseudo-random 1/N of the
 *       launches of each kernel selected for timing: launch i (counted per
 *       kernel name from tbdk_timing_enable) is timed iff splitmix64(i) % N == 0
 *       (see tbdk_timing_calls). */

/* device ordinal of the context */
int tbdk_ctx_device(const tbdk_ctx* ctx);

/* Per-kernel timing with HIP events recorded on the launch stream.
 * enable != 0 starts recording (clears previous records). */
int tbdk_timing_enable(tbdk_ctx* ctx, int enable);
/* Synchronises the recorded events and returns, for kernel `name`
 * ("pyr_build", "lk_sparse", "lk_dense" (tbdk_lk_dense), ...), the number of launches and the summed
 * device milliseconds. */
int tbdk_timing_query(tbdk_ctx* ctx, const char* name, int64_t* launches, double* total_ms);
/* Restrict recording to the comma-separated kernel names in `names` (NULL or
 * "" = all).  Each timed launch costs two event records on the host. */
int tbdk_timing_select(tbdk_ctx* ctx, const char* names);
/* Selected launches of kernel `name` since tbdk_timing_enable, timed or not:
 * with the ctx option "timing_every" = N only a 1/N sample of them records events
 * (tbdk_timing_query counts those), to keep the event records' host cost out
 * of a measured loop. */
int tbdk_timing_calls(tbdk_ctx* ctx, const char* name, int64_t* calls);

/* ---- pyramids ------------------------------------------------------------ */

/* Allocates a padded pyramid for width x height u8 frames.  The level count
 * follows cv::buildOpticalFlowPyramid's stop rule for window (win_w, win_h)
 * (video/src/lkpyramid.cpp:782-787).  Not for the hot path (hipMalloc). */
int tbdk_pyr_create(tbdk_ctx* ctx, int width, int height, int max_level,
                    int win_w, int win_h, tbdk_pyr* pyr);
int tbdk_pyr_destroy(tbdk_ctx* ctx, tbdk_pyr* pyr);

/* Builds every level of `pyr` (and its derivative planes) from the device u8
 * image `img` (row pitch in bytes).  Replaces cv::buildOpticalFlowPyramid (video/src/lkpyramid.cpp:697)
 * and, level by level, cv::cuda::pyrDown
 * (modules/cudawarping/include/opencv2/cudawarping.hpp:201) — bit-exact with
 * the CPU pyrDown_<FixPtCast<uchar,8>> (imgproc/src/pyramids.cpp:722-857). */
int tbdk_pyr_build(tbdk_ctx* ctx, const uint8_t* img, int pitch, tbdk_pyr* pyr, void* stream);
/* A u8 pyramid without derivative planes (flags TBDK_PYR_NO_DERIVS, dv[i].data
 * NULL): levels only; tbdk_pyr_build writes no Scharr planes (level 0's padded
 * copy and level 1 in one launch, then one launch per level).  PyrLK on it
 * derives the window's Scharr values in the kernel (identical results); the
 * TBD loop's pyramids are of this kind. */
int tbdk_pyr_create_levels(tbdk_ctx* ctx, int width, int height, int max_level, int win_w, int win_h,
                           tbdk_pyr* pyr);
/* Levels 1.. of a levels-only u8 pyramid (tbdk_pyr_create_levels) from the
 * device frame `img`, which becomes level 0 itself: no padded copy, as the
 * pyramid of cv::cuda::SparsePyrLKOpticalFlow, whose level 0 is the input
 * GpuMat (cudaoptflow/src/pyrlk.cpp:144-145).  tbdk_lk_sparse (its
 * several-points-per-wave kernel: impl 0 or 3, 1 channel, window width <= 31)
 * reads that level with buildOpticalFlowPyramid's reflect-101 border
 * (lkpyramid.cpp:726-740) by coordinates, with the same results as the padded
 * copy; other kernels return TBDK_EINVAL.  The frame must stay valid and
 * unchanged while the pyramid is read; the next tbdk_pyr_build gives the
 * pyramid its own level 0 again.  Levels are as tbdk_pyr_build's, bit for bit. */
int tbdk_pyr_build_borrowed(tbdk_ctx* ctx, const uint8_t* img, int pitch, tbdk_pyr* pyr, void* stream);

/* Multi-channel frames (cv::cuda::SparsePyrLKOpticalFlow takes 1, 3 or 4
 * channels, cudaoptflow/src/pyrlk.cpp:140-142,197-205; the CPU
 * calcOpticalFlowPyrLK any count, lkpyramid.cpp:55-144,178-695): a pyramid of
 * interleaved cn-channel u8 levels (cn = 1..4) with CV_16SC(2cn) derivative
 * planes.  tbdk_pyr_build fills it from an interleaved frame (pitch >=
 * width*cn); tbdk_lk_sparse on two such pyramids runs LKTrackerInvoker over
 * winW*cn elements per window row (klt_cn.hip). */
int tbdk_pyr_create_cn(tbdk_ctx* ctx, int width, int height, int cn, int max_level, int win_w, int win_h,
                       tbdk_pyr* pyr);

/* The fp16 pixel path (no reference implementation: the
 * reference's CPU PyrLK takes 8-bit levels only, lkpyramid.cpp:1272-1276, and
 * its CUDA class reads CV_32F through textures, cudaoptflow/src/pyrlk.cpp:197-205).
 * A pyramid of fp16 levels (2 bytes per pixel) and fp16 (Ix, Iy) derivative
 * pairs (4 bytes per pixel), same padding and level rule as tbdk_pyr_create.
 * tbdk_pyr_build fills it from a u8 frame (converted exactly);
 * tbdk_pyr_build_f16 from an fp16 frame (pitch in bytes).  Levels follow
 * pyrDown_<FltCast<float,8>> (imgproc/src/pyramids.cpp:722-857) in fp32,
 * rounded to fp16; tbdk_lk_sparse on two such pyramids runs LKTrackerInvoker's
 * algorithm in fp32. */
int tbdk_pyr_create_f16(tbdk_ctx* ctx, int width, int height, int max_level,
                        int win_w, int win_h, tbdk_pyr* pyr);
int tbdk_pyr_build_f16(tbdk_ctx* ctx, const uint16_t* img, int pitch, tbdk_pyr* pyr, void* stream);

/* The fp32 pixel path, for the 16U and 32F frames cv::cuda::SparsePyrLK-
 * OpticalFlow takes (cudaoptflow/src/pyrlk.cpp:189-205; the CPU PyrLK has no
 * such path): the fp16 path's algorithm with fp32 levels (4 B per pixel) and
 * fp32 (Ix, Iy) derivative pairs (8 B per pixel), nothing rounded to fp16.
 * tbdk_pyr_build fills it from a u8 frame, tbdk_pyr_build_u16 from a u16
 * frame, tbdk_pyr_build_f32 from an fp32 frame (every conversion exact;
 * pitches in bytes); tbdk_lk_sparse on two such pyramids (impl 0). */
int tbdk_pyr_create_f32(tbdk_ctx* ctx, int width, int height, int max_level,
                        int win_w, int win_h, tbdk_pyr* pyr);
int tbdk_pyr_build_u16(tbdk_ctx* ctx, const uint16_t* img, int pitch, tbdk_pyr* pyr, void* stream);
int tbdk_pyr_build_f32(tbdk_ctx* ctx, const float* img, int pitch, tbdk_pyr* pyr, void* stream);
/* The fp32 pixel path on cn = 2..4 interleaved channels: CV_16UC3/C4 and
 * CV_32FC3/C4 frames of cv::cuda::SparsePyrLKOpticalFlow (cudaoptflow/src/
 * pyrlk.cpp:197-205), computed as the CPU path handles channels
 * (lkpyramid.cpp:55-144, 178-695: windows of win_w * cn values, G and b over
 * all of them).  Levels hold cn fp32 values per pixel, the derivative planes
 * an (Ix, Iy) fp32 pair per value; tbdk_pyr_build / _build_u16 / _build_f32
 * take frames of cn interleaved u8 / u16 / fp32 values per pixel;
 * tbdk_lk_sparse (impl 0) tracks on two such pyramids.
 * Semantics are the CPU path's, not the CUDA class's: err is the L1 mean over
 * 32 * win_w * cn * win_h (lkpyramid.cpp:690; pyrlk.cu:555 divides by
 * min(cn, 3) * win_w * win_h instead, and reads 16U frames through normalised
 * [0, 1] textures), and the minEigThreshold gate applies to the raw values (the
 * CUDA class has none).  cn = 2 is accepted here, as buildOpticalFlowPyramid /
 * calcOpticalFlowPyrLK accept it; the typed-frame facades reject it as the
 * CUDA class does (pyrlk.cpp:142,228). */
int tbdk_pyr_create_f32_cn(tbdk_ctx* ctx, int width, int height, int cn, int max_level,
                           int win_w, int win_h, tbdk_pyr* pyr);

/* Synchronous copy of level `level` to host memory (GpuMat::download
 * analogue; not for the hot path).  with_border != 0 copies the padded frame
 * ((height+2*pad) rows of (width+2*pad) pixels), else the interior; rows of
 * width * cn * (1 or 2) bytes by depth (fp16 as raw bits). */
int tbdk_pyr_download(tbdk_ctx* ctx, const tbdk_pyr* pyr, int level, uint8_t* host, int host_pitch,
                      int with_border);
/* Same for the derivative plane of `level` (interior, CV_16SC(2cn) — fp16
 * pairs as raw bits for TBDK_DEPTH_16F — host_pitch in bytes). */
int tbdk_pyr_download_deriv(tbdk_ctx* ctx, const tbdk_pyr* pyr, int level, int16_t* host, int host_pitch);

/* Single-level cv::cuda::pyrDown replacement: dst = pyrDown(src),
 * dst size ((w+1)/2, (h+1)/2), plain (unpadded) device images. */
int tbdk_pyr_down_u8(tbdk_ctx* ctx, const uint8_t* src, int width, int height, int src_pitch,
                     uint8_t* dst, int dst_pitch, void* stream);

/* ---- sparse pyramidal Lucas-Kanade -------------------------------------- */

/* Replaces cv::cuda::SparsePyrLKOpticalFlow::calc
 * (modules/cudaoptflow/include/opencv2/cudaoptflow.hpp:160-180, impl
 * modules/cudaoptflow/src/pyrlk.cpp:326-349) with the numerics of the CPU
 * cv::calcOpticalFlowPyrLK (video/src/lkpyramid.cpp:1207-1377, 178-695).
 *   prev_pts / next_pts : n x float2 (x, y); next_pts is read as the initial
 *                         guess when TBDK_OPTFLOW_USE_INITIAL_FLOW is set
 *   status              : n x u8 (1 = tracked)
 *   err                 : n x f32 or NULL (L1 patch error / 32 at level 0; the
 *                         minimum eigenvalue with LK_GET_MIN_EIGENVALS; 0 where
 *                         status is 0 and the reference leaves it unset)
 *   iters               : n x i32 or NULL (Newton iterations over all levels)
 * All levels run in one launch.  prev and next must have the same depth; on
 * TBDK_DEPTH_16F / TBDK_DEPTH_32F pyramids the fp16 / fp32 pixel path runs
 * (impl must be 0). */
int tbdk_lk_sparse(tbdk_ctx* ctx, const tbdk_pyr* prev, const tbdk_pyr* next,
                   const float* prev_pts, float* next_pts, uint8_t* status, float* err,
                   int32_t* iters, int n, const tbdk_lk_params* params, void* stream);

/* Replaces cv::cuda::DensePyrLKOpticalFlow::calc(I0, I1, flow)
 * (cudaoptflow/include/opencv2/cudaoptflow.hpp:182-208, impl cudaoptflow/src/pyrlk.cpp:238-299)
 * with the CPU calcOpticalFlowPyrLK numerics at every pixel (the point grid
 * (x, y) of level 0 through the tbdk_lk_sparse kernels):
 *   flow   : device CV_32FC2, (nextPt.x - x, nextPt.y - y) per pixel, flow_pitch in bytes
 *   status : device u8 plane (status_pitch bytes) or NULL
 * TBDK_OPTFLOW_USE_INITIAL_FLOW is ignored, as in the reference (dense() never
 * reads the incoming flow); win_w/win_h <= 2 is TBDK_EINVAL (pyrlk.cpp:243).
 * With 8-bit one-channel pyramids carrying derivative planes (pads >= win + 2)
 * and an odd square window of 7..31, the previous pyramid's windows come from
 * per-phase case images (8 B per level position and sub-pixel phase: about one
 * frame of entries per level, ~71 MB at 1080p, win 13, maxLevel 3); otherwise
 * per-pixel scratch (17 B per pixel).  Either buffer is owned by the context
 * and grown on demand (growth frees the old buffer, which waits for the
 * device), so dense calls on one context must not overlap on different
 * streams: order them, or give each stream its own context. */
int tbdk_lk_dense(tbdk_ctx* ctx, const tbdk_pyr* prev, const tbdk_pyr* next, float* flow, int flow_pitch,
                  uint8_t* status, int status_pitch, const tbdk_lk_params* params, void* stream);

/* ---- good features to track over box ROIs --------------------------------- */

typedef struct tbdk_roi {
    int32_t x, y, width, height;     /* must lie inside the image */
} tbdk_roi;

/* cv::cuda::createGoodFeaturesToTrackDetector(CV_8UC1, maxCorners, qualityLevel,
 * minDistance, blockSize=3, useHarrisDetector=false)
 * (modules/cudaimgproc/include/opencv2/cudaimgproc.hpp:603-604) */
typedef struct tbdk_gftt_params {
    int32_t max_corners;             /* > 0 */
    double quality_level;            /* > 0 */
    double min_distance;             /* >= 0 */
    int32_t block_size;              /* 1..63: cornerEigenValsVecs' box filter size */
    int32_t use_harris;              /* 0: cornerMinEigenVal, 1: cornerHarris */
    double harris_k;                 /* Harris k (cudaimgproc.hpp:604 default 0.04) */
} tbdk_gftt_params;

/* Replaces CornersDetector::detect (modules/cudaimgproc/src/gftt.cpp:98-213)
 * applied to each ROI as an isolated image, with the CPU goodFeaturesToTrack
 * semantics (imgproc/src/featureselect.cpp:361-516: max over the ROI,
 * deterministic value/address ordering, greedy min-distance) — all ROIs of a
 * frame in one batch and with no host synchronisation.
 *   img        : device u8 image (width x height, row pitch in bytes)
 *   rois       : HOST array of nroi ROIs (copied during the call)
 *   corners    : device, nroi x max_corners x float2, frame coordinates
 *   counts     : device, nroi int32 (corners found; -1 if a ROI produced more
 *                candidates than the on-chip buffer holds — never truncated)
 * Scratch grows on demand (tbdk_gftt_reserve avoids allocation in the call);
 * it is the context's: calls on one context from different streams must be
 * ordered by the caller (a TBD loop has scratch of its own). */
int tbdk_gftt_rois(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch,
                   const tbdk_roi* rois, int nroi, const tbdk_gftt_params* params,
                   float* corners, int32_t* counts, void* stream);

/* cv::cuda::createMinEigenValCorner(CV_8UC1, blockSize 3, ksize 3,
 * BORDER_REFLECT_101)->compute(src, dst) (cudaimgproc/src/corners.cpp:150-189,
 * cudaimgproc.hpp:564): the minimum-eigenvalue map GFTT selects from, with
 * the CPU cornerMinEigenVal numerics (float Sobel, double box sums).
 * dst: device float plane, dst_pitch in bytes.  Uses the context's GFTT
 * scratch (one launch + one device copy on `stream`). */
int tbdk_corner_min_eig_val(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, float* dst,
                            int dst_pitch, void* stream);
/* The corner response map of any blockSize (ksize 3, BORDER_REFLECT_101):
 * cv::cuda::createMinEigenValCorner(CV_8UC1, blockSize, 3) (harris == 0) and
 * cv::cuda::createHarrisCorner(CV_8UC1, blockSize, 3, k) (harris != 0)
 * (cudaimgproc.hpp:548-566, corners.cpp:150-189), with the CPU
 * cornerMinEigenVal / cornerHarris numerics (corner.cpp:52-152,237-326;
 * Harris in the code paths an AVX x86-64 host runs).
 * block_size 3 without Harris is tbdk_corner_min_eig_val. */
int tbdk_corner_response(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, float* dst,
                         int dst_pitch, int block_size, int harris, double harris_k, void* stream);
int tbdk_gftt_reserve(tbdk_ctx* ctx, int max_rois, int64_t max_total_pixels);

/* ---- KLT box propagation ----------------------------------------------------- */

/* Result of fitting one box's tracked corners (prev -> next). */
typedef struct tbdk_box_fit {
    double m[6];                     /* 2x3 row-major [p -q tx; q p ty] */
    double cx, cy;                   /* the box's integer centre (x + w/2, y + h/2) mapped by m */
    int32_t npoints;                 /* correspondences used (status != 0) */
    int32_t valid;                   /* npoints >= min_points, non-singular, scale in (0.5, 2) */
} tbdk_box_fit;

/* Batched similarity fit per box: the non-full-affine getRTMatrix of
 * cv::estimateRigidTransform (video/src/lkpyramid.cpp:1398-1470) on each box's
 * corner pairs, then the box centre mapped through it — the Track::motionModel
 * (tbd.hpp:111) the TBD loop uses instead of constant velocity.
 *   prev_pts, next_pts : device float2 arrays (all boxes' points, concatenated)
 *   status             : device u8 per point (NULL = all used)
 *   offsets            : device int32, nboxes + 1: box i owns points [offsets[i], offsets[i+1])
 *   boxes              : device tbdk_roi per box
 *   out                : device tbdk_box_fit per box */
int tbdk_box_propagate(tbdk_ctx* ctx, const float* prev_pts, const float* next_pts, const uint8_t* status,
                       const int32_t* offsets, const tbdk_roi* boxes, int nboxes, int min_points,
                       tbdk_box_fit* out, void* stream);

/* ---- affine warp ------------------------------------------------------------ */

/* interpolation flags / border modes: the reference's values
 * (imgproc/include/opencv2/imgproc.hpp INTER_*, WARP_INVERSE_MAP;
 *  core/include/opencv2/core/base.hpp BORDER_*) */
#define TBDK_INTER_NEAREST 0
#define TBDK_INTER_LINEAR 1
#define TBDK_INTER_CUBIC 2            /* remapBicubic, BicubicTab_i (imgwarp.cpp:152-268, 860-958) */
#define TBDK_INTER_AREA 3            /* treated as INTER_LINEAR, as cv::warpAffine does */
#define TBDK_WARP_INVERSE_MAP 16
#define TBDK_BORDER_CONSTANT 0
#define TBDK_BORDER_REPLICATE 1
#define TBDK_BORDER_REFLECT 2
#define TBDK_BORDER_WRAP 3
#define TBDK_BORDER_REFLECT_101 4
#define TBDK_BORDER_TRANSPARENT 5

/* Replaces cv::cuda::warpAffine(src, dst, M, dsize, flags, borderMode, borderValue, stream)
 * (modules/cudawarping/include/opencv2/cudawarping.hpp:126; impl cudawarping/src/warp.cpp:183-320)
 * for CV_8UC1, with the numerics of the CPU cv::warpAffine
 * (imgproc/src/imgwarp.cpp:2572-2682: 10-bit fixed-point map, 5-bit sub-pixel
 * table, 15-bit bilinear weights) — bit-exact with it.
 *   src, dst : device u8 images (row pitch in bytes); dst must not alias src
 *   M        : HOST 2x3 row-major double matrix (dst <- src unless
 *              TBDK_WARP_INVERSE_MAP, then dst -> src, as in the reference)
 *   flags    : TBDK_INTER_NEAREST / LINEAR / CUBIC / AREA | TBDK_WARP_INVERSE_MAP
 *   border   : TBDK_BORDER_*; border_value used by BORDER_CONSTANT */
int tbdk_warp_affine_u8(tbdk_ctx* ctx, const uint8_t* src, int src_width, int src_height, int src_pitch,
                        uint8_t* dst, int dst_width, int dst_height, int dst_pitch, const double* M,
                        int flags, int border, int border_value, void* stream);

/* ---- dense Farneback optical flow ------------------------------------------ */

/* flag value of the reference (video/include/opencv2/video/tracking.hpp:58) */
#define TBDK_OPTFLOW_FARNEBACK_GAUSSIAN 256

/* cv::cuda::FarnebackOpticalFlow::create(numLevels, pyrScale, fastPyramids,
 * winSize, numIters, polyN, polySigma, flags)
 * (modules/cudaoptflow/include/opencv2/cudaoptflow.hpp:210-252) */
typedef struct tbdk_farneback_params {
    int32_t num_levels;              /* 5 */
    double pyr_scale;                /* 0.5; < 1 (CV_Assert, optflowgf.cpp:1113-1114) */
    int32_t fast_pyramids;           /* 0; the CUDA-only pyrDown pyramids are not provided (TBDK_EINVAL) */
    int32_t win_size;                /* 13; 1..21 */
    int32_t num_iters;               /* 10 */
    int32_t poly_n;                  /* 5; 1..15 */
    double poly_sigma;               /* 1.1 */
    int32_t flags;                   /* 0 | TBDK_OPTFLOW_FARNEBACK_GAUSSIAN | TBDK_OPTFLOW_USE_INITIAL_FLOW */
} tbdk_farneback_params;

int tbdk_farneback_default_params(tbdk_farneback_params* p);
/* level count and sizes calc uses for a width x height frame
 * (optflowgf.cpp:1125-1144): *nlevels = levels + 1, sizes[2*k] = width of level k,
 * sizes[2*k+1] = height (sizes may be NULL; else room for 2 * (num_levels + 1)) */
int tbdk_farneback_levels(int width, int height, const tbdk_farneback_params* p, int* nlevels, int32_t* sizes);

/* Replaces cv::cuda::FarnebackOpticalFlow::calc(I0, I1, flow, stream)
 * (cudaoptflow/src/farneback.cpp:164-196) with the numerics of the CPU
 * cv::calcOpticalFlowFarneback (video/src/optflowgf.cpp:1096-1190).
 *   prev, next : device u8 frames (width x height, row pitch in bytes)
 *   flow       : device CV_32FC2 output, interleaved (dx, dy) per pixel,
 *                flow_pitch in bytes (multiple of 8); with
 *                TBDK_OPTFLOW_USE_INITIAL_FLOW also the input: the coarsest
 *                level starts from its INTER_AREA resize times the level scale
 *                (optflowgf.cpp:1151-1157)
 * Scratch (15 float planes of the frame size + the blur buffer) is owned by
 * the context and grown on demand; the call is asynchronous on `stream`. */
int tbdk_farneback(tbdk_ctx* ctx, const uint8_t* prev, const uint8_t* next, int width, int height, int pitch,
                   float* flow, int flow_pitch, const tbdk_farneback_params* params, void* stream);

/* Stage entry points of tbdk_farneback (parity tests):
 * level image = resize(GaussianBlur(float(img), (smooth_size, smooth_size), sigma),
 * (dst_width, dst_height), INTER_LINEAR) (optflowgf.cpp:1170-1172); dst device
 * float plane, dst_pitch in bytes. */
int tbdk_fb_level_image(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, int dst_width,
                        int dst_height, int smooth_size, double sigma, float* dst, int dst_pitch, void* stream);
/* FarnebackPolyExp (optflowgf.cpp:116-202): src device float plane; dst = 5
 * device float planes (plane c at byte offset c * height * dst_pitch) holding
 * the reference's CV_32FC5 channels c = 0..4. */
int tbdk_fb_poly_exp(tbdk_ctx* ctx, const float* src, int width, int height, int src_pitch, int poly_n,
                     double poly_sigma, float* dst, int dst_pitch, void* stream);

/* ---- HOG people detector (cv::cuda::HOG / cv::HOGDescriptor) -------------- */

/* cv::cuda::HOG::create(win_size, block_size, block_stride, cell_size, nbins) and
 * its setters (cudaobjdetect/include/opencv2/cudaobjdetect.hpp:95-180, defaults of
 * cudaobjdetect/src/hog.cpp:230-250), computed with the CPU HOGDescriptor's
 * numerics (objdetect/src/hog.cpp) that the sample's CPU mode runs. */
typedef struct tbdk_hog_params {
    int32_t win_w, win_h;                   /* 64 x 128 (48 x 96: the Daimler detector) */
    int32_t block_w, block_h;               /* 16 x 16 */
    int32_t block_stride_x, block_stride_y; /* 8, 8 */
    int32_t cell_w, cell_h;                 /* 8, 8 */
    int32_t nbins;                          /* 9 (2..32) */
    double win_sigma;                       /* -1: (block_w + block_h) / 8 */
    double l2hys_threshold;                 /* 0.2 */
    int32_t gamma_correction;               /* 1 */
    int32_t signed_gradient;                /* 0 */
    int32_t nlevels;                        /* 64 */
    double hit_threshold;                   /* 0 */
    int32_t win_stride_x, win_stride_y;     /* 8, 8 (= block stride) */
    double scale0;                          /* 1.05 */
    int32_t group_threshold;                /* 2 */
} tbdk_hog_params;

int tbdk_hog_default_params(tbdk_hog_params* p);
/* descriptor length nbins * cells/block * blocks/window (HOGDescriptor::getDescriptorSize,
 * hog.cpp:87-99); an SVM detector has this many coefficients, or one more (the bias) */
int tbdk_hog_descriptor_size(const tbdk_hog_params* p, int* size);

/* Replaces cv::cuda::HOG::detectMultiScale(img, found_locations, confidences)
 * (cudaobjdetect/src/hog.cpp:415-470) with HOGDescriptor::detectMultiScale(img,
 * rects, weights, hit_threshold, win_stride, Size(), scale0, group_threshold)
 * (objdetect/src/hog.cpp:2051-2105), the CPU call of samples/gpu/tbd.cpp:603-605.
 *   img     : device u8 image, cn 1 (gray), 3 (BGR) or 4 (BGRA, alpha ignored)
 *   svm     : host float coefficients, svm_len = descriptor size (+ 1 bias)
 *   rects   : host int32 (x, y, w, h) x max_rects; weights: host double x max_rects
 *   nrects  : number of grouped, clipped detections (<= max_rects)
 * Synchronous: returns when the results are in the host buffers. */
int tbdk_hog_detect_multiscale(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, int cn,
                               const tbdk_hog_params* params, const float* svm, int svm_len, int32_t* rects,
                               double* weights, int max_rects, int* nrects, void* stream);
/* One level, no resize and no grouping (HOGDescriptor::detect, hog.cpp:1655-1767):
 * window corners (x, y) and scores in window order; synchronous. */
int tbdk_hog_detect(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, int cn,
                    const tbdk_hog_params* params, const float* svm, int svm_len, int32_t* xy, double* scores,
                    int max_hits, int* nhits, void* stream);
/* The HOG calls of one context share its scratch (cell table, level image,
 * gradients, hits). A call on a different stream than the context's previous HOG
 * call first synchronises that previous stream.
 * Stage entry points (parity tests).  resize(src, dst, (dw, dh), INTER_LINEAR_EXACT)
 * of a u8 image (imgproc/src/resize.cpp:732-891): */
int tbdk_hog_resize(tbdk_ctx* ctx, const uint8_t* src, int width, int height, int pitch, int cn, uint8_t* dst,
                    int dst_width, int dst_height, int dst_pitch, void* stream);
/* HOGDescriptor::computeGradient (hog.cpp:239-550): grad = 2 floats per pixel
 * (grad_pitch bytes per row), qangle = 2 bytes per pixel (qangle_pitch). */
int tbdk_hog_gradient(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, int cn,
                      const tbdk_hog_params* params, float* grad, int grad_pitch, uint8_t* qangle,
                      int qangle_pitch, void* stream);
/* normalized block histograms (HOGCache::getBlock + normalizeBlockHistogram,
 * hog.cpp:860-1248) at every block position of the gcd(win stride, block stride)
 * grid: blocks[(by * nbx + bx) * hist_size + k], hist_size = nbins * cells/block. */
int tbdk_hog_blocks(tbdk_ctx* ctx, const float* grad, int grad_pitch, const uint8_t* qangle, int qangle_pitch,
                    int width, int height, const tbdk_hog_params* params, float* blocks, void* stream);

/* ---- tracking-by-detection loop (one video stream per context) ------------ */

/* Per-stream TBD loop: pyramid -> (GFTT on new / re-detect tracks) -> PyrLK over
 * every track's corners -> per-track similarity fit (KLT box propagation, the
 * Track::motionModel hook of modules/trackingbydetection/include/opencv2/tbd.hpp:111)
 * -> cv::tbd::Tracker::performTrackingStep (modules/trackingbydetection/src/tbd.cpp:210-286)
 * restated natively.  Replaces the tracking section of samples/gpu/tbd.cpp:624-706. */
typedef struct tbdk_tbd tbdk_tbd;

typedef struct tbdk_tbd_config {
    int32_t width, height;
    /* PyrLK (cv::calcOpticalFlowPyrLK defaults except maxLevel: "3-level" = 2) */
    int32_t win, max_level, lk_iters;
    double lk_epsilon;
    float min_eig_threshold;
    /* GFTT per track box */
    int32_t max_corners;             /* <= 256 */
    double quality_level, min_distance;
    int32_t redetect_every;          /* re-detect corners every N frames (5) */
    int32_t min_points;              /* ... or when fewer points survive (32) */
    int32_t min_fit_points;          /* points needed for the box fit (4) */
    /* cv::tbd::TbdArgs (samples/gpu/tbd.cpp:249-254 defaults) */
    double cost_of_non_assignment;
    int32_t time_window_size, track_age_threshold;
    double track_visibility_threshold, track_confidence_threshold;
    /* filterTracksOutOfBounds window; the reference hard-codes 0,1280,0,720 */
    int32_t bounds_xmin, bounds_xmax, bounds_ymin, bounds_ymax;
    int32_t max_tracks;              /* point-set slots on the device */
    int32_t use_klt;                 /* 0: reference constant-velocity prediction only */
} tbdk_tbd_config;

typedef struct tbdk_detection {      /* cv::tbd::Detection (tbd.hpp:69-83) */
    int32_t id, x, y, width, height;
    double confidence;
} tbdk_detection;

typedef struct tbdk_frame_metrics {  /* per-frame TP/FN/FP/GT/c/sum d (tbd.hpp:145-151) */
    int32_t tp, fn, fp, gt, matches;
    double bbox_overlap;
    int32_t ntracks;
    int32_t lk_points;               /* corners that entered PyrLK this frame */
    int32_t klt_points;              /* ... of which tracked (status 1) */
    int32_t klt_predicted;           /* tracks predicted by the KLT fit */
    int32_t redetected;              /* point sets refreshed by GFTT this frame */
    int32_t early_gftt;              /* ... of which served by the early GFTT (tbd_loop.hip) */
    int64_t lk_iters;                /* Newton iterations over all levels (flop accounting) */
    float host_wait_us;              /* host time blocked on the device this step */
    float host_tracker_us;           /* host time in the tracker step (assignment + bookkeeping) */
    float host_step_us;              /* host time in tbdk_tbd_step, end to end */
    float host_launch_us;            /* host time issuing the pyramid / LK / fit work (before the sync) */
} tbdk_frame_metrics;

typedef struct tbdk_track_info {
    uint32_t id;
    int32_t x, y, width, height;             /* last box */
    int32_t pred_x, pred_y, pred_w, pred_h;  /* predPosition */
    int32_t age, total_visible;
    int32_t npoints;                         /* tracked corners after this frame */
    double max_confidence, bbox_overlap;
} tbdk_track_info;

/* ---- the tracker alone (host only; no device, no context) ------------------
 * cv::tbd::Tracker (modules/trackingbydetection/include/opencv2/tbd.hpp:119-184,
 * src/tbd.cpp:182-1106) as a drop-in: performTrackingStep with an optional
 * per-track predicted centroid that replaces Track::motionModel (tbd.hpp:111)
 * for the tracks it names (the KLT box-propagation hook). */
typedef struct tbdk_tracker tbdk_tracker;

typedef struct tbdk_tracker_args {   /* cv::tbd::TbdArgs (tbd.hpp:25-41) + the bounds filter */
    double cost_of_non_assignment;
    int32_t time_window_size, track_age_threshold;   /* time_window_size <= 64 */
    double track_visibility_threshold, track_confidence_threshold;
    int32_t bounds_xmin, bounds_xmax, bounds_ymin, bounds_ymax;  /* reference: 0,1280,0,720 */
} tbdk_tracker_args;

typedef struct tbdk_prediction {
    uint32_t track_id;
    int32_t valid;                   /* 0: ignored (motion model used) */
    double cx, cy;                   /* predicted box centre */
} tbdk_prediction;

/* defaults of samples/gpu/tbd.cpp:249-254 and the hard-coded filter (tbd.cpp:218) */
int tbdk_tracker_default_args(tbdk_tracker_args* args);
int tbdk_tracker_create(const tbdk_tracker_args* args, tbdk_tracker** out);
int tbdk_tracker_destroy(tbdk_tracker* t);
/* Tracker::performTrackingStep (tbd.cpp:210-286); metrics: tp, fn, fp, gt,
 * matches, bbox_overlap and ntracks are filled, the KLT fields are 0. */
int tbdk_tracker_step(tbdk_tracker* t, const tbdk_detection* dets, int ndets, int frame_id,
                      const tbdk_prediction* preds, int npreds, tbdk_frame_metrics* metrics);
/* current tracks in the tracker's order (npoints = 0); *n = number of tracks */
int tbdk_tracker_tracks(const tbdk_tracker* t, tbdk_track_info* out, int cap, int* n);

/* ---- the sample's tracking driver (host only) -------------------------------
 * samples/gpu/tbd.cpp feeds the tracker ground-truth or external detections
 * from bbox files and writes MOT metrics.  Restated natively (tbd_app.cpp). */

/* Tracker::reset (tbd.cpp:197-208) */
int tbdk_tracker_reset(tbdk_tracker* t);
/* tbdk_tracker_step that also records the tracking result of every detection
 * carrying a ground-truth id into `traj` (performTrackingStep's trajectoryMap
 * argument, tbd.cpp:236-265); traj may be NULL. */
typedef struct tbdk_trajectories tbdk_trajectories;
int tbdk_tracker_step_traj(tbdk_tracker* t, const tbdk_detection* dets, int ndets, int frame_id,
                           const tbdk_prediction* preds, int npreds, tbdk_trajectories* traj,
                           tbdk_frame_metrics* metrics);

/* glibc rand() restated with private state (srand(seed); the sample's rand()
 * is never seeded = seed 1).  Attached to a tracker, each new track draws its
 * display colour from it (3 calls, tbd.cpp:71-73), as the reference does from
 * the global rand(); the sample's history draw shares the sequence. */
typedef struct tbdk_rand tbdk_rand;
int tbdk_rand_create(uint32_t seed, tbdk_rand** out);
int tbdk_rand_destroy(tbdk_rand* r);
int tbdk_rand_next(tbdk_rand* r, int32_t* out);
int tbdk_tracker_set_rand(tbdk_tracker* t, tbdk_rand* r);   /* r NULL: colours not drawn */
/* Args::parseHistoryDistribution (samples/gpu/tbd.cpp:258-291): "7,3" -> normalised floats */
int tbdk_parse_history_distribution(const char* s, float* out, int cap, int* n);
/* one history-age draw (samples/gpu/tbd.cpp:656-671): 1 + index of the first
 * cumulative float weight above rand()/RAND_MAX, else n */
int tbdk_history_age(tbdk_rand* r, const float* dist, int n, uint32_t* age);

/* Parsed bbox files (parseBboxFile, samples/gpu/tbd.cpp:1163-1295): per class
 * (0 pedestrians, 1 vehicles) the per-frame rows of one file; camera poses
 * (object id -1 rows) and a "history|a,b,..." line shared, as in the sample.
 * Lines "frame|id|x1|x2|y1|y2[|wx|wy[|wz]]" are ground truth (more than four
 * separators, frames offset by the first frame number), "frame|x1|x2|y1|y2"
 * external detections (id -2, frames from 0). */
typedef struct tbdk_sequence tbdk_sequence;
int tbdk_sequence_create(tbdk_sequence** out);
int tbdk_sequence_destroy(tbdk_sequence* s);
/* TBDK_EINVAL where the sample's stoi/stoul/stod throw (message: tbdk_sequence_error) */
int tbdk_sequence_parse_bbox_file(tbdk_sequence* s, int cls, const char* path, uint32_t num_frames);
const char* tbdk_sequence_error(const tbdk_sequence* s);
int tbdk_sequence_info(const tbdk_sequence* s, int cls, int32_t* nframes, int32_t* nposes, int32_t* nhistory);
int tbdk_sequence_history(const tbdk_sequence* s, uint32_t* out, int cap, int* n);
int tbdk_sequence_camera_pose(const tbdk_sequence* s, int index, double* out, int cap, int* n);
/* parseDetections (samples/gpu/tbd.cpp:1297-1340): frame `frame`'s detections
 * (confidence 1.0); ground-truth rows also add their position to traj (may be NULL) */
int tbdk_sequence_detections(const tbdk_sequence* s, int cls, int frame, tbdk_trajectories* traj,
                             tbdk_detection* out, int cap, int* n);

/* std::map<int, Trajectory> (tbd.hpp:46-80) */
int tbdk_trajectories_create(tbdk_trajectories** out);
int tbdk_trajectories_destroy(tbdk_trajectories* t);
int tbdk_trajectories_add_position(tbdk_trajectories* t, int id, int frame, int x, int y, int w, int h);
int tbdk_trajectories_count(const tbdk_trajectories* t, int* n);

/* the sample's per-history-age output buffers of tracks (samples/gpu/tbd.cpp:524-531, 679-704):
 * store = buffer[slot] = getTracks(); load = setTracks(buffer[slot]) (slot < 0: empty) */
typedef struct tbdk_track_buffer tbdk_track_buffer;
int tbdk_track_buffer_create(int nslots, tbdk_track_buffer** out);
int tbdk_track_buffer_destroy(tbdk_track_buffer* b);
int tbdk_tracker_store_tracks(tbdk_tracker* t, tbdk_track_buffer* b, int slot);
int tbdk_tracker_load_tracks(tbdk_tracker* t, const tbdk_track_buffer* b, int slot);

typedef struct tbdk_scenario_metrics {  /* the "scenario|" line + totals */
    int32_t mt, pt, ml;              /* mostly tracked / partially / mostly lost trajectories */
    int32_t idsw, fm;                /* ID switches, fragmentations (sums) */
    int32_t frames;                  /* "frame|" lines */
    double mota, amota, motp;
} tbdk_scenario_metrics;

/* App::writeTrackingOutputToFile (samples/gpu/tbd.cpp:946-1120): appends the
 * history / object / frame / scenario lines to `path` (NULL or "": metrics
 * only).  frame_count = frames processed; log_switches prints the sample's
 * "[frame f] target ... switched" lines to stdout. */
int tbdk_tracking_write(const tbdk_tracker* t, const uint32_t* history_ages, int nages, int frame_count,
                        tbdk_trajectories* traj, const char* path, int log_switches, tbdk_scenario_metrics* out);

typedef struct tbdk_app_args {       /* the sample's tracking flags (samples/gpu/tbd.cpp:221-257, 293-331) */
    const char* pedestrian_bbox_filename;
    const char* vehicle_bbox_filename;
    const char* pedestrian_tracking_filepath;
    const char* vehicle_tracking_filepath;
    const char* history_distribution;   /* "--history_distribution", NULL = "1" */
    int32_t write_tracking;
    int32_t num_tracking_iters;         /* 1 */
    int32_t num_tracking_frames;        /* 100 */
    uint32_t rand_seed;                 /* 1 = the sample's unseeded rand() */
    int32_t verbose;                    /* print ID-switch lines / errors to stdout */
    tbdk_tracker_args tracker;          /* TbdArgs defaults (samples/gpu/tbd.cpp:249-254) */
} tbdk_app_args;

typedef struct tbdk_app_result {
    int64_t frames, detections;         /* over all iterations */
    tbdk_scenario_metrics scenario[2];  /* last iteration, pedestrians / vehicles */
} tbdk_app_result;

int tbdk_app_default_args(tbdk_app_args* args);
/* App::run's tracking loop (samples/gpu/tbd.cpp:479-706, 823-841) over the
 * bbox files: history-age draw, setTracks from the output buffer,
 * performTrackingStep per class, tracking output per iteration. */
int tbdk_app_run(const tbdk_app_args* args, tbdk_app_result* result);

int tbdk_tbd_default_config(int width, int height, tbdk_tbd_config* cfg);
/* Loops on one context share the context's three side streams (post-tracker
 * GFTT, look-ahead PyrLK, early GFTT), created by its first loop: loops
 * stepped concurrently from different host threads on one context serialise
 * their off-critical work on them, and tbdk_tbd_destroy / tbdk_tbd_tracks
 * synchronise those streams, so they also wait for the other loops' work.
 * Use one context per concurrently stepped loop (the bench runs one loop per
 * GPU and process), and destroy every loop before its context. */
int tbdk_tbd_create(tbdk_ctx* ctx, const tbdk_tbd_config* cfg, tbdk_tbd** out);
int tbdk_tbd_destroy(tbdk_tbd* tbd);
/* One frame through the loop.  frame: device u8 (width x height, pitch);
 * dets: HOST array.  Synchronises the stream once (predictions -> host tracker). */
int tbdk_tbd_step(tbdk_tbd* tbd, const uint8_t* frame, int pitch, int frame_id, const tbdk_detection* dets,
                  int ndets, tbdk_frame_metrics* metrics, void* stream);
/* tbdk_tbd_step when the next frame is already on the device (a decode
 * pipeline, or a clip): the next frame's pyramid is enqueued behind this
 * frame's fit (the device builds it while the host tracks), and the next
 * frame's PyrLK of every point set this step leaves unchanged behind the
 * post-tracker GFTT, without returning to the caller in between.
 * next_frame must keep its pixels until the next step, which must pass the
 * same pointer, pitch and stream to use that work (otherwise it is redone).
 * Per-frame results are identical to tbdk_tbd_step's. */
int tbdk_tbd_step_ahead(tbdk_tbd* tbd, const uint8_t* frame, int pitch, int frame_id, const tbdk_detection* dets,
                        int ndets, const uint8_t* next_frame, int next_pitch, tbdk_frame_metrics* metrics,
                        void* stream);
/* The loop of samples/gpu/tbd.cpp:624-706 over nframes resident frames:
 * frames = host array of device pointers (same pitch), frame ids
 * first_frame_id + i, frame i's detections dets[det_offsets[i] ..
 * det_offsets[i+1]) (host), metrics = nframes entries or NULL.  Equivalent to
 * tbdk_tbd_step_ahead over the sequence. */
int tbdk_tbd_run(tbdk_tbd* tbd, const uint8_t* const* frames, int pitch, int first_frame_id,
                 const tbdk_detection* dets, const int32_t* det_offsets, int nframes, tbdk_frame_metrics* metrics,
                 void* stream);
/* tbdk_tbd_run over frames in HOST memory (the sample's frame source,
 * samples/gpu/tbd.cpp:568-599: a decoded frame is uploaded, then processed):
 * frames = host pointers (same pitch; page-locked memory lets the uploads
 * overlap the loop).  Each frame is uploaded into a ring of three device
 * frames on a copy stream two frames ahead of its use, so frame i+2's upload
 * runs during frame i's work; results are identical to tbdk_tbd_run's. */
int tbdk_tbd_run_host(tbdk_tbd* tbd, const uint8_t* const* frames, int pitch, int first_frame_id,
                      const tbdk_detection* dets, const int32_t* det_offsets, int nframes,
                      tbdk_frame_metrics* metrics, void* stream);
int tbdk_tbd_tracks(tbdk_tbd* tbd, tbdk_track_info* out, int cap, int* n);
/* Attach a trajectory map (NULL detaches): every later step records, for each
 * detection with a ground-truth id (id >= 0), its position (parseDetections,
 * samples/gpu/tbd.cpp:1327-1338) and its tracking result (tbd.cpp:236-265). */
int tbdk_tbd_set_trajectories(tbdk_tbd* tbd, tbdk_trajectories* traj);
/* tbdk_tracking_write for the loop's tracker and attached trajectories */
int tbdk_tbd_tracking_write(tbdk_tbd* tbd, const uint32_t* history_ages, int nages, int frame_count,
                            const char* path, int log_switches, tbdk_scenario_metrics* out);
/* The KLT predictions the last tbdk_tbd_step handed to the tracker (one per
 * track with a valid box fit, in track order); *n = their number. */
int tbdk_tbd_predictions(const tbdk_tbd* tbd, tbdk_prediction* out, int cap, int* n);

/* ---- synthetic sequences (bench / test input) ----------------------------- */

/* Renders frames [t0, t0+nframes) of the deterministic synthetic sequence of
 * opencv_amd/csrc/synth_spec.h into `out` (device, nframes x height x pitch).
 * gt_boxes (host, may be NULL): nframes x nobj x 5 int32 {valid, x, y, w, h}. */
int tbdk_synth_render(tbdk_ctx* ctx, uint32_t seed, int width, int height, int nobj,
                      int t0, int nframes, uint8_t* out, int pitch, int32_t* gt_boxes,
                      void* stream);

/* ---- measurement ---------------------------------------------------------- */

/* Copies `bytes` (a multiple of 16; dst and src 16-byte aligned, not
 * overlapping) device to device with a hand-written 16-byte-per-lane stream
 * copy (global_load_dwordx4 / global_store_dwordx4), asynchronously on
 * `stream`; timed as kernel "hbm_copy".  bench.py's measured HBM copy peak
 * (SURVEY.md §8(d)); no reference counterpart. */
int tbdk_hbm_copy(tbdk_ctx* ctx, void* dst, const void* src, int64_t bytes, void* stream);

/* Library version string */
const char* tbdk_version(void);
/* TBDK_ABI_VERSION of the library (struct layouts of this header) */
int tbdk_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TBDK_H */
