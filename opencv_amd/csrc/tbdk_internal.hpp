// tbdk_internal.hpp — shared declarations of the HIP kernels and the C-ABI runtime.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/tbdk.h"

namespace tbdk {

__host__ __device__ inline int align_up(int v, int a) { return (v + a - 1) / a * a; }

// XCD-aware block remap (bijective for any grid size): blocks are dealt
// round-robin over the 8 XCDs, so hardware block b runs on XCD group b % 8;
// give each group a contiguous range of logical blocks so neighbouring work
// (points of one track, rows of one image band) shares one XCD's L2.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg)
{
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Border width of every padded level: >= win + 1 so the LK window plus its
// bilinear/Scharr neighbours never leaves the allocation.
inline int level_pad(int win_w, int win_h)
{
    int m = win_w > win_h ? win_w : win_h;
    int p = align_up(m + 2, 16);
    return p < 32 ? 32 : p;
}

struct TimingRec {
    const char* name;
    hipEvent_t begin, end;
};

// makes the context's device current for the scope of a C-ABI call
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

struct FbScratch;  // farneback.hip
// GFTT scratch: one per context (the standalone calls) and one per TBD loop,
// so loops sharing a context never share it across their streams
struct GfttScratch {
    void* rois = nullptr;    // GfttRoi[cap_rois]
    int* blk = nullptr;      // per-strip eigenvalue maxima
    void* cand = nullptr;    // local-maximum words (uint64 per strip row)
    void* planes = nullptr;  // cap_px floats (eig)
    void* resp = nullptr;    // blockSize != 3 / Harris: cov (3 floats) + row sums (3 doubles) per pixel
    int cap_rois = 0;
    int64_t cap_px = 0;
    int64_t cap_resp_px = 0;
};
struct HogScratch;  // hog.hip

}  // namespace tbdk

struct tbdk_ctx {
    int device = 0;
    std::atomic<bool> timing{false};
    // guards the timing state below (timing_only, timing_calls, recs,
    // free_events): a TBD loop's launch worker records launches too
    std::mutex timing_mu;
    int opt_gftt_eig_redo = 0;  // tbdk_ctx_set_option("gftt_eig_redo")
    int opt_pyr_xcd = 1;       // tbdk_ctx_set_option("pyr_xcd"): pyramid roles' row bands per XCD
    int opt_pyr_rows = 1;      // tbdk_ctx_set_option("pyr_rows"): rows per thread of the two-role u8 build (1, 2, 4)
    int opt_pyr_fuse = 1;      // tbdk_ctx_set_option("pyr_fuse"): 1 the two-role launch + one per level, 2 levels 0-2 in one tiled launch (slower, A/B), 0 one launch per level
    int opt_lk_solo = 4;       // tbdk_ctx_set_option("lk_solo"): LkArgs::solo_min of the lk_multi launches
    int opt_lk_scharr_fly = 0; // tbdk_ctx_set_option("lk_scharr_fly"): lk_multi derives Ix/Iy itself
    int opt_lk_impl = 0;        // tbdk_ctx_set_option("lk_impl"): PyrLK kernel under impl 0
    int opt_lk_seg_inline = 1;  // tbdk_ctx_set_option("lk_seg_inline"): segment lists in the kernel arguments
    int opt_fb_prep_ahead = 1;  // tbdk_ctx_set_option("fb_prep_ahead"): Farneback level prep on a side stream
    int opt_hog_level_streams = 3;  // tbdk_ctx_set_option("hog_level_streams"): lanes of detectMultiScale
    int opt_hog_window_tiled = 1;  // tbdk_ctx_set_option("hog_window_tiled"): LDS-tiled window pass
    int opt_hog_block_tiled = 1;  // tbdk_ctx_set_option("hog_block_tiled"): LDS-tiled block kernel where it applies
    int opt_tbd_early_gftt = 2;  // tbdk_ctx_set_option("tbd_early_gftt")
    int opt_tbd_spec_la = 1;     // tbdk_ctx_set_option("tbd_spec_lookahead")
    int opt_tbd_zero_copy = 1;   // tbdk_ctx_set_option("tbd_zero_copy"), read by tbdk_tbd_create
    int opt_tbd_fit_flag = 1;    // tbdk_ctx_set_option("tbd_fit_flag"), read by tbdk_tbd_create
    int opt_tbd_early_order = 0;  // tbdk_ctx_set_option("tbd_early_order"): where the early GFTT is launched in a step (round 6: 0)
    int opt_tbd_early_prio = 0;  // tbdk_ctx_set_option("tbd_early_prio"), read by tbdk_tbd_create
    int opt_tbd_early_la = 1;    // tbdk_ctx_set_option("tbd_early_la"): look-ahead PyrLK of early GFTT rows
    int opt_tbd_pyr_derivs = 0;  // tbdk_ctx_set_option("tbd_pyr_derivs"): loop pyramids with Scharr planes (A/B)
    int opt_tbd_fit_inline = 1;  // tbdk_ctx_set_option("tbd_fit_inline"): the fit table in the kernel arguments
    int opt_gftt_inline = 1;     // tbdk_ctx_set_option("gftt_inline"): GFTT ROI tables in the kernel arguments
    int opt_tbd_fit_wgpub = 1;   // tbdk_ctx_set_option("tbd_fit_wgpub"): one system-scope release per fit workgroup
    int opt_tbd_la_pyr_side = 2;  // tbdk_ctx_set_option("tbd_la_pyr_side"): where the look-ahead pyramid is built
    int opt_tbd_post_direct = 1;  // tbdk_ctx_set_option("tbd_post_direct"): next step waits for the early GFTT itself
    int opt_tbd_la_defer = 0;    // tbdk_ctx_set_option("tbd_la_defer"): look-ahead PyrLK launched by the next step
    int opt_gftt_compact = 1;    // tbdk_ctx_set_option("gftt_compact"): GFTT writes only its candidates' values
    int opt_tbd_ahead_at = 0;    // tbdk_ctx_set_option("tbd_ahead_at"): where a step launches the ahead GFTT (0..2)
    int opt_tbd_gftt_ahead = 1;  // tbdk_ctx_set_option("tbd_gftt_ahead"): tbdk_tbd_run's early GFTT a frame ahead
    int opt_tbd_borrow_l0 = 0;   // tbdk_ctx_set_option("tbd_borrow_l0"): tbdk_tbd_run's pyramids take the frame as level 0 (A/B)
    int opt_tbd_fit_gate = 1;    // tbdk_ctx_set_option("tbd_fit_gate"): the host launches the fit once the look-ahead PyrLK is done
    int opt_tbd_async_la = 0;    // tbdk_ctx_set_option("tbd_async_la"): look-ahead launches by a worker thread (read by tbdk_tbd_create)
    std::string timing_only;  // ",name,name," filter of tbdk_timing_select ("" = all)
    int timing_every = 1;     // tbdk_ctx_set_option("timing_every"): events on every Nth selected launch
    std::vector<std::pair<std::string, int64_t>> timing_calls;  // selected launches per name (sampled or not)
    std::vector<tbdk::TimingRec> recs;
    std::vector<hipEvent_t> free_events;
    tbdk::GfttScratch gftt;  // grown on demand, or up front by tbdk_gftt_reserve
    tbdk::FbScratch* fb = nullptr;  // dense Farneback planes (farneback.hip)
    void* dense_buf = nullptr;      // dense PyrLK grid / next points / status (klt_dense.hip)
    void* dcase_buf = nullptr;      // dense PyrLK case images (klt_dense.hip)
    size_t dcase_cap = 0;           // bytes
    int opt_lk_dense_case = 1;      // tbdk_ctx_set_option("lk_dense_case"): dense PyrLK from case images
    tbdk::HogScratch* hog = nullptr;  // HOG level image, gradients, blocks, hits (hog.hip)
    int64_t dense_cap = 0;          // pixels
    // the TBD loop's side streams (post-tracker work, look-ahead PyrLK, early
    // GFTT), created by the context's first loop and kept for every later one,
    // so that each loop gets the first loop's stream -> hardware-queue mapping
    // (HIP deals streams to the few hardware queues as they are created; a
    // loop created after other streams otherwise lands on a different, often
    // slower, mapping).  Not at context creation: streams created then shift
    // the queue the caller's stream gets at its first use (HOG's lanes then
    // shared it: 1.36k -> 0.92k frames/s).  Loops on one context share them
    // (stream order only adds dependencies).
    std::mutex tbd_mu;
    hipStream_t tbd_side = nullptr, tbd_la = nullptr, tbd_early = nullptr;
};

namespace tbdk {

// RAII-free helpers used by the C-ABI around each launch.
int timing_begin(tbdk_ctx* ctx, const char* name, hipStream_t s);
void timing_end(tbdk_ctx* ctx, int rec, hipStream_t s);

// frees the context's Farneback scratch (farneback.hip)
void fb_release(tbdk_ctx* ctx);
void hog_release(tbdk_ctx* ctx);
void hog_create_lanes(tbdk_ctx* ctx);
void fb_create_streams(tbdk_ctx* ctx);

// ---- kernels (klt_pyr.hip) ----
hipError_t launch_pad_copy(const uint8_t* src, int spitch, const tbdk_level& dst, hipStream_t s);
hipError_t launch_pyr_down_padded(const tbdk_level& src, const tbdk_level& dst, hipStream_t s);
hipError_t launch_pyr_down_plain(const uint8_t* src, int w, int h, int spitch, uint8_t* dst, int dpitch,
                                 hipStream_t s);
// Scharr derivative planes (interior only; the zero frame is written once at allocation)
hipError_t launch_scharr_levels(const tbdk_pyr& pyr, hipStream_t s);
// every u8 level of pyr from the frame (fused launches where the levels allow)
// skip_l0: levels 1.. only, level 0 being the frame itself (pyr.lv[0] already
// points at it, pad 0; the two-role launch with no copy role)
hipError_t launch_pyr_levels(const uint8_t* img, int pitch, const tbdk_pyr& pyr, int fuse, int rows, int xcd,
                             hipStream_t s, bool skip_l0 = false);
// tbdk_pyr.flags bit (internal): level 0 is borrowed -- lv[0] is the caller's
// frame (pad 0), built by pyr_build_borrowed for the TBD loop; only the
// several-points-per-wave PyrLK kernel reads such a level (reflect-101 at its
// edges by coordinates)
constexpr int32_t kPyrL0Borrowed = 1 << 30;
// the u8 levels-only pyramid of a frame with level 0 borrowed from the frame
// (no padded copy); own_l0: the pyramid's own level-0 buffer, restored by
// pyr_restore_l0
int pyr_build_borrowed(tbdk_ctx* ctx, const uint8_t* img, int pitch, tbdk_pyr* pyr, hipStream_t s);
// a borrowed pyramid's level 0 copied into its own padded buffer (own_l0) and
// made its level 0 again
int pyr_restore_l0(tbdk_ctx* ctx, tbdk_pyr* pyr, const tbdk_level& own_l0, hipStream_t s);
// the fp16 pyramid (klt_f16.hip): level 0 from a u8 (img_f16 = 0) or fp16 frame,
// the fp16 pyrDown levels and the fp16 derivative pairs
hipError_t launch_pyr_build_f16(const uint8_t* img, int pitch, int img_f16, const tbdk_pyr& pyr, hipStream_t s);
// fp32 pixel path: src_kind 0 u8, 1 u16, 2 fp32 frame
hipError_t launch_pyr_build_f32(const uint8_t* img, int pitch, int src_kind, const tbdk_pyr& pyr, hipStream_t s);
// role-split fp16 / fp32 pyramid build (klt_pyr_fp.hip); kind: 0 u8, 1 u16, 2 f32, 3 f16 frame
hipError_t launch_pyr_build_fp(const uint8_t* img, int pitch, int kind, bool f32, const tbdk_pyr& pyr, int rows,
                               int xcd, hipStream_t s);

// ---- kernels (klt_lk.hip) ----
struct LkLevel {
    const uint8_t* I;
    const uint8_t* J;
    const uint8_t* D;   // derivative plane of I (int16x2 per pixel), may be null
    int w, h, ipitch, jpitch, ipad, jpad, dpitch, dpad;
    // dense mode (klt_dense.hip): the level's case images, element (y, x) of case
    // c at C[c * cstride + y * cpitch + x] for y, x from -border on
    const uint2* C;
    int64_t cstride;
    int cpitch;
};

constexpr int kSegInline = 256;  // segment list entries LkArgs can carry itself

struct LkArgs {
    LkLevel lv[TBDK_MAX_LEVELS];
    // optional segmented layout: point i = seg * seg_stride + j is valid iff
    // j < seg_counts[seg]; invalid points are skipped (outputs untouched).
    // With seg_list, launch index k runs segment seg_list[k / seg_stride].
    const int32_t* seg_counts;
    const int32_t* seg_list;
    int seg_stride;
    int seg_ninl;  // > 0: the segment list is seg_inl[0, seg_ninl) instead of seg_list
    int max_level, win_w, win_h, max_count, flags, n;
    int cn;  // channels (klt_cn.hip; the one-channel kernels ignore it)
    double eps2;
    float min_eig;
    const float* prev_pts;
    float* next_pts;
    uint8_t* status;
    float* err;
    int32_t* iters;
    // dense mode: point k of the launch is pixel (k % dense_w, k / dense_w);
    // outputs the flow (next - pixel, CV_32FC2, flow_pitch bytes) and the status
    // plane (dstatus_pitch bytes; may be null)
    int dense_w;
    float* flow;
    int flow_pitch;
    uint8_t* dstatus;
    int dstatus_pitch;
    // the segment list carried in the kernel arguments (ctx option lk_seg_inline):
    // the TBD loop's lists live in pinned host memory (zero-copy), where every
    // wave's first load would be a round trip over the host link
    uint16_t seg_inl[kSegInline];
    // lk_multi: a wave whose other points have stopped runs its last point's
    // remaining Newton steps on all its lanes from step solo_min on (0: never;
    // ctx option lk_solo)
    int solo_min;
#ifdef TBDK_LK_TRACE
    unsigned trace_base;  // probe builds: first trace record of this launch (klt_lk_multi.hip)
#endif
};

// launch index -> point index under the segmented layout, -1 if none
__device__ __forceinline__ int seg_point(const LkArgs& a, int k)
{
    if (k >= a.n) return -1;
    if (!a.seg_counts) return k;
    const int seg = k / a.seg_stride, j = k - seg * a.seg_stride;
    const int s = a.seg_ninl > 0 ? (int)a.seg_inl[seg] : a.seg_list ? a.seg_list[seg] : seg;
    return j < a.seg_counts[s] ? s * a.seg_stride + j : -1;
}

// dense mode of lk_internal (klt_dense.hip): the case images of every level
// and the flow / status outputs
struct LkDense {
    const uint2* C[TBDK_MAX_LEVELS];
    int64_t cstride[TBDK_MAX_LEVELS];
    int cpitch[TBDK_MAX_LEVELS];
    int w;
    float* flow;
    int flow_pitch;
    uint8_t* status;
    int status_pitch;
};

// argument checking + kernel choice shared by tbdk_lk_sparse and the TBD loop
int lk_internal(tbdk_ctx* ctx, const tbdk_pyr* prev, const tbdk_pyr* next, const float* prev_pts, float* next_pts,
                uint8_t* status, float* err, int32_t* iters, int n, const tbdk_lk_params* p,
                const int32_t* seg_counts, int seg_stride, void* stream, const int32_t* seg_list = nullptr,
                const LkDense* dense = nullptr, const int32_t* seg_list_host = nullptr);
int map_status(hipError_t e);
// multi-channel u8 pyramids and PyrLK (klt_cn.hip)
hipError_t launch_pyr_cn(const uint8_t* img, int pitch, const tbdk_pyr& pyr, hipStream_t s);
hipError_t launch_lk_cn(const LkArgs& a, hipStream_t s);
size_t lk_cn_smem_bytes(int win_w, int win_h, int cn);
hipError_t launch_lk_cn_f32(const LkArgs& a, hipStream_t s);
size_t lk_cn_f32_smem_bytes(int win_w, int win_h, int cn);
hipError_t launch_pyr_build_f32_cn(const uint8_t* img, int pitch, int kind, const tbdk_pyr& pyr, hipStream_t s);

size_t lk_smem_bytes(int win_w, int win_h);
hipError_t launch_lk_sparse(const LkArgs& a, hipStream_t s);
// register-strip kernel (klt_lk_strip.hip); returns hipErrorNotSupported for
// windows without an instantiation (caller falls back to launch_lk_sparse)
bool lk_strip_supported(int win_w, int win_h);
hipError_t launch_lk_strip(const LkArgs& a, hipStream_t s);
// several points per wave (klt_lk_multi.hip), same results
bool lk_multi_supported(int win_w, int win_h);
// fly: Scharr derivatives computed in the kernel (no derivative planes read)
hipError_t launch_lk_multi(const LkArgs& a, bool fly, hipStream_t s);
// dense mode of the several-points-per-wave kernel (klt_dense.hip: case images in a.lv[].C)
hipError_t launch_lk_multi_dense(const LkArgs& a, hipStream_t s);
// the fp16 pixel path (klt_f16.hip)
bool lk_f16_supported(int win_w, int win_h);
hipError_t launch_lk_f16(const LkArgs& a, bool f32, hipStream_t s);  // fp16 or (f32) fp32 pixel path

// ---- box propagation (box_fit.hip) ----
hipError_t launch_box_propagate(const float* prev, const float* next, const uint8_t* status, const int32_t* offsets,
                                const tbdk_roi* boxes, int nboxes, int min_points, tbdk_box_fit* out, hipStream_t s);

// ---- affine warp (warp.hip) ----
void invert_affine(const double* M, double* out);
hipError_t launch_warp_affine(const uint8_t* src, int sw, int sh, int spitch, uint8_t* dst, int dw, int dh, int dpitch,
                              const double* minv, int inter, int border, int cval, hipStream_t s);

// ---- synthetic renderer (synth.hip) ----
struct SynPoseDev;  // == syn_pose
hipError_t launch_hbm_copy(const void* src, void* dst, size_t n16, hipStream_t s);
hipError_t launch_synth(const void* poses_dev, int nobj, uint32_t bgseed, int W, int H, int nframes,
                        uint8_t* out, int pitch, hipStream_t s);

}  // namespace tbdk

namespace tbdk {
// ---- GFTT over ROIs (klt_gftt.hip) ----
struct GfttRoi {
    int x, y, w, h;
    int off;   // first value of this ROI in the eigenvalue plane (rows gftt_epitch(w) floats apart)
    int moff;  // first local-maximum word of this ROI (one uint64 per strip row)
    int cblk;  // first kGfttStrip-column strip of this ROI in the flat per-strip grid
};
// output columns per wave of the eigenvalue walk: lanes 4..59 (4 halo lanes per
// side: eigenvalues are exact in lanes 2..61, the 3x3 local-maximum test in 3..60).
// 56 columns = 224 bytes of eigenvalues, a whole number of 32-byte sectors, and
// eigenvalue rows gftt_epitch(w) floats apart from 32-byte aligned ROI offsets:
// every strip row is written as whole sectors (58 columns of a tight plane wrote
// ~1.7x the plane's bytes in partial sectors)
constexpr int kGfttStrip = 56;
constexpr int kGfttHalo = 4;
__host__ __device__ constexpr int gftt_epitch(int w) { return (w + 7) & ~7; }
// a ROI table entry carried in the kernel arguments (GfttArgs::inl)
struct GfttRoiC {
    uint16_t x, y, w, h;
    int off, moff, cblk;
};
constexpr int kGfttInline = 128;
struct GfttArgs {
    const uint8_t* img;
    int pitch;
    const GfttRoi* rois;
    int nroi;
    int ncblk;       // strips over all ROIs (eigenvalue workgroups)
    float* eig;      // min eigenvalue per ROI pixel
    int* blk_max;    // per strip: max eigenvalue key
    uint64_t* lmax;  // per strip row: ballot of the lanes holding an interior 3x3 local maximum
    int cap;         // LDS candidate capacity per ROI (power of two)
    int img_bytes;   // LDS for the per-ROI byte image of the greedy walk (0: list mode)
    int max_corners;
    double quality, min_distance;
    float2* corners;  // nroi rows of corner_stride (>= max_corners) float2
    int corner_stride;
    int32_t* counts;  // nroi (-1: candidate overflow)
    int eig_redo;     // test option: walk every eig strip segment in sequence
    // != 0: no eigenvalue plane; per strip row only its local maxima's values,
    // packed in lane order at the row's first columns (ctx option gftt_compact;
    // only with quality <= 1, where a ROI whose max is <= 0 has no candidate)
    int compact;
    // > 0: the ROI table is inl[0, nroi) instead of rois (ctx option gftt_inline):
    // the TBD loop's tables live in pinned host memory, where the eigenvalue
    // kernel's binary search over them is a chain of host-link round trips
    int ninl;
    GfttRoiC inl[kGfttInline];
};
constexpr int kGfttCap = 16384;  // candidates per ROI (LDS-resident for the sort)
// scratch sizes for (rois, pixels): strips <= px/60 + rois; local-maximum words
// (ROIs of at least 3x3 only) <= px/60 + px/3
inline int64_t gftt_max_cblocks(int rois, int64_t px) { return px / kGfttStrip + rois; }
inline int64_t gftt_max_words(int64_t px) { return px / kGfttStrip + px / 3 + 1; }
size_t gftt_select_smem(int cap, int max_corners, int img_bytes);
void gftt_plan(GfttArgs& a, int max_area);  // sets cap and img_bytes
struct GfttPlan {
    int nroi = 0, ncblk = 0, max_area = 0, max_w = 0, max_h = 0;
    int64_t total = 0;  // ROI pixels
    int64_t words = 0;  // local-maximum words
};
// host side of tbdk_gftt_rois: validate and lay out the ROI table (tab: nroi entries)
int gftt_prepare(const tbdk_roi* rois, int nroi, int width, int height, const tbdk_gftt_params* p, GfttRoi* tab,
                 GfttPlan* plan);
// launches with a device-resident ROI table (uploaded by the caller on stream s)
// after_eig (optional): recorded between the eigenvalue and select launches
// scratch sized for max_rois ROIs of max_px pixels in total (grows only)
int gftt_reserve(GfttScratch& sc, int device, int max_rois, int64_t max_px);
void gftt_scratch_free(GfttScratch& sc);
// h_rois (optional): a host-readable copy of the table, carried in the kernel
// arguments when it fits (ctx option gftt_inline)
int gftt_launch(tbdk_ctx* ctx, GfttScratch& sc, const uint8_t* img, int pitch, const GfttRoi* d_rois, const GfttPlan& plan,
                const tbdk_gftt_params* p, float* corners, int32_t* counts, hipStream_t s,
                hipEvent_t after_eig = nullptr, int corner_stride = 0,  // 0: max_corners
                const GfttRoi* h_rois = nullptr);
hipError_t launch_gftt(const GfttArgs& a, hipStream_t s, hipEvent_t after_eig = nullptr);
hipError_t launch_gftt_eig(const GfttArgs& a, hipStream_t s);  // eigenvalue planes only
hipError_t launch_gftt_select(const GfttArgs& a, hipStream_t s);
// blockSize != 3 or Harris (klt_gftt_resp.hip): the response plane, strip
// maxima and local-maximum words in gftt_eig_kernel's layout
struct GfttRespArgs {
    const uint8_t* img;
    int pitch;
    const GfttRoi* rois;
    int nroi;
    float* cov;      // 3 floats per ROI pixel
    double* rs;      // 3 doubles per ROI pixel
    float* eig;      // response per ROI pixel
    int* blk_max;
    uint64_t* lmax;
    int block;       // boxFilter size
    int harris;      // 0: min eigenvalue, 1: Harris
    float k, k2;     // Sobel taps x 1/(4*block*255)
    float kf;        // (float)harris_k (the SIMD paths)
    double hk;       // harris_k (the scalar path)
};
hipError_t launch_gftt_resp(const GfttRespArgs& a, int ncblk, int max_w, int max_h, int max_area, hipStream_t s);
int gftt_reserve_resp(GfttScratch& sc, int device, int64_t max_px);
inline bool gftt_generic(const tbdk_gftt_params* p) { return p->block_size != 3 || p->use_harris != 0; }
}  // namespace tbdk
