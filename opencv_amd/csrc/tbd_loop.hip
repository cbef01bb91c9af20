// tbd_loop.hip — the per-stream tracking-by-detection loop (C ABI tbdk_tbd_*).
//
// Per frame (one HIP stream, one host thread per stream / GPU):
//   1. pyramid of the new frame (levels only, one fused launch)          [HIP]
//   2. sparse PyrLK of every live track's corners, prev -> new frame     [HIP, one launch,
//      segmented layout: slot s owns points s*256 .. s*256+count[s]-1]
//   3. tbd_fit_kernel, one wave per live track: ballot-compaction of the
//      tracked points (they become next frame's corners) and the 4-DOF
//      similarity fit of getRTMatrix (video/src/lkpyramid.cpp:1436-1468),
//      giving the KLT-propagated centroid                                [HIP]
//   4. predictions -> host (the single stream sync of the frame)
//   5. cv::tbd::Tracker::performTrackingStep restated natively, with the
//      KLT centroid as Track::motionModel (tbd.hpp:111)                 [host C++]
//   6. GFTT in the boxes of new tracks and of tracks due for re-detection
//      (every `redetect_every` frames or < min_points corners) into GFTT rows
//      of the slot arrays; the next step tracks such a set from its row and
//      its fit compacts the tracked points into the slot                  [HIP]
// Early GFTT: a new track's box is its detection's box (tbd.cpp:1043-1055), so
// GFTT over the detections that will surely start new tracks (boxes beyond the
// tracker's bounds filter, tbd.cpp:218,306-331: any track on them is deleted
// before the assignment) is launched at the start of the step, off the
// critical path; after the tracker step, new tracks whose box equals such a
// detection box take those corners (the same ROI of the same frame, so the
// same corners), every other refreshed set runs the post-tracker GFTT.  On
// re-detection frames the early GFTT also runs on the box each existing track
// will get if the tracker assigns it the detection overlapping it most.
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <new>
#include <queue>
#include <thread>
#include <vector>

#include "box_fit.hpp"
#include "flat_map.hpp"
#include "tbd_tracker.hpp"
#include "tbdk_internal.hpp"

namespace tbdk {

constexpr int kSlotPts = 256;  // corner capacity per track
constexpr int kEarlySets = 3;  // early GFTT row sets (this step's, the next frame's ahead, the previous step's)
constexpr int kRowSets = 2 + kEarlySets;  // rows of the slot arrays, in units of max_tracks (see tbdk_tbd::src_row)

struct FitEntry {
    int slot;
    int x, y, w, h;  // the track's last box (centroid convention of tbd.cpp:1064-1065)
    int src;         // >= 0: a refreshed set, its corners (and PyrLK results) in GFTT row src
};

// the fit table carried in the kernel arguments (ctx option tbd_fit_inline): the
// zero-copy table lives in pinned host memory, where each fit wave's first load
// is a round trip over the host link on the frame's critical chain
struct FitEntryC {
    uint16_t slot;
    int16_t src;
    int16_t x, y;
    uint16_t w, h;
};
constexpr int kFitInline = 256;
struct FitInline {
    FitEntryC e[kFitInline];
};

struct FitOut {
    double cx, cy;  // KLT-propagated centroid
    double scale;
    int valid;
    int n;          // corners still tracked (kept in the slot)
    int npts;       // corners that entered LK this frame
    int iters;      // Newton iterations of those corners over all levels (flop accounting)
};

// One wave per live track, kFitWaves tracks per workgroup.  Fit terms follow
// getRTMatrix's non-full-affine branch (float products summed in double),
// accumulated wave-parallel in a fixed order (box_fit.hpp: wave_fit_similarity).
#ifndef TBDK_FIT_WAVES
#define TBDK_FIT_WAVES 8  // tracks (waves) per fit workgroup (tuning builds)
#endif
constexpr int kFitWaves = TBDK_FIT_WAVES;
__global__ __launch_bounds__(64 * kFitWaves) void tbd_fit_kernel(const FitEntry* __restrict__ ents, int nents,
                                                                 float2* __restrict__ slot_pts,
                                                                 const float2* __restrict__ slot_next,
                                                                 const uint8_t* __restrict__ slot_status,
                                                                 const int32_t* __restrict__ slot_iters,
                                                                 int32_t* __restrict__ slot_counts,
                                                                 FitOut* __restrict__ out, int min_fit,
                                                                 unsigned* __restrict__ fit_cnt, int32_t* flag, int tag,
                                                                 int inl, const FitInline fi, int wg_pub)
{
    __shared__ float2 s_a[kFitWaves][kSlotPts], s_b[kFitWaves][kSlotPts];
    __shared__ FitOut s_out[kFitWaves];  // wg_pub: the workgroup's results, published by wave 0
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int e = blockIdx.x * kFitWaves + wv;
    if (e < nents) {
        float2* sa = s_a[wv];
        float2* sb = s_b[wv];
        FitEntry E;
        if (inl) {
            const FitEntryC c = fi.e[e];
            E = FitEntry{c.slot, c.x, c.y, c.w, c.h, c.src};
        } else {
            E = ents[e];
        }
        const int row = E.src >= 0 ? E.src : E.slot;  // where the tracked set and its PyrLK results are
        const int c0 = slot_counts[row];
        const int cnt = c0 < 0 ? 0 : c0;  // -1: GFTT candidate overflow, no corners
        const size_t base = (size_t)E.slot * kSlotPts, rb = (size_t)row * kSlotPts;
        int m = 0, it = 0;
        // every chunk's loads first (one memory round trip for the wave, not one
        // per chunk of 64 points), issued together with the count's (the row's
        // whole capacity is read and masked by the count afterwards), then the
        // ballot compaction in point order
        constexpr int kChunks = kSlotPts / 64;
        uint8_t stv[kChunks];
        int itv[kChunks];
        float2 pv[kChunks], nv[kChunks];
#pragma unroll
        for (int c = 0; c < kChunks; ++c) {
            const int j = c * 64 + lane;
            stv[c] = slot_status[rb + j];
            itv[c] = slot_iters[rb + j];
            pv[c] = slot_pts[rb + j];
            nv[c] = slot_next[rb + j];
        }
#pragma unroll
        for (int c = 0; c < kChunks; ++c) {
            if (c * 64 + lane >= cnt) {
                stv[c] = 0;
                itv[c] = 0;
            }
        }
#pragma unroll
        for (int c = 0; c < kChunks; ++c) {
            const bool ok = stv[c] != 0;
            it += itv[c];
            const unsigned long long bal = __ballot(ok);
            if (ok) {
                const int pos = m + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
                sa[pos] = pv[c];
                sb[pos] = nv[c];
            }
            m += __popcll(bal);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's compacted lists (its own LDS)
        __builtin_amdgcn_wave_barrier();
        for (int j = lane; j < m; j += 64) slot_pts[base + j] = sb[j];
        for (int off = 32; off >= 1; off >>= 1) it += __shfl_xor(it, off, 64);
        const SimilarityFit f = wave_fit_similarity(sa, sb, m, lane);
        if (lane == 0) {
            slot_counts[E.slot] = m;
            FitOut o;
            o.n = m;
            o.npts = cnt;
            o.iters = it;
            o.valid = 0;
            o.cx = o.cy = 0.0;
            o.scale = 0.0;
            if (m >= min_fit && m > 0 && f.ok) {
                const double cx0 = E.x + E.w / 2, cy0 = E.y + E.h / 2;
                o.cx = f.p * cx0 - f.q * cy0 + f.tx;
                o.cy = f.q * cx0 + f.p * cy0 + f.ty;
                o.scale = sqrt(f.p * f.p + f.q * f.q);
                o.valid = (o.scale > 0.5 && o.scale < 2.0 && isfinite(o.cx) && isfinite(o.cy)) ? 1 : 0;
            }
            if (flag && wg_pub) s_out[wv] = o;
            else out[e] = o;
        }
        // without wg_pub every wave that wrote a FitOut releases it at system
        // scope itself: the workgroup barrier below orders waves only at
        // workgroup scope, and thread 0's release waits only for its own wave's
        // stores (each release writes the XCD's L2 back)
        if (flag && !wg_pub) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    // wg_pub: every wave waits until its own global stores (compacted slot
    // points, slot count) are acknowledged by the L2 before the workgroup
    // barrier, so wave 0's single system-scope release after it (an L2
    // write-back of every dirty line) covers all eight waves' stores.  Without
    // this wait a wave's stores could still be in flight when the release runs:
    // the barrier orders the waves at workgroup scope only.  The look-ahead
    // PyrLK on another stream reads them once the host sees the flag, with no
    // kernel boundary in between.
    if (flag && wg_pub) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    if (flag) {
        // publish: after the workgroup's barrier one thread counts the
        // workgroup's results at system scope; the last workgroup resets the
        // count for the next launch (stream-ordered) and raises the frame's tag
        __syncthreads();
        const int first = blockIdx.x * kFitWaves;
        const int nin = nents - first < kFitWaves ? nents - first : kFitWaves;
        if (wg_pub && threadIdx.x < 64) {  // wave 0 stores the workgroup's results and releases them once
            if ((int)threadIdx.x < nin) out[first + threadIdx.x] = s_out[threadIdx.x];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
        if (threadIdx.x == 0) {
            // the workgroup's results were released above (system scope: wave 0's
            // fence, or every wave's own); the count itself is relaxed, and the
            // last workgroup's acquire fence pairs with those release fences
            // (fence-fence synchronisation through the count's release sequence)
            // before its release store of the flag, which the host acquires
            if (!wg_pub) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // the waves' releases, cumulated by the barrier
            const unsigned prev =
                __hip_atomic_fetch_add(fit_cnt, (unsigned)nin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev + (unsigned)nin == (unsigned)nents) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                *fit_cnt = 0u;
                __hip_atomic_store(flag, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// The loop's launch worker (ctx option tbd_async_la): a host thread that issues
// the look-ahead PyrLK launches (the speculative one after the fit sync, the
// post-tracker one at the end of the step) while the loop's own thread goes on
// with the tracker step and the next frame.  Those launches feed no result back
// to the host within the step, so each is a job handed over in FIFO order; the
// loop drains the queue (waits for every posted job) before any host call that
// depends on what a job enqueued: a wait on la_done, a launch on the look-ahead
// stream, the end of a public call.  A HIP launch costs 2.4-3.4 us of host time
//  and the speculative block ~6-14 us, all of it on the frame's
// host chain between the fit and the next critical PyrLK launch.
class LaunchWorker {
public:
    explicit LaunchWorker(int device) : device_(device), th_([this] { run(); }) {}
    ~LaunchWorker()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    // queue f (runs on the worker, in posting order)
    void post(std::function<int()> f)
    {
        while (head_.load(std::memory_order_relaxed) - tail_.load(std::memory_order_acquire) >= kJobs)
            __builtin_ia32_pause();
        jobs_[head_.load(std::memory_order_relaxed) % kJobs] = std::move(f);
        head_.fetch_add(1, std::memory_order_seq_cst);  // seq_cst pair with run()'s sleeping_ / head_
        if (sleeping_.load(std::memory_order_seq_cst)) {
            std::lock_guard<std::mutex> lk(mu_);
            cv_.notify_one();
        }
    }
    // wait until every posted job has run; the first error since the last drain
    int drain()
    {
        while (tail_.load(std::memory_order_acquire) != head_.load(std::memory_order_relaxed)) __builtin_ia32_pause();
        return err_.exchange(TBDK_OK);
    }

private:
    static constexpr unsigned kJobs = 8;
    static constexpr double kSpinUs = 1000.0;  // spin this long for the next job, then sleep
    void run()
    {
        (void)hipSetDevice(device_);
        using clk = std::chrono::steady_clock;
        auto idle0 = clk::now();
        for (;;) {
            const unsigned tl = tail_.load(std::memory_order_relaxed);
            if (head_.load(std::memory_order_acquire) != tl) {
                const int r = jobs_[tl % kJobs]();
                jobs_[tl % kJobs] = nullptr;
                if (r != TBDK_OK) {
                    int ok = TBDK_OK;
                    err_.compare_exchange_strong(ok, r);
                }
                tail_.store(tl + 1, std::memory_order_release);
                idle0 = clk::now();
                continue;
            }
            if (std::chrono::duration<double, std::micro>(clk::now() - idle0).count() < kSpinUs) {
                for (int p = 0; p < 16; ++p) __builtin_ia32_pause();
                continue;
            }
            std::unique_lock<std::mutex> lk(mu_);
            sleeping_.store(true, std::memory_order_seq_cst);
            cv_.wait(lk, [&] { return stop_ || head_.load(std::memory_order_seq_cst) != tail_.load(std::memory_order_relaxed); });
            sleeping_.store(false, std::memory_order_relaxed);
            if (stop_ && head_.load(std::memory_order_acquire) == tail_.load(std::memory_order_relaxed)) return;
            idle0 = clk::now();
        }
    }
    int device_;
    std::function<int()> jobs_[kJobs];
    std::atomic<unsigned> head_{0}, tail_{0};
    std::atomic<int> err_{TBDK_OK};
    std::atomic<bool> sleeping_{false};
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    std::thread th_;  // last: started once the members above exist
};

}  // namespace tbdk

using namespace tbdk;

struct tbdk_tbd {
    tbdk_ctx* ctx = nullptr;
    LaunchWorker* worker = nullptr;  // ctx option tbd_async_la (read by tbdk_tbd_create)
    tbdk_tbd_config cfg;
    // three pyramids in rotation: this frame's (cur), the previous frame's and
    // the look-ahead frame's, so the look-ahead build never overwrites a
    // pyramid this step's PyrLK still reads
    tbdk_pyr pyr[3];
    // each pyramid's own level-0 buffer; inside tbdk_tbd_run (ctx option
    // tbd_borrow_l0) level 0 is the caller's frame itself, whose pointer stays
    // valid for the whole call, and the padded copy is not made
    tbdk_level own_l0[3];
    bool borrow = false;
    int cur = 0;
    bool last_fit = false;  // the previous step ran PyrLK and synced on its fit
    bool have_prev = false;
    tbd::Tracker* tracker = nullptr;
    tbdk_trajectories* traj = nullptr;  // caller-owned; records per-object tracking results
    // device
    float2* slot_pts = nullptr;
    float2* slot_next = nullptr;
    uint8_t* slot_status = nullptr;
    int32_t* slot_iters = nullptr;
    int32_t* slot_counts = nullptr;
    FitEntry* d_ents = nullptr;
    FitInline fit_inl;  // this step's fit table as kernel arguments
    FitOut* d_fit = nullptr;
    GfttRoi* d_tab = nullptr;  // device mirror of h_tab
    // post-tracker work (the GFTT of refreshed sets the early GFTT missed) runs on `side`, so the next
    // frame's pyramid, enqueued on the caller's stream, overlaps it; the
    // caller's stream waits for `post_done` before its LK launch
    hipStream_t side = nullptr;
    hipEvent_t post_done = nullptr;
    // what the next step's refreshed-set PyrLK waits for: post_done, or (ctx
    // option tbd_post_direct, no post-tracker GFTT) the early GFTT's own event
    hipEvent_t post_wait = nullptr;
    // look-ahead (tbdk_tbd_step_ahead): the next frame's pyramid, enqueued
    // behind this frame's fit (built while the host tracks), and the next
    // frame's PyrLK of the point sets this step leaves unchanged, enqueued
    // behind the post-tracker GFTT
    hipEvent_t fit_done = nullptr;   // this frame's predictions are on the host
    hipEvent_t la_ready = nullptr;   // look-ahead pyramid complete (recorded on the step's stream)
    hipEvent_t lk_issued = nullptr;  // tbd_la_pyr_side: this step's PyrLK launches (on the step's stream) done
    hipEvent_t step_begin = nullptr; // tbd_la_pyr_side 2: the caller's work on the step's stream before the step
    hipEvent_t la_done = nullptr;    // look-ahead PyrLK complete (recorded on la_s)
    // the look-ahead PyrLK runs on its own stream behind the GFTT eigenvalue
    // kernel, so the refreshed sets' PyrLK of the next step (caller's stream)
    // does not queue behind it; only the fit waits for it
    hipStream_t la_s = nullptr;
    hipEvent_t eig_done = nullptr;   // this step's GFTT eigenvalue kernel complete (on `side`)
    int32_t* h_la = nullptr;         // look-ahead slot list (pinned) / device copy
    int32_t* d_la = nullptr;
    std::vector<int> la_list;        // the la_member slots
    std::vector<char> la_member;     // slot tracked by the look-ahead PyrLK
    // speculative look-ahead PyrLK, launched before the tracker step for the
    // sets that will stay unchanged unless the tracker deletes the track (n >=
    // min_points, KLT prediction inside the bounds filter, no re-detection
    // frame): [slots] pinned / device, membership
    int32_t* h_spec = nullptr;
    int32_t* d_spec = nullptr;
    // look-ahead PyrLK of this step's early GFTT rows (option tbd_early_la): the
    // rows it tracked into the next frame (ers_row), which the next step's
    // refreshed-set PyrLK then skips; their staged list
    std::vector<char> ers_row;
    std::vector<int> ers_list;
    int32_t* h_ers = nullptr;
    int32_t* d_ers = nullptr;
    std::vector<int> spec_list;
    std::vector<char> spec_member;
    const uint8_t* la_frame = nullptr;
    int la_pitch = 0;
    hipStream_t la_stream = nullptr;
    bool la_pyr = false;             // pyr[cur] already holds la_frame's pyramid
    bool la_lk = false;              // ... and the la_member slots are tracked into it
    int la_defer_n = 0;              // look-ahead PyrLK left to the next step (h_la's first la_defer_n slots)
    bool la_defer_eig = false;       // ... behind the post-tracker GFTT's eigenvalue kernel
    // pinned host staging (reuse rules: see tbdk_tbd_step)
    // [fit entries: S FitEntry][LK slot lists: S int32 (unchanged sets, then refreshed ones)]
    void* h_pre = nullptr;
    void* d_pre = nullptr;
    int32_t* h_lists = nullptr;
    int32_t* d_lists = nullptr;
    std::vector<char> refreshed;  // slot got new corners in the last post phase
    std::vector<int32_t> b_list;  // scratch: refreshed slots in track order
    FitEntry* h_ents = nullptr;
    FitOut* h_fit = nullptr;
    // the post-tracker GFTT's ROI table (pinned; uploaded, or read in place)
    GfttRoi* h_tab = nullptr;
    // GFTT rows: the corner sets of refreshed tracks stay where GFTT writes them
    // and are tracked from there; the next fit compacts the tracked points into
    // the slot.  Rows of the slot arrays: [0, S) slots, [S, 4S) the early GFTT's
    // rows (three sets by step, eb: this step's, eb + 1 the next frame's GFTT
    // launched ahead, eb + 2 the previous step's, read by this step's PyrLK and
    // fit), [4S, 5S) the post-tracker GFTT's rows.  src_row[slot] = the
    // refreshed set's row until the next fit.
    std::vector<int> src_row;
    std::vector<int> src_list;
    // early GFTT (see the top of the file): ROI tables by row set (pinned; a
    // table is rewritten three steps later, after fit syncs that order its
    // upload), device table, corner rows and counts
    GfttRoi* h_etab[kEarlySets] = {nullptr, nullptr, nullptr};
    GfttRoi* d_etab = nullptr;
    int eb = 0;  // early-row set of this step
    std::vector<tbdk_roi> erois;                  // this step's early ROIs
    FlatMap<uint64_t> erow_of;                    // ROI box -> early corner row
    // the next frame's early GFTT launched ahead by tbdk_tbd_run (ctx option
    // tbd_gftt_ahead): the new-track ROIs of that frame's detections, in row set
    // eb + 1, over the caller's frame; the step of that frame takes them over
    // and launches only the ROIs they miss (re-detection guesses)
    int ahead_id = INT_MIN;
    const uint8_t* ahead_frame = nullptr;
    int ahead_pitch = 0;
    int ahead_set = -1;                           // row set of an ahead launch not yet taken over
    bool ahead_any = false;                       // an ahead launch in this tbdk_tbd_run call
    hipEvent_t ahead_tail = nullptr;              // tbdk_tbd_run's end: the early stream's work on its frames
    std::vector<tbdk_roi> ahead_rois;
    FlatMap<uint64_t> ahead_row_of;
    std::vector<int> det_order;                   // scratch: detections by left edge
    GfttScratch gftt;   // the early GFTT's (early_s); the loop's own, not the context's
    GfttScratch gftt2;  // the post-tracker GFTT's (side), so the next step's early GFTT need not wait for it
    hipEvent_t pyr_ready = nullptr;               // this step's pyramid built on the step's stream
    // zero-copy staging: the kernels read the pinned host tables (fit entries,
    // slot lists, GFTT ROI tables) and the fit kernel
    // writes its results to pinned host memory directly, through device
    // mappings of the coherent pinned buffers; no copy is issued (d_pre, d_fit,
    // d_tab, d_la, d_spec, d_etab are those mappings, not device allocations)
    bool zc = false;
    // fit completion by flag (zero copy, option tbd_fit_flag): the fit's last
    // wave stores the frame's tag to h_flag (through its mapping d_flag) at
    // system scope; d_fitcnt counts the finished waves
    bool fit_flag = false;
    int32_t* h_flag = nullptr;
    int32_t* d_flag = nullptr;
    unsigned* d_fitcnt = nullptr;
    int fit_tag = 0;
    hipStream_t early_s = nullptr;                // lowest priority: off the critical path
    bool own_side = false, own_la = false, own_early = false;  // created here, not the context's
    hipEvent_t early_done[kEarlySets] = {nullptr, nullptr, nullptr};  // per row set: its last GFTT launch done
    // host bookkeeping; slots are handed out lowest-first so the LK launch
    // covers only [0, max live slot] x 256 points
    std::priority_queue<int, std::vector<int>, std::greater<int>> free_slots;
    FlatMap<unsigned> slot_of;                     // track id -> slot
    FlatMap<unsigned> npts_of;                     // track id -> corners after last fit
    std::vector<tbd::Detection> dets;
    std::vector<tbd::Prediction> preds;
    std::vector<tbdk_roi> rois;
    // tbdk_tbd_run_host: uploaded frames, a ring of three device frames filled
    // on `up_s` two frames ahead; copied[k] = ring[k] holds its frame,
    // freed[k] = the steps that read ring[k] (its pyramid) are enqueued before it
    uint8_t* ring[3] = {nullptr, nullptr, nullptr};
    int ring_pitch = 0;
    hipStream_t up_s = nullptr;
    hipEvent_t copied[3] = {nullptr, nullptr, nullptr};
    hipEvent_t freed[3] = {nullptr, nullptr, nullptr};
};

namespace {

// Cross-stream edge: stream s waits for event ev only while ev's work is still
// pending.  A wait enqueues a barrier packet that the consumer queue's
// packet processor resolves before the next kernel starts; work that is
// complete when the edge is enqueued needs none (its results are visible to
// every later dispatch).  Event completion is monotonic, so the query cannot
// skip a wait that is needed.
hipError_t wait_if_pending(hipStream_t s, hipEvent_t ev)
{
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return hipSuccess;
    if (q != hipErrorNotReady) return q;
    return hipStreamWaitEvent(s, ev, 0);
}

inline uint64_t box_key(int x, int y, int w, int h)
{
    return ((uint64_t)(uint16_t)x << 48) | ((uint64_t)(uint16_t)y << 32) | ((uint64_t)(uint16_t)w << 16) |
           (uint64_t)(uint16_t)h;
}

// the launch worker's queue drained (a no-op without the worker): the first
// error of a posted job, else TBDK_OK
inline int drain(tbdk_tbd* t) { return t->worker ? t->worker->drain() : TBDK_OK; }

// run f now, or (launch worker) post it
inline int run_or_post(tbdk_tbd* t, std::function<int()> f)
{
    if (!t->worker) return f();
    t->worker->post(std::move(f));
    return TBDK_OK;
}

// a frame's pyramid into P: borrowed level 0 inside tbdk_tbd_run (levels 1..
// only), else the padded copy (a pyramid that was borrowed gets its own level
// 0 buffer back first)
int build_pyr(tbdk_tbd* t, const uint8_t* img, int pitch, tbdk_pyr& P, hipStream_t s)
{
    const int i = (int)(&P - t->pyr);
    if (t->borrow) return pyr_build_borrowed(t->ctx, img, pitch, &P, s);
    if (P.flags & kPyrL0Borrowed) {
        P.lv[0] = t->own_l0[i];
        P.flags &= ~kPyrL0Borrowed;
    }
    return tbdk_pyr_build(t->ctx, img, pitch, &P, s);
}

// the end of a borrowing tbdk_tbd_run: the pyramid the next step reads as its
// previous frame's gets its level 0 copied into its own buffer (the caller's
// frame may go away after the call); the others only point at their own
// buffers again (each is rebuilt before it is read)
int end_borrow(tbdk_tbd* t, hipStream_t s)
{
    if (!t->borrow) return TBDK_OK;
    t->borrow = false;
    int rc = TBDK_OK;
    for (int i = 0; i < 3; ++i) {
        tbdk_pyr& P = t->pyr[i];
        if (!(P.flags & kPyrL0Borrowed)) continue;
        if (i == (t->cur + 2) % 3 && t->have_prev) {
            const int r = pyr_restore_l0(t->ctx, &P, t->own_l0[i], s);
            if (rc == TBDK_OK) rc = r;
        } else {
            P.lv[0] = t->own_l0[i];
            P.flags &= ~kPyrL0Borrowed;
        }
    }
    // the last step's GFTT (early / post-tracker streams) still reads a frame:
    // the caller's stream waits for it, so synchronising that stream covers
    // every read of the caller's frames
    if (rc == TBDK_OK && t->post_wait) rc = map_status(wait_if_pending(s, t->post_wait));
    return rc;
}

int release(tbdk_tbd* t)
{
    if (!t) return TBDK_OK;
    if (t->worker) {  // every posted launch issued before the streams are synchronised
        (void)t->worker->drain();
        delete t->worker;
        t->worker = nullptr;
    }
    if (t->side) (void)hipStreamSynchronize(t->side);
    if (t->post_done) (void)hipEventDestroy(t->post_done);
    if (t->fit_done) (void)hipEventDestroy(t->fit_done);
    if (t->la_s) (void)hipStreamSynchronize(t->la_s);
    if (t->la_done) (void)hipEventDestroy(t->la_done);
    if (t->la_ready) (void)hipEventDestroy(t->la_ready);
    if (t->lk_issued) (void)hipEventDestroy(t->lk_issued);
    if (t->step_begin) (void)hipEventDestroy(t->step_begin);
    if (t->la_s && t->own_la) (void)hipStreamDestroy(t->la_s);
    if (t->eig_done) (void)hipEventDestroy(t->eig_done);
    if (t->side && t->own_side) (void)hipStreamDestroy(t->side);
    for (int i = 0; i < 3; ++i)
        if (t->pyr[i].storage) tbdk_pyr_destroy(t->ctx, &t->pyr[i]);
    if (t->pyr_ready) (void)hipEventDestroy(t->pyr_ready);
    if (t->early_s) (void)hipStreamSynchronize(t->early_s);
    if (t->early_s && t->own_early) (void)hipStreamDestroy(t->early_s);
    for (hipEvent_t& ev : t->early_done)
        if (ev) (void)hipEventDestroy(ev);
    if (t->ahead_tail) (void)hipEventDestroy(t->ahead_tail);
    gftt_scratch_free(t->gftt);
    gftt_scratch_free(t->gftt2);
    if (t->up_s) (void)hipStreamSynchronize(t->up_s);
    for (int k = 0; k < 3; ++k) {
        if (t->freed[k]) (void)hipEventSynchronize(t->freed[k]);
        if (t->ring[k]) (void)hipFree(t->ring[k]);
        if (t->copied[k]) (void)hipEventDestroy(t->copied[k]);
        if (t->freed[k]) (void)hipEventDestroy(t->freed[k]);
    }
    if (t->up_s) (void)hipStreamDestroy(t->up_s);
    void* dev[] = {t->slot_pts, t->slot_next, t->slot_status, t->slot_iters, t->slot_counts, t->d_fitcnt};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    if (!t->zc) {
        void* staged[] = {t->d_pre, t->d_fit, t->d_tab, t->d_la, t->d_etab, t->d_spec, t->d_ers};
        for (void* p : staged)
            if (p) (void)hipFree(p);
    }
    void* host[] = {t->h_pre, t->h_fit, t->h_tab, t->h_la, t->h_etab[0], t->h_spec, t->h_flag, t->h_ers};
    for (void* p : host)
        if (p) (void)hipHostFree(p);
    delete t->tracker;
    delete t;
    return TBDK_OK;
}

}  // namespace

extern "C" {

int tbdk_tbd_default_config(int width, int height, tbdk_tbd_config* c)
{
    if (!c || width <= 0 || height <= 0) return TBDK_EINVAL;
    std::memset(c, 0, sizeof(*c));
    c->width = width;
    c->height = height;
    c->win = 21;
    c->max_level = 2;  // "3-level PyrLK" (levels - 1)
    c->lk_iters = 30;
    c->lk_epsilon = 0.01;
    c->min_eig_threshold = 1e-4f;
    c->max_corners = 256;
    c->quality_level = 0.01;
    c->min_distance = 3.0;
    c->redetect_every = 5;
    c->min_points = 32;
    c->min_fit_points = 4;
    c->cost_of_non_assignment = 10.0;
    c->time_window_size = 16;
    c->track_age_threshold = 4;
    c->track_visibility_threshold = 0.3;
    c->track_confidence_threshold = 0.2;
    c->bounds_xmin = 0;
    c->bounds_xmax = 1280;
    c->bounds_ymin = 0;
    c->bounds_ymax = 720;
    c->max_tracks = 1024;
    c->use_klt = 1;
    return TBDK_OK;
}

int tbdk_tbd_create(tbdk_ctx* ctx, const tbdk_tbd_config* cfg, tbdk_tbd** out)
{
    if (!ctx || !cfg || !out) return TBDK_EINVAL;
    *out = nullptr;
    if (cfg->max_corners <= 0 || cfg->max_corners > kSlotPts || cfg->max_tracks <= 0 || cfg->win < 3 ||
        cfg->win > 31 || cfg->redetect_every <= 0 || cfg->time_window_size <= 0 ||
        cfg->time_window_size > (int)tbd::kMaxTimeWindow)
        return TBDK_EINVAL;
    tbdk_tbd* t = new (std::nothrow) tbdk_tbd();
    if (!t) return TBDK_ENOMEM;
    t->ctx = ctx;
    t->cfg = *cfg;
    std::memset(t->pyr, 0, sizeof(t->pyr));
    int rc = TBDK_OK;
    for (int i = 0; i < 3 && rc == TBDK_OK; ++i)
        // levels only: PyrLK derives the window's Scharr values itself, so the
        // build writes no derivative planes (ctx option tbd_pyr_derivs = 1: with
        // the planes, for A/B runs; same results)
        rc = ctx->opt_tbd_pyr_derivs
                 ? tbdk_pyr_create(ctx, cfg->width, cfg->height, cfg->max_level, cfg->win, cfg->win, &t->pyr[i])
                 : tbdk_pyr_create_levels(ctx, cfg->width, cfg->height, cfg->max_level, cfg->win, cfg->win, &t->pyr[i]);
    if (rc != TBDK_OK) {
        release(t);
        return rc;
    }
    for (int i = 0; i < 3; ++i) t->own_l0[i] = t->pyr[i].lv[0];
    const size_t S = (size_t)cfg->max_tracks;
    hipError_t e = hipSuccess;
    auto dm = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, bytes);
        if (e == hipSuccess) e = hipMemset(*p, 0, bytes);
    };
    t->zc = ctx->opt_tbd_zero_copy != 0;
    auto hm = [&](void** p, size_t bytes) {
        if (e == hipSuccess)
            e = hipHostMalloc(p, bytes, t->zc ? hipHostMallocMapped | hipHostMallocCoherent : hipHostMallocDefault);
    };
    // a staged table: its device copy, or (zero-copy) the mapping of the pinned buffer
    auto sm = [&](void** d, void* h, size_t bytes) {
        if (e != hipSuccess) return;
        if (t->zc) e = hipHostGetDevicePointer(d, h, 0);
        else dm(d, bytes);
    };
    // 4 S rows: the slots, two sets of early GFTT rows, the post-tracker GFTT rows
    dm(reinterpret_cast<void**>(&t->slot_pts), sizeof(float2) * kRowSets * S * kSlotPts);
    dm(reinterpret_cast<void**>(&t->slot_next), sizeof(float2) * kRowSets * S * kSlotPts);
    dm(reinterpret_cast<void**>(&t->slot_status), kRowSets * S * kSlotPts);
    dm(reinterpret_cast<void**>(&t->slot_iters), sizeof(int32_t) * kRowSets * S * kSlotPts);
    dm(reinterpret_cast<void**>(&t->slot_counts), sizeof(int32_t) * kRowSets * S);
    const size_t pre_bytes = (sizeof(FitEntry) + sizeof(int32_t)) * S;
    hm(&t->h_pre, pre_bytes);
    hm(reinterpret_cast<void**>(&t->h_fit), sizeof(FitOut) * S);
    hm(reinterpret_cast<void**>(&t->h_tab), sizeof(GfttRoi) * S);
    hm(reinterpret_cast<void**>(&t->h_la), sizeof(int32_t) * S);
    hm(reinterpret_cast<void**>(&t->h_spec), sizeof(int32_t) * S);
    hm(reinterpret_cast<void**>(&t->h_ers), sizeof(int32_t) * S);
    hm(reinterpret_cast<void**>(&t->h_etab[0]), kEarlySets * sizeof(GfttRoi) * S);
    for (int k = 1; k < kEarlySets; ++k)
        if (t->h_etab[0]) t->h_etab[k] = t->h_etab[0] + (size_t)k * S;
    sm(&t->d_pre, t->h_pre, pre_bytes);
    sm(reinterpret_cast<void**>(&t->d_fit), t->h_fit, sizeof(FitOut) * S);
    sm(reinterpret_cast<void**>(&t->d_tab), t->h_tab, sizeof(GfttRoi) * S);
    sm(reinterpret_cast<void**>(&t->d_la), t->h_la, sizeof(int32_t) * S);
    sm(reinterpret_cast<void**>(&t->d_spec), t->h_spec, sizeof(int32_t) * S);
    sm(reinterpret_cast<void**>(&t->d_ers), t->h_ers, sizeof(int32_t) * S);
    sm(reinterpret_cast<void**>(&t->d_etab), t->h_etab[0], kEarlySets * sizeof(GfttRoi) * S);
    t->fit_flag = t->zc && ctx->opt_tbd_fit_flag != 0;
    if (t->fit_flag) {
        hm(reinterpret_cast<void**>(&t->h_flag), 64);
        sm(reinterpret_cast<void**>(&t->d_flag), t->h_flag, 64);
        dm(reinterpret_cast<void**>(&t->d_fitcnt), 64);
        if (e == hipSuccess) __atomic_store_n(t->h_flag, 0, __ATOMIC_RELEASE);
    }
    if (t->h_pre && t->d_pre) {
        t->h_ents = static_cast<FitEntry*>(t->h_pre);
        t->h_lists = reinterpret_cast<int32_t*>(t->h_ents + S);
        t->d_ents = static_cast<FitEntry*>(t->d_pre);
        t->d_lists = reinterpret_cast<int32_t*>(t->d_ents + S);
    }
    t->refreshed.assign((size_t)S, 0);
    t->la_member.assign((size_t)S, 0);
    t->spec_member.assign((size_t)S, 0);
    t->ers_row.assign((size_t)kRowSets * S, 0);
    t->b_list.assign((size_t)S, 0);
    t->src_row.assign((size_t)S, -1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->pyr_ready, hipEventDisableTiming);
    // the post-tracker GFTT heads the next frame's critical path (the refreshed
    // sets' PyrLK waits for it): it gets the highest priority, ahead of the
    // look-ahead PyrLK it shares the device with
    int prio_least = 0, prio_greatest = 0;
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    if (e == hipSuccess) {  // the context's loop streams, made by its first loop (see tbdk_ctx::tbd_side)
        std::lock_guard<std::mutex> lk(ctx->tbd_mu);
        if (!ctx->tbd_side && hipStreamCreateWithPriority(&ctx->tbd_side, hipStreamNonBlocking, prio_greatest) != hipSuccess)
            ctx->tbd_side = nullptr;
        if (!ctx->tbd_la && hipStreamCreateWithPriority(&ctx->tbd_la, hipStreamNonBlocking, prio_least) != hipSuccess)
            ctx->tbd_la = nullptr;
        if (!ctx->tbd_early && hipStreamCreateWithPriority(&ctx->tbd_early, hipStreamNonBlocking, prio_least) != hipSuccess)
            ctx->tbd_early = nullptr;
    }
    // the context's streams when it has them (see tbdk_ctx::tbd_side), else our own
    if (e == hipSuccess && ctx->tbd_side) t->side = ctx->tbd_side;
    else if (e == hipSuccess && (e = hipStreamCreateWithPriority(&t->side, hipStreamNonBlocking, prio_greatest)) == hipSuccess)
        t->own_side = true;
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->post_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->fit_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->la_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->la_ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->lk_issued, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->step_begin, hipEventDisableTiming);
    // the look-ahead PyrLK at the lowest priority (on gfx950 the range is
    // normal..high, so this is the default; a high-priority caller stream for
    // the critical PyrLK measured no difference either)
    if (e == hipSuccess && ctx->tbd_la) t->la_s = ctx->tbd_la;
    else if (e == hipSuccess && (e = hipStreamCreateWithPriority(&t->la_s, hipStreamNonBlocking, prio_least)) == hipSuccess)
        t->own_la = true;
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->eig_done, hipEventDisableTiming);
    // the early GFTT at the lowest priority (ctx option tbd_early_prio, read here:
    // 1 = the highest, for launch orders that put it behind the critical PyrLK)
    if (e == hipSuccess && ctx->tbd_early && !ctx->opt_tbd_early_prio) {
        t->early_s = ctx->tbd_early;
    } else if (e == hipSuccess) {
        e = hipStreamCreateWithPriority(&t->early_s, hipStreamNonBlocking,
                                        ctx->opt_tbd_early_prio ? prio_greatest : prio_least);
        if (e == hipSuccess) t->own_early = true;
    }
    for (hipEvent_t& ev : t->early_done)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->ahead_tail, hipEventDisableTiming);
    if (e != hipSuccess) {
        release(t);
        return map_status(e);
    }
    tbd::TbdArgs a;
    a.costOfNonAssignment = cfg->cost_of_non_assignment;
    a.timeWindowSize = (unsigned)cfg->time_window_size;
    a.trackAgeThreshold = (unsigned)cfg->track_age_threshold;
    a.trackVisibilityThreshold = cfg->track_visibility_threshold;
    a.trackConfidenceThreshold = cfg->track_confidence_threshold;
    a.shouldStoreMetrics = true;
    a.boundsXmin = cfg->bounds_xmin;
    a.boundsXmax = cfg->bounds_xmax;
    a.boundsYmin = cfg->bounds_ymin;
    a.boundsYmax = cfg->bounds_ymax;
    t->tracker = new (std::nothrow) tbd::Tracker(a);
    if (!t->tracker) {
        release(t);
        return TBDK_ENOMEM;
    }
    for (int s = 0; s < cfg->max_tracks; ++s) t->free_slots.push(s);
    // at most max_tracks live entries each (tracks holding a slot; early ROIs)
    t->slot_of = FlatMap<unsigned>(4 * (size_t)cfg->max_tracks);
    t->npts_of = FlatMap<unsigned>(4 * (size_t)cfg->max_tracks);
    t->erow_of = FlatMap<uint64_t>(4 * (size_t)cfg->max_tracks);
    t->ahead_row_of = FlatMap<uint64_t>(4 * (size_t)cfg->max_tracks);
    if (ctx->opt_tbd_async_la) {
        t->worker = new (std::nothrow) LaunchWorker(ctx->device);
        if (!t->worker) {
            release(t);
            return TBDK_ENOMEM;
        }
    }
    rc = gftt_reserve(t->gftt, ctx->device, cfg->max_tracks, (int64_t)cfg->width * cfg->height * 2);
    if (rc == TBDK_OK) rc = gftt_reserve(t->gftt2, ctx->device, cfg->max_tracks, (int64_t)cfg->width * cfg->height * 2);
    if (rc != TBDK_OK) {
        release(t);
        return rc;
    }
    *out = t;
    return TBDK_OK;
}

int tbdk_tbd_destroy(tbdk_tbd* t) { return release(t); }

int tbdk_tbd_set_trajectories(tbdk_tbd* t, tbdk_trajectories* traj)
{
    if (!t) return TBDK_EINVAL;
    t->traj = traj;
    return TBDK_OK;
}

int tbdk_tbd_tracking_write(tbdk_tbd* t, const uint32_t* history_ages, int nages, int frame_count, const char* path,
                            int log_switches, tbdk_scenario_metrics* out)
{
    if (!t || !t->traj || nages < 0 || (nages > 0 && !history_ages) || frame_count < 0) return TBDK_EINVAL;
    std::vector<unsigned> ages(history_ages, history_ages + nages);
    return app::write_tracking_output(*t->tracker, ages, t->traj->map, (unsigned)frame_count, path,
                                      log_switches ? stdout : nullptr, out)
               ? TBDK_OK
               : TBDK_EINVAL;
}

}  // extern "C"

namespace {

// Host-phase profile of step_impl (probe builds, -DTBDK_STEP_PROFILE): the
// time between successive marks, summed over steps, read by
// tbdk_probe_step_profile (tools/probe_step_host.py)
#ifdef TBDK_STEP_PROFILE
constexpr int kStepMarks = 12;
double g_step_prof[kStepMarks];
long g_step_prof_n = 0;
#define STEP_MARK(i) (sp_t[(i)] = std::chrono::steady_clock::now(), sp_set[(i)] = true)
// sub-segments of the speculative PyrLK block: SUB_MARK(k) adds the time since
// the previous SUB_MARK (or SUB_START) to g_sub_prof[k]
double g_sub_prof[8];
long g_sub_n = 0;
#define SUB_START() (sub_t0 = std::chrono::steady_clock::now())
#define SUB_MARK(k)                                                                                          \
    do {                                                                                                     \
        const auto sub_t1 = std::chrono::steady_clock::now();                                                \
        g_sub_prof[(k)] += std::chrono::duration<double, std::micro>(sub_t1 - sub_t0).count();             \
        sub_t0 = sub_t1;                                                                                     \
    } while (0)
#else
#define STEP_MARK(i) ((void)0)
#define SUB_START() ((void)0)
#define SUB_MARK(k) ((void)0)
#endif

// One frame.  With next != nullptr the step also enqueues look-ahead work for
// the next frame: its pyramid behind this frame's fit (the device has it to run
// while the host tracker runs), and its PyrLK of the unchanged point sets
// behind the post-tracker GFTT; the next step skips what was done.
int step_impl(tbdk_tbd* t, const uint8_t* frame, int pitch, int frame_id, const tbdk_detection* dets, int ndets,
              const uint8_t* next, int next_pitch, tbdk_frame_metrics* metrics, hipStream_t s,
              const tbdk_detection* next_dets = nullptr, int next_ndets = -1)
{
    if (!t || !frame || ndets < 0 || (ndets > 0 && !dets) || pitch < t->cfg.width ||
        (next && next_pitch < t->cfg.width))
        return TBDK_EINVAL;
    using clk = std::chrono::steady_clock;
    const auto t_step0 = clk::now();
#ifdef TBDK_STEP_PROFILE
    clk::time_point sp_t[kStepMarks];
    bool sp_set[kStepMarks] = {};
    sp_t[0] = t_step0;
    sp_set[0] = true;
    clk::time_point sub_t0 = t_step0;
#endif
    double launch_us = 0.0;
    const tbdk_tbd_config& c = t->cfg;
    tbdk_pyr& P = t->pyr[t->cur];
    tbdk_pyr& Pprev = t->pyr[(t->cur + 2) % 3];
    (void)hipSetDevice(t->ctx->device);
    int rc = TBDK_OK;

    // ---- the previous step's look-ahead, if it was for this frame
    const bool la_valid = t->la_pyr && t->la_frame == frame && t->la_pitch == pitch;
    const bool had_la_lk = t->la_lk;
    const bool la_lk = la_valid && had_la_lk;


    if (t->la_pyr && t->la_stream != s) {  // the look-ahead pyramid was built on another stream
        hipError_t e = wait_if_pending(s, t->la_ready);
        if (e != hipSuccess) return map_status(e);
    }
    if (had_la_lk && !la_valid) {  // discarded: it may still read the pyramid about to be rebuilt
        rc = drain(t);
        if (rc != TBDK_OK) return rc;
        hipError_t e = wait_if_pending(s, t->la_done);
        if (e != hipSuccess) return map_status(e);
    }
    t->la_pyr = t->la_lk = false;
    // tbd_la_pyr_side 2 (the look-ahead pyramid enqueued right after this
    // step's critical PyrLK): mark the caller's work on s before this step
    const bool early_pyr = next && t->ctx->opt_tbd_la_pyr_side == 2 && t->last_fit;
    if (early_pyr) {
        const hipError_t e = hipEventRecord(t->step_begin, s);
        if (e != hipSuccess) return map_status(e);
    }
    if (!la_valid) {
        rc = build_pyr(t, frame, pitch, P, s);
        if (rc != TBDK_OK) return rc;
        hipError_t e = hipEventRecord(t->pyr_ready, s);
        if (e != hipSuccess) return map_status(e);
    }
    const tbdk_gftt_params gp{c.max_corners, c.quality_level, c.min_distance, 3};
    if (c.use_klt && t->ctx->opt_tbd_early_gftt) {
        // the early GFTT stream: behind this frame's pyramid (recorded where it
        // was built; the wait is taken now, before this step re-records la_ready
        // for the next frame).  It need not wait for the previous step's
        // post-tracker GFTT (scratch of its own), and the early rows it writes
        // (set eb) were last read two steps ago, before a fit this host synced.
        hipError_t e = wait_if_pending(t->early_s, la_valid ? t->la_ready : t->pyr_ready);
        if (e != hipSuccess) return map_status(e);
    }

    // ---- early GFTT over the detections that will start new tracks: every
    // detection before the first tracks exist, else those beyond the tracker's
    // bounds filter (a track on them is predicted there and deleted before the
    // assignment).  On the low-priority `early_s`, launched first in the step
    // (it is needed only after the tracker step, and overlaps this step's
    // PyrLK and fit); the
    // post-tracker phase takes its corners for every refreshed set whose box
    // equals one of these ROIs.
    const int S = c.max_tracks;
    const int erow0 = S * (1 + t->eb);  // this step's early GFTT rows (see tbdk_tbd::src_row)
    // the ROIs the previous step launched ahead for this frame (tbd_gftt_ahead):
    // this step's early ROIs start with them, in their rows
    const bool ahead_in = t->ahead_id == frame_id && t->ahead_frame == frame && t->ahead_pitch == pitch;
    if (ahead_in) {
        std::swap(t->erois, t->ahead_rois);
        std::swap(t->erow_of, t->ahead_row_of);
    } else {
        t->erois.clear();
        t->erow_of.clear();
        if (t->ahead_set == t->eb) {  // launched for another frame: it may still read this set's pinned table
            const hipError_t e = hipEventSynchronize(t->early_done[t->eb]);
            if (e != hipSuccess) return map_status(e);
        }
    }
    t->ahead_id = INT_MIN;
    t->ahead_set = -1;
    bool early_launched = ahead_in && !t->erois.empty();
    // one launch of the early GFTT over rois[0, n) into row set `set` from row
    // `row0` on, over the image at img (the pinned table at h_etab[set] + tab0)
    auto early_launch = [&](const tbdk_roi* rois, int n, int set, int tab0, const uint8_t* img, int ipitch) -> int {
        GfttPlan eplan;
        GfttRoi* htab = t->h_etab[set] + tab0;
        int rc2 = gftt_prepare(rois, n, c.width, c.height, &gp, htab, &eplan);
        if (rc2 != TBDK_OK) return rc2;
        hipStream_t es = t->early_s;  // ordered at the top of the step
        const GfttRoi* dtab = t->zc ? t->d_etab + (htab - t->h_etab[0]) : t->d_etab;
        if (!t->zc) {
            hipError_t e = hipMemcpyAsync(t->d_etab, htab, sizeof(GfttRoi) * n, hipMemcpyHostToDevice, es);
            if (e != hipSuccess) return map_status(e);
        }
        const int row0 = S * (1 + set) + tab0;
        rc2 = gftt_launch(t->ctx, t->gftt, img, ipitch, dtab, eplan, &gp,
                          reinterpret_cast<float*>(t->slot_pts + (size_t)row0 * kSlotPts), t->slot_counts + row0, es,
                          nullptr, kSlotPts, htab);
        if (rc2 != TBDK_OK) return rc2;
        return map_status(hipEventRecord(t->early_done[set], es));
    };
    auto launch_early_gftt = [&]() -> int {
        if (!c.use_klt || !t->ctx->opt_tbd_early_gftt) return TBDK_OK;
        const size_t n0 = t->erois.size();  // taken over from the ahead launch
        const bool all_new = t->tracker->getTracks().empty();
        for (int i = 0; i < ndets && (int)t->erois.size() < c.max_tracks; ++i) {
            const tbdk_detection& d = dets[i];
            const bool beyond = d.x >= c.bounds_xmax || d.y >= c.bounds_ymax || d.x + d.width < c.bounds_xmin ||
                                d.y + d.height < c.bounds_ymin;
            if (!all_new && !beyond) continue;
            const int x0 = std::max(d.x, 0), y0 = std::max(d.y, 0);
            const int x1 = std::min(d.x + d.width, c.width), y1 = std::min(d.y + d.height, c.height);
            if (x1 - x0 < 3 || y1 - y0 < 3) continue;
            if (!t->erow_of.insert(box_key(x0, y0, x1 - x0, y1 - y0), (int)t->erois.size())) continue;
            t->erois.push_back(tbdk_roi{x0, y0, x1 - x0, y1 - y0});
        }
        // re-detection frames: every existing track's set is refreshed in its box
        // after updateAssignedTracks (tbd.cpp:948-965), which depends only on the
        // assigned detection and the track's box history; speculate the detection
        // of largest overlap with the track's last box and GFTT that box early
        // (a track assigned otherwise, or not at all, takes the post-tracker GFTT)
        if (t->ctx->opt_tbd_early_gftt >= 2 && !all_new && frame_id % c.redetect_every == 0 && ndets > 0) {
            auto& order = t->det_order;
            order.resize((size_t)ndets);
            int maxw = 0;
            for (int i = 0; i < ndets; ++i) {
                order[(size_t)i] = i;
                maxw = std::max(maxw, dets[i].width);
            }
            std::sort(order.begin(), order.end(), [&](int a, int b) { return dets[a].x < dets[b].x; });
            for (const auto& tr : t->tracker->getTracks()) {
                if ((int)t->erois.size() >= c.max_tracks) break;
                if (!t->slot_of.find(tr.id)) continue;
                const tbd::Rect& lb = tr.bboxes.back();
                if (lb.x >= c.bounds_xmax || lb.y >= c.bounds_ymax) continue;  // deleted by the bounds filter
                auto lo = std::lower_bound(order.begin(), order.end(), lb.x - maxw,
                                           [&](int a, int x) { return dets[a].x < x; });
                int best = -1;
                double bo = 0.0;
                for (auto it = lo; it != order.end() && dets[*it].x <= lb.x + lb.width; ++it) {
                    const tbdk_detection& d = dets[*it];
                    const double o = tbd::computeBoundingBoxOverlap(lb, tbd::Rect(d.x, d.y, d.width, d.height));
                    if (o > bo) {
                        bo = o;
                        best = *it;
                    }
                }
                if (best < 0) continue;
                const tbdk_detection& d = dets[best];
                const unsigned nprior = tr.historyLength < 4 ? (unsigned)tr.historyLength : 4u;
                unsigned wsum = 0, hsum = 0;
                for (unsigned k = tr.bboxes.size() - nprior; k < tr.bboxes.size(); ++k) {
                    wsum += tr.bboxes[k].width;
                    hsum += tr.bboxes[k].height;
                }
                const int w = (int)((wsum + d.width) / (nprior + 1)), h = (int)((hsum + d.height) / (nprior + 1));
                const tbd::Rect r = tbd::rect_from_point2d((double)d.x + (d.width / 2 - w / 2),
                                                           (double)d.y + (d.height / 2 - h / 2), w, h);
                const int x0 = std::max(r.x, 0), y0 = std::max(r.y, 0);
                const int x1 = std::min(r.x + r.width, c.width), y1 = std::min(r.y + r.height, c.height);
                if (x1 - x0 < 3 || y1 - y0 < 3) continue;
                if (!t->erow_of.insert(box_key(x0, y0, x1 - x0, y1 - y0), (int)t->erois.size())) continue;
                t->erois.push_back(tbdk_roi{x0, y0, x1 - x0, y1 - y0});
            }
        }
        if (t->erois.size() > n0) {  // the ROIs no ahead launch covered
            const tbdk_level& L0 = P.lv[0];
            const int r2 = early_launch(t->erois.data() + n0, (int)(t->erois.size() - n0), t->eb, (int)n0,
                                        L0.data + (size_t)L0.pad * L0.pitch + L0.pad, L0.pitch);
            if (r2 != TBDK_OK) return r2;
            early_launched = true;
        }
        return TBDK_OK;
    };
    // the next frame's new-track ROIs (its detections beyond the bounds filter,
    // as above), launched ahead over the caller's next frame into the next row
    // set: that frame's step takes them over, so its refreshed-set PyrLK no
    // longer waits for a GFTT launched one step before it (tbdk_tbd_run knows
    // the next frame's detections).  Where (ctx option tbd_ahead_at): 0 right
    // after this step's early launch, 1 after the critical PyrLK launch, 2 just
    // before the host waits for the fit (its host work off the frame's chain)
    bool ahead_done = false;
    auto launch_gftt_ahead = [&](int at) -> int {
        if (ahead_done || at < t->ctx->opt_tbd_ahead_at) return TBDK_OK;
        ahead_done = true;
        if (!c.use_klt || !t->ctx->opt_tbd_early_gftt) return TBDK_OK;
        const bool all_new = t->tracker->getTracks().empty();
        if (next && next_dets && next_ndets > 0 && t->ctx->opt_tbd_gftt_ahead && !all_new) {
            const int nb = (t->eb + 1) % kEarlySets;
            t->ahead_rois.clear();
            t->ahead_row_of.clear();
            for (int i = 0; i < next_ndets && (int)t->ahead_rois.size() < c.max_tracks; ++i) {
                const tbdk_detection& d = next_dets[i];
                const bool beyond = d.x >= c.bounds_xmax || d.y >= c.bounds_ymax || d.x + d.width < c.bounds_xmin ||
                                    d.y + d.height < c.bounds_ymin;
                if (!beyond) continue;
                const int x0 = std::max(d.x, 0), y0 = std::max(d.y, 0);
                const int x1 = std::min(d.x + d.width, c.width), y1 = std::min(d.y + d.height, c.height);
                if (x1 - x0 < 3 || y1 - y0 < 3) continue;
                if (!t->ahead_row_of.insert(box_key(x0, y0, x1 - x0, y1 - y0), (int)t->ahead_rois.size())) continue;
                t->ahead_rois.push_back(tbdk_roi{x0, y0, x1 - x0, y1 - y0});
            }
            if (!t->ahead_rois.empty()) {
                const int r2 = early_launch(t->ahead_rois.data(), (int)t->ahead_rois.size(), nb, 0, next, next_pitch);
                if (r2 != TBDK_OK) return r2;
                t->ahead_id = frame_id + 1;
                t->ahead_frame = next;
                t->ahead_pitch = next_pitch;
                t->ahead_set = nb;
                t->ahead_any = true;
            }
        }
        return TBDK_OK;
    };
    // ctx option tbd_early_order: 0 launches the early GFTT first in the step, 1
    // right after the critical (refreshed-set) PyrLK, 2 after the fit and the
    // next pyramid, just before the host waits (its host work then runs while
    // the device tracks; the early GFTT stream still waits for this frame's
    // pyramid, taken above)
    const int early_order = t->ctx->opt_tbd_early_order;
    if (early_order == 0) {
        rc = launch_early_gftt();
        if (rc == TBDK_OK) rc = launch_gftt_ahead(0);
        if (rc != TBDK_OK) return rc;
    }
    STEP_MARK(1);

    // No host wait here: the pinned staging buffers written before this step's
    // fit sync (h_ents, h_lists) were last read by uploads issued before the
    // previous step's sync, and those written after it (h_tab, h_la) are only
    // rewritten after this step's sync, which orders every
    // earlier upload.  So this frame's pyramid / LK / fit queue up behind the
    // previous GFTT.
    double wait_us = 0.0, gate_us = 0.0;  // gate: the host's wait before the fit launch (tbd_fit_gate)
    bool synced = false;  // has this step waited for the stream (see above)?

    // ---- KLT propagation of every live track.  Slots whose point set the previous
    // frame's post-tracker work (on `side`) leaves untouched are tracked first,
    // overlapping that work (or were tracked by the look-ahead); the refreshed
    // ones after it completes.
    std::vector<tbd::Track>& tracks = t->tracker->getTracks();
    int nents = 0, klt_points = 0, klt_pred = 0, lk_points = 0, nA = 0, nB = 0;
    bool merged = false;  // the unchanged and refreshed sets in one PyrLK launch
    bool pyr_enqueued = false;  // the look-ahead pyramid already enqueued (tbd_la_pyr_side 2)
    int64_t lk_iters = 0;
    t->preds.clear();
    const bool run_klt = c.use_klt && t->have_prev && !tracks.empty();
    tbdk_lk_params lp;
    lp.win_w = lp.win_h = c.win;
    lp.max_level = c.max_level;
    lp.max_count = c.lk_iters;
    lp.epsilon = c.lk_epsilon;
    lp.flags = 0;
    lp.min_eig_threshold = c.min_eig_threshold;
    lp.impl = 0;
    // the look-ahead PyrLK of the n unchanged sets in h_la, pyramid A -> B, on
    // la_s behind the look-ahead pyramid and (eig) the post-tracker GFTT's
    // eigenvalue kernel
    // (launch worker: posted; h_la, la_ready and eig_done are rewritten only
    // after a drain)
    auto launch_la = [&](int n, bool eig, tbdk_pyr& A, tbdk_pyr& B) -> int {
        const bool wait_ready = t->la_stream != t->la_s;
        tbdk_pyr* pa = &A;
        tbdk_pyr* pb = &B;
        return run_or_post(t, [t, n, eig, wait_ready, lp, pa, pb]() -> int {
            hipStream_t ls = t->la_s;
            hipError_t e = wait_ready ? wait_if_pending(ls, t->la_ready) : hipSuccess;
            if (e == hipSuccess && eig) e = wait_if_pending(ls, t->eig_done);
            if (e == hipSuccess && !t->zc)
                e = hipMemcpyAsync(t->d_la, t->h_la, sizeof(int32_t) * n, hipMemcpyHostToDevice, ls);
            if (e != hipSuccess) return map_status(e);
            const int r = lk_internal(t->ctx, pa, pb, reinterpret_cast<const float*>(t->slot_pts),
                                      reinterpret_cast<float*>(t->slot_next), t->slot_status, nullptr, t->slot_iters,
                                      n * kSlotPts, &lp, t->slot_counts, kSlotPts, ls, t->d_la, nullptr, t->h_la);
            if (r != TBDK_OK) return r;
            return map_status(hipEventRecord(t->la_done, ls));
        });
    };
    // the previous step's deferred look-ahead PyrLK (ctx option tbd_la_defer),
    // launched below once this step's critical PyrLK is; dropped with the look-ahead
    const int la_defer = la_lk ? t->la_defer_n : 0;
    t->la_defer_n = 0;
    if (run_klt) {
        for (const auto& tr : tracks) {
            const int* it = t->slot_of.find(tr.id);
            if (!it) continue;
            const int slot = *it;
            const tbd::Rect& b = tr.bboxes.back();
            const int src = t->src_row[(size_t)slot];
            t->h_ents[nents++] = FitEntry{slot, b.x, b.y, b.width, b.height, src};
            if (src >= 0) {  // refreshed: tracked from its GFTT row (unless the look-ahead did)
                if (!(la_lk && t->ers_row[(size_t)src])) t->b_list[nB++] = src;
            }
            else if (!(la_lk && t->la_member[(size_t)slot])) t->h_lists[nA++] = slot;
        }
        // refreshed sets after the unchanged ones (a separate scratch list: with
        // every slot live, nA + nB == S and the two ranges tile h_lists exactly)
        std::copy(t->b_list.begin(), t->b_list.begin() + nB, t->h_lists + nA);
        const size_t bytes = sizeof(FitEntry) * S + sizeof(int32_t) * (size_t)(nA + nB);
        if (!t->zc) {
            hipError_t e = hipMemcpyAsync(t->d_pre, t->h_pre, bytes, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) return map_status(e);
        }
        // the unchanged sets go first, overlapping the previous step's
        // post-tracker work; when that work is already complete (the first frame
        // of a run, steps without look-ahead) both kinds of sets wait for nothing
        // and one launch of nA + nB sets replaces two back-to-back ones
        merged = nA > 0 && nB > 0 && (!t->post_wait || hipEventQuery(t->post_wait) == hipSuccess);
        if (nA > 0 && !merged) {
            rc = lk_internal(t->ctx, &Pprev, &P, reinterpret_cast<const float*>(t->slot_pts),
                             reinterpret_cast<float*>(t->slot_next), t->slot_status, nullptr, t->slot_iters,
                             nA * kSlotPts, &lp, t->slot_counts, kSlotPts, s, t->d_lists, nullptr, t->h_lists);
            if (rc != TBDK_OK) return rc;
        }
    }
    for (int sl : t->la_list) t->la_member[(size_t)sl] = 0;
    t->la_list.clear();
    for (int r : t->ers_list) t->ers_row[(size_t)r] = 0;
    t->ers_list.clear();
    for (int sl : t->src_list) t->src_row[(size_t)sl] = -1;  // the fit compacts them into their slots
    t->src_list.clear();


    STEP_MARK(2);
    std::fill(t->refreshed.begin(), t->refreshed.end(), 0);
    {  // the previous step's early and post-tracker GFTT (their rows) before the refreshed sets
        hipError_t e = t->post_wait ? wait_if_pending(s, t->post_wait) : hipSuccess;
        if (e != hipSuccess) return map_status(e);
    }
    tbdk_pyr& Pnext = t->pyr[(t->cur + 1) % 3];  // the look-ahead pyramid: two frames back's buffer
    // side (ctx option tbd_la_pyr_side): built on the look-ahead stream behind
    // this step's PyrLK launches (lk_issued; they read the buffer it
    // overwrites), beside the fit, so the look-ahead PyrLK that follows it on
    // that stream needs no cross-stream edge
    auto enqueue_next_pyr = [&](bool side, bool wait = true) -> int {
        // the posted look-ahead launches first (they read la_ready; in stream
        // order on la_s ahead of this build, as without the worker)
        const int dr = drain(t);
        if (dr != TBDK_OK) return dr;
        hipStream_t ps = s;
        if (side) {
            ps = t->la_s;
            // without the wait for this step's PyrLK: behind the caller's work
            // on its stream before this step (the next frame's upload, say)
            const hipError_t e = wait ? hipStreamWaitEvent(ps, t->lk_issued, 0) : wait_if_pending(ps, t->step_begin);
            if (e != hipSuccess) return map_status(e);
        }
        t->la_frame = next;
        t->la_pitch = next_pitch;
        t->la_stream = ps;
        t->la_pyr = true;
        const int r = build_pyr(t, next, next_pitch, Pnext, ps);
        if (r != TBDK_OK) return r;
        return map_status(hipEventRecord(t->la_ready, ps));  // the next frame's pyramid (and this fit) done
    };
    if (run_klt) {
        if (nB > 0) {
            const int first = merged ? 0 : nA, nsets = merged ? nA + nB : nB;
            rc = lk_internal(t->ctx, &Pprev, &P, reinterpret_cast<const float*>(t->slot_pts),
                             reinterpret_cast<float*>(t->slot_next), t->slot_status, nullptr, t->slot_iters,
                             nsets * kSlotPts, &lp, t->slot_counts, kSlotPts, s, t->d_lists + first, nullptr,
                             t->h_lists + first);
            if (rc != TBDK_OK) return rc;
        }
        if (la_defer > 0) {
            rc = launch_la(la_defer, t->la_defer_eig, Pprev, P);
            if (rc != TBDK_OK) return rc;
        }
        // tbd_la_pyr_side 2: the look-ahead pyramid now, on the look-ahead
        // stream with no wait: its buffer held the pyramid of two frames back,
        // whose last readers (the previous step's PyrLK, the GFTT before it)
        // completed before the previous step's fit, which the host synced on
        if (early_pyr) {
            rc = enqueue_next_pyr(true, false);
            if (rc != TBDK_OK) return rc;
            pyr_enqueued = true;
        }
        STEP_MARK(3);
        if (early_order == 1) {
            rc = launch_early_gftt();
            if (rc != TBDK_OK) return rc;
        }
        if (early_order <= 1) {
            rc = launch_gftt_ahead(1);
            if (rc != TBDK_OK) return rc;
        }
        hipError_t e = hipSuccess;  // zero-copy without a look-ahead wait sets it nowhere below
        if (la_lk) {  // the fit reads the look-ahead PyrLK's results
            rc = drain(t);
            if (rc != TBDK_OK) return rc;
            if (t->ctx->opt_tbd_fit_gate) {
                // ctx option tbd_fit_gate: the host waits for the look-ahead PyrLK
                // and then launches the fit behind this step's PyrLK on the same
                // stream, with no cross-queue barrier packet between them (the
                // packet cost ~15 us after the PyrLK ended, on the critical chain;
                // the look-ahead launch usually ends well before this one)
                const auto tg0 = clk::now();
                while ((e = hipEventQuery(t->la_done)) == hipErrorNotReady) {
                    for (int p = 0; p < 16; ++p) __builtin_ia32_pause();
                    if (std::chrono::duration<double, std::micro>(clk::now() - tg0).count() > 2000.0) {
                        e = hipEventSynchronize(t->la_done);  // not the per-frame case
                        break;
                    }
                }
                if (e != hipSuccess) return map_status(e);
                gate_us = std::chrono::duration<double, std::micro>(clk::now() - tg0).count();
            } else {
                e = wait_if_pending(s, t->la_done);
                if (e != hipSuccess) return map_status(e);
            }
        }
        const bool pyr_side = next && !pyr_enqueued && t->ctx->opt_tbd_la_pyr_side;
        if (pyr_side) {
            e = hipEventRecord(t->lk_issued, s);
            if (e != hipSuccess) return map_status(e);
        }
        const bool by_flag = t->fit_flag && nents > 0;
        const int tag = by_flag ? ++t->fit_tag : 0;
        int inl = t->ctx->opt_tbd_fit_inline && nents <= kFitInline ? 1 : 0;
        for (int q = 0; q < nents && inl; ++q) {  // the table into the kernel arguments, if it fits
            const FitEntry& f = t->h_ents[q];
            const bool fits = f.slot >= 0 && f.slot <= 0xFFFF && f.src >= -0x8000 && f.src <= 0x7FFF &&
                              f.x >= -0x8000 && f.x <= 0x7FFF && f.y >= -0x8000 && f.y <= 0x7FFF && f.w >= 0 &&
                              f.w <= 0xFFFF && f.h >= 0 && f.h <= 0xFFFF;
            if (fits)
                t->fit_inl.e[q] = FitEntryC{(uint16_t)f.slot, (int16_t)f.src, (int16_t)f.x, (int16_t)f.y,
                                            (uint16_t)f.w, (uint16_t)f.h};
            else
                inl = 0;
        }
        int rec = timing_begin(t->ctx, "tbd_fit", s);
        hipLaunchKernelGGL(tbd_fit_kernel, dim3((nents + kFitWaves - 1) / kFitWaves), dim3(64 * kFitWaves), 0, s,
                           t->d_ents, nents, t->slot_pts, t->slot_next,
                           t->slot_status, t->slot_iters, t->slot_counts, t->d_fit, c.min_fit_points,
                           by_flag ? t->d_fitcnt : nullptr, by_flag ? t->d_flag : nullptr, tag, inl, t->fit_inl,
                           t->ctx->opt_tbd_fit_wgpub);
        timing_end(t->ctx, rec, s);
        if (!t->zc) e = hipMemcpyAsync(t->h_fit, t->d_fit, sizeof(FitOut) * nents, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && !by_flag) e = hipEventRecord(t->fit_done, s);
        if (e != hipSuccess) return map_status(e);
        if (next && !pyr_enqueued) {  // runs on the device while this step waits for the fit and tracks
            rc = enqueue_next_pyr(pyr_side);
            if (rc != TBDK_OK) return rc;
        }
        if (early_order == 2) {
            rc = launch_early_gftt();
            if (rc != TBDK_OK) return rc;
        }
        rc = launch_gftt_ahead(2);
        if (rc != TBDK_OK) return rc;
        auto ts0 = clk::now();
        STEP_MARK(4);
        launch_us = std::chrono::duration<double, std::micro>(ts0 - t_step0).count() - gate_us;
        wait_us += gate_us;
        // the one host wait of the frame, on the critical path: poll instead of
        // a blocking synchronize (its wake-up latency is part of every frame).
        // The poll pauses between queries (the core's sibling thread keeps its
        // issue slots) and gives up the core after kSpinUs: a fit that takes
        // that long is not the per-frame case, and a blocking wait then costs
        // nothing that matters.  One host core per loop while it spins
        // (threading).
        // Past kYieldUs (several times a frame's fit wait) each poll gives the
        // core away once (sched_yield), so ranks sharing a host's cores (8 GPUs,
        // a CPU share each) do not starve each other's tracker threads.
        constexpr double kSpinUs = 2000.0, kYieldUs = 300.0;
        auto pause_or_yield = [&](double us) {
            if (us > kYieldUs) sched_yield();
            else
                for (int p = 0; p < 16; ++p) __builtin_ia32_pause();
        };
        if (by_flag) {
            // the fit's flag; past kSpinUs the stream is synchronized (it holds
            // the fit, then the next pyramid) and the flag read once more
            e = hipSuccess;
            while (__atomic_load_n(t->h_flag, __ATOMIC_ACQUIRE) != tag) {
                const double us = std::chrono::duration<double, std::micro>(clk::now() - ts0).count();
                pause_or_yield(us);
                if (us > kSpinUs) {
                    e = hipStreamSynchronize(s);
                    if (e == hipSuccess && __atomic_load_n(t->h_flag, __ATOMIC_ACQUIRE) != tag) e = hipErrorUnknown;
                    break;
                }
            }
        } else {
            while ((e = hipEventQuery(t->fit_done)) == hipErrorNotReady) {
                const double us = std::chrono::duration<double, std::micro>(clk::now() - ts0).count();
                pause_or_yield(us);
                if (us > kSpinUs) {
                    e = hipEventSynchronize(t->fit_done);
                    break;
                }
            }
        }
        wait_us += std::chrono::duration<double, std::micro>(clk::now() - ts0).count();
        if (e != hipSuccess) return map_status(e);
        synced = true;
        STEP_MARK(5);
        for (int k = 0; k < nents; ++k) {
            const FitOut& o = t->h_fit[k];
            // map back: entries were filled in track order, skipping slotless tracks
            klt_points += o.n;
            lk_points += o.npts;
            lk_iters += o.iters;
        }
        int k = 0;
        for (const auto& tr : tracks) {
            if (!t->slot_of.find(tr.id)) continue;
            const FitOut& o = t->h_fit[k++];
            t->npts_of.set(tr.id, o.n);
            if (o.valid) {
                t->preds.push_back(tbd::Prediction{tr.id, 1, o.cx, o.cy});
                klt_pred++;
            }
        }
        STEP_MARK(6);
        // ---- speculative look-ahead PyrLK (see tbdk_tbd::spec_list): runs while the
        // host tracks; the post-tracker phase adds the unchanged sets it missed
        if (next && t->ctx->opt_tbd_spec_la && frame_id % c.redetect_every != 0) {
            SUB_START();
            rc = drain(t);  // h_spec is rewritten below
            if (rc != TBDK_OK) return rc;
            int ns = 0;
            k = 0;
            for (const auto& tr : tracks) {
                const int* it = t->slot_of.find(tr.id);
                if (!it) continue;
                const FitOut& o = t->h_fit[k++];
                if (o.n < c.min_points || !o.valid) continue;
                const tbd::Rect& bb = tr.bboxes.back();  // predictNewLocationsOfTracks + filterTracksOutOfBounds
                const tbd::Rect r =
                    tbd::rect_from_point2d(o.cx - bb.width / 2, o.cy - bb.height / 2, bb.width, bb.height);
                if (r.x + r.width < c.bounds_xmin || r.x >= c.bounds_xmax || r.y + r.height < c.bounds_ymin ||
                    r.y >= c.bounds_ymax)
                    continue;
                t->h_spec[ns++] = *it;
            }
            SUB_MARK(0);
            if (ns > 0) {
                // (launch worker: posted, so the tracker step below starts now)
                const bool wait_ready = t->la_stream != t->la_s;
                tbdk_pyr* pa = &P;
                tbdk_pyr* pb = &Pnext;
                rc = run_or_post(t, [t, ns, wait_ready, lp, pa, pb]() -> int {
                    hipStream_t ls = t->la_s;
                    hipError_t e2 = wait_ready ? wait_if_pending(ls, t->la_ready) : hipSuccess;
                    if (e2 == hipSuccess && !t->zc)
                        e2 = hipMemcpyAsync(t->d_spec, t->h_spec, sizeof(int32_t) * ns, hipMemcpyHostToDevice, ls);
                    if (e2 != hipSuccess) return map_status(e2);
                    const int r = lk_internal(t->ctx, pa, pb, reinterpret_cast<const float*>(t->slot_pts),
                                              reinterpret_cast<float*>(t->slot_next), t->slot_status, nullptr,
                                              t->slot_iters, ns * kSlotPts, &lp, t->slot_counts, kSlotPts, ls,
                                              t->d_spec, nullptr, t->h_spec);
                    if (r != TBDK_OK) return r;
                    return map_status(hipEventRecord(t->la_done, ls));
                });
                if (rc != TBDK_OK) return rc;
                SUB_MARK(3);
                for (int q = 0; q < ns; ++q) {
                    t->spec_member[(size_t)t->h_spec[q]] = 1;
                    t->spec_list.push_back(t->h_spec[q]);
                }
                t->la_lk = true;
                SUB_MARK(4);
#ifdef TBDK_STEP_PROFILE
                g_sub_n++;
#endif
            }
        }
        // ---- look-ahead PyrLK of this step's early GFTT rows (option
        // tbd_early_la; 1: re-detection frames, where the speculative PyrLK above
        // does not run and the device would idle through the host tracker step,
        // 2: every frame).  Each early row is the corner set a track refreshed in
        // this step's ROI will be tracked from in the next step (new tracks, the
        // re-detection guesses the tracker confirms), so the next step's PyrLK
        // of the refreshed sets skips the rows tracked here: the same points, the
        // same pyramids (this frame's and the look-ahead), the same results.
        const int ela = t->ctx->opt_tbd_early_la;
        const int ne = (int)t->erois.size();
        if (next && early_launched && ne > 0 && (ela >= 2 || (ela == 1 && frame_id % c.redetect_every == 0))) {
            rc = drain(t);  // la_s and la_done from this thread below
            if (rc != TBDK_OK) return rc;
            for (int q = 0; q < ne; ++q) t->h_ers[q] = erow0 + q;
            hipStream_t ls = t->la_s;
            e = t->la_stream == ls ? hipSuccess : wait_if_pending(ls, t->la_ready);
            if (e == hipSuccess) e = wait_if_pending(ls, t->early_done[t->eb]);
            if (e == hipSuccess && !t->zc)
                e = hipMemcpyAsync(t->d_ers, t->h_ers, sizeof(int32_t) * ne, hipMemcpyHostToDevice, ls);
            if (e != hipSuccess) return map_status(e);
            rc = lk_internal(t->ctx, &P, &Pnext, reinterpret_cast<const float*>(t->slot_pts),
                             reinterpret_cast<float*>(t->slot_next), t->slot_status, nullptr, t->slot_iters,
                             ne * kSlotPts, &lp, t->slot_counts, kSlotPts, ls, t->d_ers, nullptr, t->h_ers);
            if (rc != TBDK_OK) return rc;
            e = hipEventRecord(t->la_done, ls);
            if (e != hipSuccess) return map_status(e);
            for (int q = 0; q < ne; ++q) {
                t->ers_row[(size_t)(erow0 + q)] = 1;
                t->ers_list.push_back(erow0 + q);
            }
            t->la_lk = true;
        }
    } else {
        if (early_order != 0) {
            rc = launch_early_gftt();
            if (rc != TBDK_OK) return rc;
        }
        rc = launch_gftt_ahead(2);
        if (rc != TBDK_OK) return rc;
        if (next) {
            // the next pyramid is rebuilt over the previous frame's, which the
            // previous step's look-ahead PyrLK (on la_s) may still be reading
            if (had_la_lk) {
                rc = drain(t);
                if (rc != TBDK_OK) return rc;
                hipError_t e = wait_if_pending(s, t->la_done);
                if (e != hipSuccess) return map_status(e);
            }
            rc = enqueue_next_pyr(false);
            if (rc != TBDK_OK) return rc;
        }
    }

    STEP_MARK(7);
    // ---- host tracker step (cv::tbd::Tracker::performTrackingStep)
    t->dets.resize((size_t)ndets);
    for (int i = 0; i < ndets; ++i) {
        tbd::Detection& d = t->dets[i];
        d.id = dets[i].id;
        d.frame_id = frame_id;
        d.bbox = tbd::Rect(dets[i].x, dets[i].y, dets[i].width, dets[i].height);
        d.confidence = dets[i].confidence;
    }
    auto tt0 = clk::now();
    if (t->traj) app::add_positions(t->traj->map, t->dets, frame_id);
    t->tracker->performTrackingStep(t->dets, frame_id, t->preds.data(), (int)t->preds.size(),
                                    t->traj ? &t->traj->map : nullptr);
    const double tracker_us = std::chrono::duration<double, std::micro>(clk::now() - tt0).count();
    STEP_MARK(8);
    if (!synced) {  // no fit this step: order the previous step's uploads before reusing h_tab
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return map_status(e);
    }
    for (unsigned id : t->tracker->deletedIds) {
        if (const int* it = t->slot_of.find(id)) {
            t->free_slots.push(*it);
            t->slot_of.erase(id);
        }
        t->npts_of.erase(id);
    }
    // ---- corners for new tracks and tracks due for re-detection: each such set
    // is its GFTT row (an early row when the early GFTT ran on its box, else a
    // row of the post-tracker GFTT below), tracked from there by the next step
    t->rois.clear();
    int nroi = 0, nearly = 0;
    const int prow0 = (1 + kEarlySets) * S;  // the post-tracker GFTT's rows
    if (c.use_klt) {
        for (const auto& tr : t->tracker->getTracks()) {
            const int* it = t->slot_of.find(tr.id);
            bool is_new = !it;
            int slot;
            if (is_new) {
                if (t->free_slots.empty()) continue;  // slot pool exhausted: track runs on the motion model
                slot = t->free_slots.top();
                t->free_slots.pop();
                t->slot_of.set(tr.id, slot);
            } else {
                slot = *it;
                const int* np = t->npts_of.find(tr.id);
                const int n = np ? *np : 0;
                if (frame_id % c.redetect_every != 0 && n >= c.min_points) continue;
            }
            const tbd::Rect& b = tr.bboxes.back();
            int x0 = std::max(b.x, 0), y0 = std::max(b.y, 0);
            int x1 = std::min(b.x + b.width, c.width), y1 = std::min(b.y + b.height, c.height);
            t->refreshed[(size_t)slot] = 1;
            t->npts_of.set(tr.id, c.max_corners);  // refreshed at the next fit
            t->src_list.push_back(slot);
            if (x1 - x0 < 3 || y1 - y0 < 3) {  // nothing to detect in: empty point set
                t->rois.push_back(tbdk_roi{0, 0, 1, 1});
            } else {
                if (const int* er = t->erow_of.find(box_key(x0, y0, x1 - x0, y1 - y0))) {
                    // the early GFTT ran on this ROI of this frame
                    t->src_row[(size_t)slot] = erow0 + *er;
                    nearly++;
                    continue;
                }
                t->rois.push_back(tbdk_roi{x0, y0, x1 - x0, y1 - y0});
            }
            t->src_row[(size_t)slot] = prow0 + nroi++;
        }
    }
    STEP_MARK(9);
    // ---- the post-tracker GFTT (side stream, behind the early GFTT whose rows
    // the next step reads and whose scratch it reuses).  With a next frame, the
    // PyrLK of the point sets this leaves unchanged is enqueued after it (the
    // look-ahead PyrLK): the GFTT heads the next frame's critical path, so it is
    // queued first and the PyrLK fills the device around it.
    // tbd_post_direct: with no post-tracker GFTT the next step waits for the
    // early GFTT's event itself (no side-stream wait and marker on the host's
    // way to that step; each early row set has its own event, so the next
    // step's early launches, whatever their order, re-record other sets' events)
    const bool post_direct = nroi == 0 && early_launched && t->ctx->opt_tbd_post_direct;
    if (early_launched && !post_direct) {
        hipError_t e = wait_if_pending(t->side, t->early_done[t->eb]);
        if (e != hipSuccess) return map_status(e);
    }
    if (nroi > 0) {
        GfttPlan plan;
        rc = gftt_prepare(t->rois.data(), nroi, c.width, c.height, &gp, t->h_tab, &plan);
        if (rc != TBDK_OK) return rc;
        if (!t->zc) {
            hipError_t e = hipMemcpyAsync(t->d_tab, t->h_tab, sizeof(GfttRoi) * nroi, hipMemcpyHostToDevice, t->side);
            if (e != hipSuccess) return map_status(e);
        }
        const tbdk_level& L0 = P.lv[0];
        rc = gftt_launch(t->ctx, t->gftt2, L0.data + (size_t)L0.pad * L0.pitch + L0.pad, L0.pitch, t->d_tab, plan, &gp,
                         reinterpret_cast<float*>(t->slot_pts + (size_t)prow0 * kSlotPts), t->slot_counts + prow0,
                         t->side, next ? t->eig_done : nullptr, kSlotPts, t->h_tab);
        if (rc != TBDK_OK) return rc;
    }
    // post_done also after an early GFTT none of whose ROIs was used: the next
    // step's fit sync then orders that GFTT's table upload before the staging
    // table is rewritten (two steps later)
    if (post_direct) {
        t->post_wait = t->early_done[t->eb];
    } else if (nroi > 0 || early_launched) {
        hipError_t e = hipEventRecord(t->post_done, t->side);
        if (e != hipSuccess) return map_status(e);
        t->post_wait = t->post_done;
    }
    STEP_MARK(10);
    // ---- look-ahead: PyrLK of the next frame for every live track whose point
    // set was not refreshed just now (exactly the next step's unchanged sets)
    if (next) {
        if (c.use_klt && !t->tracker->getTracks().empty()) {
            int n = 0;  // unchanged sets the speculative PyrLK did not cover
            for (const auto& tr : t->tracker->getTracks()) {
                const int* it = t->slot_of.find(tr.id);
                if (!it || t->refreshed[(size_t)*it]) continue;
                t->la_member[(size_t)*it] = 1;
                t->la_list.push_back(*it);
                if (!t->spec_member[(size_t)*it]) t->h_la[n++] = *it;
            }
            if (n > 0) {
                // on la_s, after the fit and the pyramid (la_ready) and behind the
                // GFTT eigenvalue kernel: its many large workgroups would otherwise
                // wait for the long-lived PyrLK waves to drain
                if (t->ctx->opt_tbd_la_defer) {
                    // launched by the next step right after its critical PyrLK
                    // (off the host chain between this fit and that launch)
                    t->la_defer_n = n;
                    t->la_defer_eig = nroi > 0;
                } else {
                    rc = launch_la(n, nroi > 0, P, Pnext);
                    if (rc != TBDK_OK) return rc;
                }
                t->la_lk = true;
            }
        }
    }
    for (int sl : t->spec_list) t->spec_member[(size_t)sl] = 0;
    t->spec_list.clear();
    t->cur = (t->cur + 1) % 3;
    t->last_fit = run_klt && synced;
    t->eb = (t->eb + 1) % kEarlySets;
    t->have_prev = true;

    STEP_MARK(11);
#ifdef TBDK_STEP_PROFILE
    {  // segments between consecutive marks that were both reached
        int prev = 0;
        bool all = true;
        for (int i = 1; i < kStepMarks; ++i) all = all && sp_set[i];
        if (all) {
            for (int i = 1; i < kStepMarks; ++i) {
                g_step_prof[i] += std::chrono::duration<double, std::micro>(sp_t[i] - sp_t[prev]).count();
                prev = i;
            }
            g_step_prof_n++;
        }
    }
#endif
    if (metrics) {
        const tbd::Tracker& tk = *t->tracker;
        metrics->tp = tk.truePositives.back();
        metrics->fn = tk.falseNegatives.back();
        metrics->fp = tk.falsePositives.back();
        metrics->gt = tk.groundTruths.back();
        metrics->matches = tk.numMatches.back();
        metrics->bbox_overlap = tk.bboxOverlap.back();
        metrics->ntracks = (int)t->tracker->getTracks().size();
        metrics->klt_points = klt_points;
        metrics->lk_points = lk_points;
        metrics->lk_iters = lk_iters;
        metrics->early_gftt = nearly;
        metrics->klt_predicted = klt_pred;
        metrics->redetected = nroi + nearly;
        metrics->host_wait_us = (float)wait_us;
        metrics->host_tracker_us = (float)tracker_us;
        metrics->host_launch_us = (float)launch_us;
        metrics->host_step_us = (float)std::chrono::duration<double, std::micro>(clk::now() - t_step0).count();
    }
    return TBDK_OK;
}

// every public call returns with all of its work enqueued (the launch worker's
// queue drained): the caller may synchronise its streams or the device
int finish(tbdk_tbd* t, int rc)
{
    const int d = t ? drain(t) : TBDK_OK;
    return rc != TBDK_OK ? rc : d;
}

}  // namespace

extern "C" {

#ifdef TBDK_STEP_PROFILE
// average us per profiled step of each segment [mark i-1, mark i) into out[1..];
// out[0] = the number of steps; the sums are reset
int tbdk_probe_step_profile(double* out, int cap)
{
    if (!out || cap < kStepMarks) return TBDK_EINVAL;
    out[0] = (double)g_step_prof_n;
    for (int i = 1; i < kStepMarks; ++i) {
        out[i] = g_step_prof_n ? g_step_prof[i] / g_step_prof_n : 0.0;
        g_step_prof[i] = 0.0;
    }
    g_step_prof_n = 0;
    if (cap >= kStepMarks + 6) {  // the speculative block's sub-segments, per block run
        out[kStepMarks] = (double)g_sub_n;
        for (int k = 0; k < 5; ++k) out[kStepMarks + 1 + k] = g_sub_n ? g_sub_prof[k] / g_sub_n : 0.0;
    }
    for (double& v : g_sub_prof) v = 0.0;
    g_sub_n = 0;
    return TBDK_OK;
}
#endif

int tbdk_tbd_step(tbdk_tbd* t, const uint8_t* frame, int pitch, int frame_id, const tbdk_detection* dets,
                  int ndets, tbdk_frame_metrics* metrics, void* stream)
{
    return finish(t, step_impl(t, frame, pitch, frame_id, dets, ndets, nullptr, 0, metrics,
                               static_cast<hipStream_t>(stream)));
}

int tbdk_tbd_step_ahead(tbdk_tbd* t, const uint8_t* frame, int pitch, int frame_id, const tbdk_detection* dets,
                        int ndets, const uint8_t* next_frame, int next_pitch, tbdk_frame_metrics* metrics,
                        void* stream)
{
    return finish(t, step_impl(t, frame, pitch, frame_id, dets, ndets, next_frame, next_pitch, metrics,
                               static_cast<hipStream_t>(stream)));
}

int tbdk_tbd_run(tbdk_tbd* t, const uint8_t* const* frames, int pitch, int first_frame_id,
                 const tbdk_detection* dets, const int32_t* det_offsets, int nframes, tbdk_frame_metrics* metrics,
                 void* stream)
{
    if (!t || nframes < 0 || (nframes > 0 && (!frames || !det_offsets))) return TBDK_EINVAL;
    for (int i = 0; i < nframes; ++i)
        if (!frames[i] || det_offsets[i + 1] < det_offsets[i] || det_offsets[i] < 0) return TBDK_EINVAL;
    if (nframes > 0 && det_offsets[nframes] > det_offsets[0] && !dets) return TBDK_EINVAL;
    // ctx option tbd_borrow_l0: the frames stay valid for the whole call, so
    // their pyramids take them as level 0 (derivative-plane pyramids excepted)
    hipStream_t s = static_cast<hipStream_t>(stream);
    t->borrow = t->ctx->opt_tbd_borrow_l0 && !t->ctx->opt_tbd_pyr_derivs && t->ctx->opt_pyr_fuse &&
                t->cfg.width >= 2 * (t->cfg.win + 2) && t->cfg.height >= 2 * (t->cfg.win + 2);
    t->ahead_any = false;
    // the caller's stream after the early GFTT work launched ahead over its frames
    auto end_ahead = [&]() -> int {
        if (!t->ahead_any) return TBDK_OK;
        t->ahead_any = false;
        hipError_t e = hipEventRecord(t->ahead_tail, t->early_s);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, t->ahead_tail, 0);
        return map_status(e);
    };
    for (int i = 0; i < nframes; ++i) {
        const uint8_t* next = i + 1 < nframes ? frames[i + 1] : nullptr;
        const bool nd = next && dets;
        int rc = step_impl(t, frames[i], pitch, first_frame_id + i, dets ? dets + det_offsets[i] : nullptr,
                           det_offsets[i + 1] - det_offsets[i], next, pitch, metrics ? metrics + i : nullptr, s,
                           nd ? dets + det_offsets[i + 1] : nullptr, nd ? det_offsets[i + 2] - det_offsets[i + 1] : -1);
        if (rc != TBDK_OK) {
            (void)finish(t, TBDK_OK);
            (void)end_ahead();
            (void)end_borrow(t, s);
            return rc;
        }
    }
    const int rc = finish(t, TBDK_OK);
    const int ra = end_ahead();
    const int rb = end_borrow(t, s);
    return rc != TBDK_OK ? rc : ra != TBDK_OK ? ra : rb;
}

int tbdk_tbd_run_host(tbdk_tbd* t, const uint8_t* const* frames, int pitch, int first_frame_id,
                      const tbdk_detection* dets, const int32_t* det_offsets, int nframes,
                      tbdk_frame_metrics* metrics, void* stream)
{
    if (!t || nframes < 0 || (nframes > 0 && (!frames || !det_offsets || pitch < t->cfg.width))) return TBDK_EINVAL;
    for (int i = 0; i < nframes; ++i)
        if (!frames[i] || det_offsets[i + 1] < det_offsets[i] || det_offsets[i] < 0) return TBDK_EINVAL;
    if (nframes > 0 && det_offsets[nframes] > det_offsets[0] && !dets) return TBDK_EINVAL;
    if (nframes == 0) return TBDK_OK;
    (void)hipSetDevice(t->ctx->device);
    const int W = t->cfg.width, H = t->cfg.height;
    hipError_t e = hipSuccess;
    if (!t->up_s) {  // the ring, its stream and events: once per loop
        t->ring_pitch = (W + 255) & ~255;
        for (int k = 0; k < 3 && e == hipSuccess; ++k) {
            e = hipMalloc(reinterpret_cast<void**>(&t->ring[k]), (size_t)t->ring_pitch * H + 256);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&t->copied[k], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&t->freed[k], hipEventDisableTiming);
        }
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&t->up_s, hipStreamNonBlocking);
        if (e != hipSuccess) return map_status(e);
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    // upload of frame j into ring[j % 3], behind the steps that last read that
    // buffer (freed: recorded after step j - 3, whose look-ahead built frame
    // j - 2's pyramid from ring[(j - 2) % 3], and whose own pyramid came from
    // ring[(j - 3) % 3])
    auto upload = [&](int j) -> hipError_t {
        const int k = j % 3;
        hipError_t r = hipStreamWaitEvent(t->up_s, t->freed[k], 0);
        if (r == hipSuccess)
            r = hipMemcpy2DAsync(t->ring[k], (size_t)t->ring_pitch, frames[j], (size_t)pitch, (size_t)W, (size_t)H,
                                 hipMemcpyHostToDevice, t->up_s);
        if (r == hipSuccess) r = hipEventRecord(t->copied[k], t->up_s);
        return r;
    };
    e = upload(0);
    if (e == hipSuccess && nframes > 1) e = upload(1);
    if (e != hipSuccess) return map_status(e);
    for (int i = 0; i < nframes; ++i) {
        // this step reads frame i (its pyramid, unless the previous step built
        // it) and frame i + 1 (the look-ahead pyramid)
        e = hipStreamWaitEvent(s, t->copied[i % 3], 0);
        if (e == hipSuccess && i + 1 < nframes) e = hipStreamWaitEvent(s, t->copied[(i + 1) % 3], 0);
        if (e == hipSuccess && i + 2 < nframes) e = upload(i + 2);  // ring[(i + 2) % 3] held frame i - 1
        if (e != hipSuccess) return map_status(e);
        const uint8_t* next = i + 1 < nframes ? t->ring[(i + 1) % 3] : nullptr;
        int rc = step_impl(t, t->ring[i % 3], t->ring_pitch, first_frame_id + i,
                           dets ? dets + det_offsets[i] : nullptr, det_offsets[i + 1] - det_offsets[i], next,
                           t->ring_pitch, metrics ? metrics + i : nullptr, s);
        if (rc != TBDK_OK) return finish(t, rc);
        e = hipEventRecord(t->freed[i % 3], s);
        if (e != hipSuccess) return finish(t, map_status(e));
    }
    return finish(t, TBDK_OK);
}

int tbdk_tbd_predictions(const tbdk_tbd* t, tbdk_prediction* out, int cap, int* n)
{
    if (!t || !n || cap < 0 || (cap > 0 && !out)) return TBDK_EINVAL;
    int k = 0;
    for (const auto& p : t->preds) {
        if (k >= cap) break;
        out[k++] = tbdk_prediction{p.id, p.valid, p.cx, p.cy};
    }
    *n = (int)t->preds.size();
    return TBDK_OK;
}

int tbdk_tbd_tracks(tbdk_tbd* t, tbdk_track_info* out, int cap, int* n)
{
    if (!t || !n || cap < 0 || (cap > 0 && !out)) return TBDK_EINVAL;
    const auto& tracks = t->tracker->getTracks();
    std::vector<int32_t> counts(kRowSets * (size_t)t->cfg.max_tracks);  // slots and GFTT rows
    if (const int d = drain(t)) return d;
    (void)hipSetDevice(t->ctx->device);
    hipError_t e = hipStreamSynchronize(t->side);  // post-tracker work (behind the early GFTT) runs on `side`
    if (e == hipSuccess && t->early_s) e = hipStreamSynchronize(t->early_s);  // the early GFTT rows (tbd_post_direct)
    if (e == hipSuccess) e = hipMemcpy(counts.data(), t->slot_counts, sizeof(int32_t) * counts.size(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return map_status(e);
    int k = 0;
    for (const auto& tr : tracks) {
        if (k >= cap) break;
        tbdk_track_info& o = out[k++];
        const tbd::Rect& b = tr.bboxes.back();
        o.id = tr.id;
        o.x = b.x;
        o.y = b.y;
        o.width = b.width;
        o.height = b.height;
        o.pred_x = tr.predPosition.x;
        o.pred_y = tr.predPosition.y;
        o.pred_w = tr.predPosition.width;
        o.pred_h = tr.predPosition.height;
        o.age = (int32_t)tr.age;
        o.total_visible = (int32_t)tr.totalVisibleCount;
        const int* it = t->slot_of.find(tr.id);
        if (!it) {
            o.npoints = 0;
        } else {  // a refreshed set is still its GFTT row
            const int src = t->src_row[(size_t)*it];
            o.npoints = std::max(0, counts[(size_t)(src >= 0 ? src : *it)]);
        }
        o.max_confidence = tr.maxConfidence;
        o.bbox_overlap = tr.bboxOverlap;
    }
    *n = (int)tracks.size();
    return TBDK_OK;
}

}  // extern "C"
