// runtime.hip — the C ABI of include/tbdk.h: contexts, pyramids, launches,
// per-kernel HIP-event timing.  Host code, compiled by hipcc for gfx950.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "synth_spec.h"
#include "tbdk_internal.hpp"

namespace tbdk {

static hipEvent_t take_event(tbdk_ctx* ctx)
{
    if (!ctx->free_events.empty()) {
        hipEvent_t e = ctx->free_events.back();
        ctx->free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

static uint64_t sample_hash(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// is `name` in the ",a,b," selection (no allocation: the launch sites call
// this once per launch while timing is on)
static bool timing_selected(const std::string& only, const char* name)
{
    const size_t n = std::strlen(name);
    for (size_t p = only.find(name); p != std::string::npos; p = only.find(name, p + 1))
        if (p > 0 && only[p - 1] == ',' && p + n < only.size() && only[p + n] == ',') return true;
    return false;
}

int timing_begin(tbdk_ctx* ctx, const char* name, hipStream_t s)
{
    if (!ctx->timing.load(std::memory_order_relaxed)) return -1;
    std::lock_guard<std::mutex> lk(ctx->timing_mu);
    if (!ctx->timing_only.empty() && !timing_selected(ctx->timing_only, name)) return -1;
    int64_t* calls = nullptr;
    for (auto& c : ctx->timing_calls)
        if (c.first == name) calls = &c.second;
    if (!calls) {
        ctx->timing_calls.emplace_back(name, 0);
        calls = &ctx->timing_calls.back().second;
    }
    // sampled: launch i is timed iff splitmix64(i) % N == 0 -- a pseudo-random 1/N
    // subset, so a per-frame pattern of differently sized launches (the TBD loop's
    // four PyrLK call sites) cannot line up with the sampling period
    if (sample_hash((uint64_t)(*calls)++) % (uint64_t)ctx->timing_every != 0) return -1;
    TimingRec r{name, take_event(ctx), take_event(ctx)};
    if (!r.begin || !r.end) return -1;
    (void)hipEventRecord(r.begin, s);
    ctx->recs.push_back(r);
    return (int)ctx->recs.size() - 1;
}

void timing_end(tbdk_ctx* ctx, int rec, hipStream_t s)
{
    if (rec < 0) return;
    hipEvent_t end;
    {
        std::lock_guard<std::mutex> lk(ctx->timing_mu);
        end = ctx->recs[rec].end;
    }
    (void)hipEventRecord(end, s);
}

static int map_err(hipError_t e)
{
    if (e == hipSuccess) return TBDK_OK;
    if (e == hipErrorOutOfMemory) return TBDK_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return TBDK_ENODEV;
    return TBDK_EHIP;
}

int map_status(hipError_t e) { return map_err(e); }

}  // namespace tbdk

using namespace tbdk;

extern "C" {

const char* tbdk_version(void) { return "tbdk 0.1 (gfx950)"; }

int tbdk_abi_version(void) { return TBDK_ABI_VERSION; }

int tbdk_ctx_create(int device, tbdk_ctx** out)
{
    if (!out) return TBDK_EINVAL;
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return TBDK_ENODEV;
    if (device < 0 || device >= n) return TBDK_ENODEV;
    tbdk_ctx* c = new (std::nothrow) tbdk_ctx();
    if (!c) return TBDK_ENOMEM;
    c->device = device;
    {
        DeviceGuard g(device);
        // best effort, side streams first (HOG and Farneback create what is missing
        // on first use): Farneback's prep stream, then the default HOG lanes, so
        // that with 4 hardware queues neither shares one with the caller's stream
        fb_create_streams(c);
        hog_create_lanes(c);
    }
    *out = c;
    return TBDK_OK;
}

int tbdk_ctx_destroy(tbdk_ctx* ctx)
{
    if (!ctx) return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    for (auto& r : ctx->recs) {
        (void)hipEventDestroy(r.begin);
        (void)hipEventDestroy(r.end);
    }
    for (auto e : ctx->free_events) (void)hipEventDestroy(e);
    gftt_scratch_free(ctx->gftt);
    fb_release(ctx);
    hog_release(ctx);
    if (ctx->dense_buf) (void)hipFree(ctx->dense_buf);
    if (ctx->dcase_buf) (void)hipFree(ctx->dcase_buf);
    for (hipStream_t st : {ctx->tbd_side, ctx->tbd_la, ctx->tbd_early})
        if (st) (void)hipStreamDestroy(st);
    delete ctx;
    return TBDK_OK;
}

int tbdk_ctx_device(const tbdk_ctx* ctx) { return ctx ? ctx->device : TBDK_EINVAL; }

int tbdk_timing_enable(tbdk_ctx* ctx, int enable)
{
    if (!ctx) return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    std::lock_guard<std::mutex> lk(ctx->timing_mu);
    for (auto& r : ctx->recs) {
        ctx->free_events.push_back(r.begin);
        ctx->free_events.push_back(r.end);
    }
    ctx->recs.clear();
    ctx->timing_calls.clear();
    ctx->timing = enable != 0;
    return TBDK_OK;
}

int tbdk_ctx_set_option(tbdk_ctx* ctx, const char* name, int64_t value)
{
    if (!ctx || !name) return TBDK_EINVAL;
    if (std::strcmp(name, "gftt_eig_redo") == 0) {
        ctx->opt_gftt_eig_redo = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "timing_every") == 0) {
        if (value < 1 || value > (1 << 20)) return TBDK_EINVAL;
        ctx->timing_every = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_early_gftt") == 0) {
        if (value < 0 || value > 2) return TBDK_EINVAL;
        ctx->opt_tbd_early_gftt = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_spec_lookahead") == 0) {
        ctx->opt_tbd_spec_la = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_zero_copy") == 0) {
        ctx->opt_tbd_zero_copy = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_fit_flag") == 0) {
        ctx->opt_tbd_fit_flag = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_early_la") == 0) {
        if (value < 0 || value > 2) return TBDK_EINVAL;
        ctx->opt_tbd_early_la = value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_early_prio") == 0) {
        ctx->opt_tbd_early_prio = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_early_order") == 0) {
        if (value < 0 || value > 2) return TBDK_EINVAL;
        ctx->opt_tbd_early_order = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "fb_prep_ahead") == 0) {
        ctx->opt_fb_prep_ahead = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "hog_level_streams") == 0) {
        if (value < 1 || value > 4) return TBDK_EINVAL;
        ctx->opt_hog_level_streams = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "hog_window_tiled") == 0) {
        ctx->opt_hog_window_tiled = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "hog_block_tiled") == 0) {
        if (value < 0 || value > 2) return TBDK_EINVAL;
        ctx->opt_hog_block_tiled = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_pyr_derivs") == 0) {
        ctx->opt_tbd_pyr_derivs = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_fit_wgpub") == 0) {
        ctx->opt_tbd_fit_wgpub = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_la_pyr_side") == 0) {
        if (value < 0 || value > 2) return TBDK_EINVAL;
        ctx->opt_tbd_la_pyr_side = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_post_direct") == 0) {
        ctx->opt_tbd_post_direct = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_fit_gate") == 0) {
        ctx->opt_tbd_fit_gate = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_la_defer") == 0) {
        ctx->opt_tbd_la_defer = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "gftt_compact") == 0) {
        ctx->opt_gftt_compact = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_borrow_l0") == 0) {
        ctx->opt_tbd_borrow_l0 = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_async_la") == 0) {
        ctx->opt_tbd_async_la = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "gftt_inline") == 0) {
        ctx->opt_gftt_inline = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_fit_inline") == 0) {
        ctx->opt_tbd_fit_inline = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "pyr_fuse") == 0) {
        if (value < 0 || value > 2) return TBDK_EINVAL;
        ctx->opt_pyr_fuse = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "pyr_xcd") == 0) {
        ctx->opt_pyr_xcd = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "pyr_rows") == 0) {
        if (value != 1 && value != 2 && value != 4) return TBDK_EINVAL;
        ctx->opt_pyr_rows = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "lk_dense_case") == 0) {
        ctx->opt_lk_dense_case = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "lk_scharr_fly") == 0) {
        ctx->opt_lk_scharr_fly = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "lk_seg_inline") == 0) {
        ctx->opt_lk_seg_inline = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_ahead_at") == 0) {
        if (value < 0 || value > 2) return TBDK_EINVAL;
        ctx->opt_tbd_ahead_at = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "tbd_gftt_ahead") == 0) {
        ctx->opt_tbd_gftt_ahead = value != 0;
        return TBDK_OK;
    }
    if (std::strcmp(name, "lk_solo") == 0) {
        if (value < 0 || value > 100) return TBDK_EINVAL;
        ctx->opt_lk_solo = (int)value;
        return TBDK_OK;
    }
    if (std::strcmp(name, "lk_impl") == 0) {  // kernel used when tbdk_lk_params.impl is 0 (auto)
        if (value < 0 || value > 3) return TBDK_EINVAL;
        ctx->opt_lk_impl = (int)value;
        return TBDK_OK;
    }
    return TBDK_EINVAL;
}

int tbdk_timing_select(tbdk_ctx* ctx, const char* names)
{
    if (!ctx) return TBDK_EINVAL;
    std::lock_guard<std::mutex> lk(ctx->timing_mu);
    ctx->timing_only.clear();
    if (names && *names) {
        ctx->timing_only = ",";
        for (const char* c = names; *c; ++c)
            if (*c != ' ') ctx->timing_only += *c;
        ctx->timing_only += ",";
    }
    return TBDK_OK;
}

int tbdk_timing_query(tbdk_ctx* ctx, const char* name, int64_t* launches, double* total_ms)
{
    if (!ctx || !name) return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    std::lock_guard<std::mutex> lk(ctx->timing_mu);
    int64_t cnt = 0;
    double tot = 0.0;
    for (auto& r : ctx->recs) {
        if (std::strcmp(r.name, name) != 0) continue;
        hipError_t e = hipEventSynchronize(r.end);
        if (e != hipSuccess) return map_err(e);
        float ms = 0.f;
        e = hipEventElapsedTime(&ms, r.begin, r.end);
        if (e != hipSuccess) return map_err(e);
        cnt++;
        tot += ms;
    }
    if (launches) *launches = cnt;
    if (total_ms) *total_ms = tot;
    return TBDK_OK;
}

int tbdk_timing_calls(tbdk_ctx* ctx, const char* name, int64_t* calls)
{
    if (!ctx || !name || !calls) return TBDK_EINVAL;
    *calls = 0;
    std::lock_guard<std::mutex> lk(ctx->timing_mu);
    for (auto& c : ctx->timing_calls)
        if (c.first == name) *calls = c.second;
    return TBDK_OK;
}

}  // extern "C"

// both depths: u8 (1 B/px) levels + int16x2 derivatives, or fp16 (2 B/px) + fp16x2
static int pyr_create(tbdk_ctx* ctx, int width, int height, int max_level, int win_w, int win_h, int depth,
                      int flags, tbdk_pyr* pyr, int cn = 1)
{
    if (!ctx || !pyr || width <= 0 || height <= 0 || max_level < 0 || win_w <= 2 || win_h <= 2 || win_w > 63 ||
        win_h > 63 || cn < 1 || cn > 4)
        return TBDK_EINVAL;
    const int bpp = (depth == TBDK_DEPTH_32F ? 4 : depth == TBDK_DEPTH_16F ? 2 : 1) * cn;
    const int dbpp = (depth == TBDK_DEPTH_32F ? 8 : 4) * cn;  // derivative pair bytes per pixel
    DeviceGuard g(ctx->device);
    std::memset(pyr, 0, sizeof(*pyr));
    if (max_level >= TBDK_MAX_LEVELS) max_level = TBDK_MAX_LEVELS - 1;
    const int pad = level_pad(win_w, win_h);
    // level sizes and the buildOpticalFlowPyramid stop rule (lkpyramid.cpp:782-787)
    int w = width, h = height, nlev = 0;
    size_t offs[TBDK_MAX_LEVELS], doffs[TBDK_MAX_LEVELS], total = 0;
    for (int level = 0; level <= max_level; ++level) {
        tbdk_level& L = pyr->lv[level];
        L.width = w;
        L.height = h;
        L.pad = pad;
        L.pitch = align_up((w + 2 * pad) * bpp, 256);
        offs[level] = total;
        total += (size_t)L.pitch * (h + 2 * pad) + 256;  // +256: aligned over-reads of the last row
        total = (total + 255) & ~(size_t)255;
        tbdk_level& D = pyr->dv[level];
        D.width = w;
        D.height = h;
        D.pad = pad;
        D.pitch = align_up((w + 2 * pad) * dbpp, 256);
        doffs[level] = total;
        if (!(flags & TBDK_PYR_NO_DERIVS)) {
            total += (size_t)D.pitch * (h + 2 * pad) + 256;
            total = (total + 255) & ~(size_t)255;
        }
        nlev = level + 1;
        w = (w + 1) / 2;
        h = (h + 1) / 2;
        if (w <= win_w || h <= win_h) break;
    }
    void* mem = nullptr;
    hipError_t e = hipMalloc(&mem, total);
    if (e != hipSuccess) return map_err(e);
    // the derivative planes' BORDER_CONSTANT frame is zero once and never rewritten
    // (levels only: every byte a reader can reach is rewritten by each build)
    e = hipMemset(mem, 0, total);
    if (e != hipSuccess) {
        (void)hipFree(mem);
        return map_err(e);
    }
    pyr->storage = mem;
    pyr->nlevels = nlev;
    pyr->win_w = win_w;
    pyr->win_h = win_h;
    pyr->depth = depth;
    pyr->flags = flags;
    pyr->cn = cn;
    for (int level = 0; level < nlev; ++level) {
        pyr->lv[level].data = static_cast<uint8_t*>(mem) + offs[level];
        pyr->dv[level].data = (flags & TBDK_PYR_NO_DERIVS) ? nullptr : static_cast<uint8_t*>(mem) + doffs[level];
    }
    return TBDK_OK;
}

extern "C" {

int tbdk_pyr_create(tbdk_ctx* ctx, int width, int height, int max_level, int win_w, int win_h, tbdk_pyr* pyr)
{
    return pyr_create(ctx, width, height, max_level, win_w, win_h, TBDK_DEPTH_8U, 0, pyr);
}

int tbdk_pyr_create_levels(tbdk_ctx* ctx, int width, int height, int max_level, int win_w, int win_h, tbdk_pyr* pyr)
{
    return pyr_create(ctx, width, height, max_level, win_w, win_h, TBDK_DEPTH_8U, TBDK_PYR_NO_DERIVS, pyr);
}

int tbdk_pyr_create_cn(tbdk_ctx* ctx, int width, int height, int cn, int max_level, int win_w, int win_h,
                       tbdk_pyr* pyr)
{
    return pyr_create(ctx, width, height, max_level, win_w, win_h, TBDK_DEPTH_8U, 0, pyr, cn);
}

int tbdk_pyr_create_f32(tbdk_ctx* ctx, int width, int height, int max_level, int win_w, int win_h, tbdk_pyr* pyr)
{
    return pyr_create(ctx, width, height, max_level, win_w, win_h, TBDK_DEPTH_32F, 0, pyr);
}

int tbdk_pyr_create_f32_cn(tbdk_ctx* ctx, int width, int height, int cn, int max_level, int win_w, int win_h,
                           tbdk_pyr* pyr)
{
    if (cn < 1 || cn > 4) return TBDK_EINVAL;
    return pyr_create(ctx, width, height, max_level, win_w, win_h, TBDK_DEPTH_32F, 0, pyr, cn);
}

int tbdk_pyr_create_f16(tbdk_ctx* ctx, int width, int height, int max_level, int win_w, int win_h, tbdk_pyr* pyr)
{
    return pyr_create(ctx, width, height, max_level, win_w, win_h, TBDK_DEPTH_16F, 0, pyr);
}

int tbdk_pyr_destroy(tbdk_ctx* ctx, tbdk_pyr* pyr)
{
    if (!ctx || !pyr) return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    if (pyr->storage) (void)hipFree(pyr->storage);
    std::memset(pyr, 0, sizeof(*pyr));
    return TBDK_OK;
}

int tbdk_pyr_build(tbdk_ctx* ctx, const uint8_t* img, int pitch, tbdk_pyr* pyr, void* stream)
{
    const int cn = pyr && pyr->cn > 1 ? pyr->cn : 1;
    if (!ctx || !img || !pyr || pyr->nlevels <= 0 || pitch < pyr->lv[0].width * cn) return TBDK_EINVAL;
    if (cn > 1 && pyr->depth == TBDK_DEPTH_16F) return TBDK_EINVAL;
    if (pyr->flags & kPyrL0Borrowed) {  // a borrowed level 0 (tbdk_pyr_build_borrowed): the own buffer again
        tbdk_level& L = pyr->lv[0];
        L.pad = level_pad(pyr->win_w, pyr->win_h);
        L.pitch = align_up(L.width + 2 * L.pad, 256);  // u8 levels only (pyr_create's layout)
        L.data = static_cast<uint8_t*>(pyr->storage);
        pyr->flags &= ~kPyrL0Borrowed;
    }
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rec = timing_begin(ctx, "pyr_build", s);
    hipError_t e;
    if (cn > 1 && pyr->depth == TBDK_DEPTH_32F) {
        e = launch_pyr_build_f32_cn(img, pitch, 0, *pyr, s);
    } else if (cn > 1) {
        e = launch_pyr_cn(img, pitch, *pyr, s);
    } else if (pyr->depth == TBDK_DEPTH_16F) {
        e = ctx->opt_pyr_fuse ? launch_pyr_build_fp(img, pitch, 0, false, *pyr, ctx->opt_pyr_rows, ctx->opt_pyr_xcd, s)
                              : launch_pyr_build_f16(img, pitch, 0, *pyr, s);
    } else if (pyr->depth == TBDK_DEPTH_32F) {
        e = ctx->opt_pyr_fuse ? launch_pyr_build_fp(img, pitch, 0, true, *pyr, ctx->opt_pyr_rows, ctx->opt_pyr_xcd, s)
                              : launch_pyr_build_f32(img, pitch, 0, *pyr, s);
    } else {
        e = launch_pyr_levels(img, pitch, *pyr, ctx->opt_pyr_fuse, ctx->opt_pyr_rows, ctx->opt_pyr_xcd, s);
        if (e == hipSuccess && !(pyr->flags & TBDK_PYR_NO_DERIVS)) e = launch_scharr_levels(*pyr, s);
    }
    timing_end(ctx, rec, s);
    return map_err(e);
}

int tbdk_pyr_build_borrowed(tbdk_ctx* ctx, const uint8_t* img, int pitch, tbdk_pyr* pyr, void* stream)
{
    if (!ctx || !img || !pyr || pyr->nlevels <= 0 || !pyr->storage) return TBDK_EINVAL;
    if (pyr->flags & kPyrL0Borrowed) {  // borrowing already: its own level 0 descriptor first
        tbdk_level& L = pyr->lv[0];
        L.pad = level_pad(pyr->win_w, pyr->win_h);
        L.pitch = align_up(L.width + 2 * L.pad, 256);
        L.data = static_cast<uint8_t*>(pyr->storage);
        pyr->flags &= ~kPyrL0Borrowed;
    }
    return tbdk::pyr_build_borrowed(ctx, img, pitch, pyr, static_cast<hipStream_t>(stream));
}

}  // extern "C"

int tbdk::pyr_build_borrowed(tbdk_ctx* ctx, const uint8_t* img, int pitch, tbdk_pyr* pyr, hipStream_t s)
{
    if (!ctx || !img || !pyr || pyr->nlevels <= 0 || pyr->cn > 1 || pyr->depth != TBDK_DEPTH_8U ||
        !(pyr->flags & TBDK_PYR_NO_DERIVS) || pitch < pyr->lv[0].width || !ctx->opt_pyr_fuse)
        return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    pyr->lv[0].data = const_cast<uint8_t*>(img);
    pyr->lv[0].pitch = pitch;
    pyr->lv[0].pad = 0;
    pyr->flags |= kPyrL0Borrowed;
    int rec = timing_begin(ctx, "pyr_build", s);
    const hipError_t e = launch_pyr_levels(img, pitch, *pyr, ctx->opt_pyr_fuse, ctx->opt_pyr_rows, ctx->opt_pyr_xcd, s,
                                           true);
    timing_end(ctx, rec, s);
    return map_err(e);
}

int tbdk::pyr_restore_l0(tbdk_ctx* ctx, tbdk_pyr* pyr, const tbdk_level& own_l0, hipStream_t s)
{
    if (!ctx || !pyr) return TBDK_EINVAL;
    if (!(pyr->flags & kPyrL0Borrowed)) return TBDK_OK;
    DeviceGuard g(ctx->device);
    const hipError_t e = launch_pad_copy(pyr->lv[0].data, pyr->lv[0].pitch, own_l0, s);
    pyr->lv[0] = own_l0;
    pyr->flags &= ~kPyrL0Borrowed;
    return map_err(e);
}

extern "C" {

int tbdk_pyr_build_f16(tbdk_ctx* ctx, const uint16_t* img, int pitch, tbdk_pyr* pyr, void* stream)
{
    if (!ctx || !img || !pyr || pyr->nlevels <= 0 || pyr->depth != TBDK_DEPTH_16F || pitch < 2 * pyr->lv[0].width ||
        pitch % 2 != 0)
        return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rec = timing_begin(ctx, "pyr_build", s);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(img);
    hipError_t e = ctx->opt_pyr_fuse ? launch_pyr_build_fp(p, pitch, 3, false, *pyr, ctx->opt_pyr_rows, ctx->opt_pyr_xcd, s)
                                     : launch_pyr_build_f16(p, pitch, 1, *pyr, s);
    timing_end(ctx, rec, s);
    return map_err(e);
}

static int pyr_build_f32_from(tbdk_ctx* ctx, const void* img, int pitch, int bytes_per_px, int kind, tbdk_pyr* pyr,
                              void* stream)
{
    const int cn = pyr && pyr->cn > 1 ? pyr->cn : 1;
    if (!ctx || !img || !pyr || pyr->nlevels <= 0 || pyr->depth != TBDK_DEPTH_32F ||
        pitch < bytes_per_px * cn * pyr->lv[0].width || pitch % bytes_per_px != 0)
        return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rec = timing_begin(ctx, "pyr_build", s);
    hipError_t e = cn > 1 ? launch_pyr_build_f32_cn(static_cast<const uint8_t*>(img), pitch, kind, *pyr, s)
               : ctx->opt_pyr_fuse ? launch_pyr_build_fp(static_cast<const uint8_t*>(img), pitch, kind, true, *pyr, ctx->opt_pyr_rows, ctx->opt_pyr_xcd, s)
                                   : launch_pyr_build_f32(static_cast<const uint8_t*>(img), pitch, kind, *pyr, s);
    timing_end(ctx, rec, s);
    return map_err(e);
}

int tbdk_pyr_build_u16(tbdk_ctx* ctx, const uint16_t* img, int pitch, tbdk_pyr* pyr, void* stream)
{
    return pyr_build_f32_from(ctx, img, pitch, 2, 1, pyr, stream);
}

int tbdk_pyr_build_f32(tbdk_ctx* ctx, const float* img, int pitch, tbdk_pyr* pyr, void* stream)
{
    return pyr_build_f32_from(ctx, img, pitch, 4, 2, pyr, stream);
}

int tbdk_pyr_download(tbdk_ctx* ctx, const tbdk_pyr* pyr, int level, uint8_t* host, int host_pitch,
                      int with_border)
{
    if (!ctx || !pyr || !host || level < 0 || level >= pyr->nlevels) return TBDK_EINVAL;
    const tbdk_level& L = pyr->lv[level];
    const int bpp = (pyr->depth == TBDK_DEPTH_32F ? 4 : pyr->depth == TBDK_DEPTH_16F ? 2 : 1) * (pyr->cn > 1 ? pyr->cn : 1);
    const int w = with_border ? L.width + 2 * L.pad : L.width;
    const int h = with_border ? L.height + 2 * L.pad : L.height;
    if (host_pitch < w * bpp) return TBDK_EINVAL;
    const uint8_t* src = with_border ? L.data : L.data + (size_t)L.pad * L.pitch + (size_t)L.pad * bpp;
    DeviceGuard g(ctx->device);
    hipError_t e = hipMemcpy2D(host, host_pitch, src, L.pitch, (size_t)w * bpp, h, hipMemcpyDeviceToHost);
    return map_err(e);
}

int tbdk_pyr_download_deriv(tbdk_ctx* ctx, const tbdk_pyr* pyr, int level, int16_t* host, int host_pitch)
{
    if (!ctx || !pyr || !host || level < 0 || level >= pyr->nlevels || !pyr->dv[level].data) return TBDK_EINVAL;
    const tbdk_level& D = pyr->dv[level];
    const int bpp = (pyr->depth == TBDK_DEPTH_32F ? 8 : 4) * (pyr->cn > 1 ? pyr->cn : 1);
    if (host_pitch < D.width * bpp) return TBDK_EINVAL;
    const uint8_t* src = D.data + (size_t)D.pad * D.pitch + (size_t)D.pad * bpp;
    DeviceGuard g(ctx->device);
    hipError_t e = hipMemcpy2D(host, host_pitch, src, D.pitch, (size_t)D.width * bpp, D.height, hipMemcpyDeviceToHost);
    return map_err(e);
}

int tbdk_pyr_down_u8(tbdk_ctx* ctx, const uint8_t* src, int width, int height, int src_pitch, uint8_t* dst,
                     int dst_pitch, void* stream)
{
    if (!ctx || !src || !dst || width <= 0 || height <= 0 || src_pitch < width || dst_pitch < (width + 1) / 2)
        return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rec = timing_begin(ctx, "pyr_down", s);
    hipError_t e = launch_pyr_down_plain(src, width, height, src_pitch, dst, dst_pitch, s);
    timing_end(ctx, rec, s);
    return map_err(e);
}

int tbdk_lk_sparse(tbdk_ctx* ctx, const tbdk_pyr* prev, const tbdk_pyr* next, const float* prev_pts,
                   float* next_pts, uint8_t* status, float* err, int32_t* iters, int n, const tbdk_lk_params* p,
                   void* stream)
{
    return tbdk::lk_internal(ctx, prev, next, prev_pts, next_pts, status, err, iters, n, p, nullptr, 0, stream);
}

}  // extern "C"

int tbdk::lk_internal(tbdk_ctx* ctx, const tbdk_pyr* prev, const tbdk_pyr* next, const float* prev_pts,
                      float* next_pts, uint8_t* status, float* err, int32_t* iters, int n, const tbdk_lk_params* p,
                      const int32_t* seg_counts, int seg_stride, void* stream, const int32_t* seg_list,
                      const LkDense* dense, const int32_t* seg_list_host)
{
    if (!ctx || !prev || !next || !p || n < 0) return TBDK_EINVAL;
    if (n == 0) return TBDK_OK;
    if (dense ? !dense->flow : (!prev_pts || !next_pts || !status)) return TBDK_EINVAL;
    if (p->win_w <= 2 || p->win_h <= 2 || p->win_w > 63 || p->win_h > 63 || p->max_level < 0) return TBDK_EINVAL;
    if (prev->nlevels <= 0 || next->nlevels <= 0) return TBDK_EINVAL;
    if (prev->depth != next->depth ||
        (prev->depth != TBDK_DEPTH_8U && prev->depth != TBDK_DEPTH_16F && prev->depth != TBDK_DEPTH_32F))
        return TBDK_EINVAL;
    const bool f32 = prev->depth == TBDK_DEPTH_32F;
    const bool f16 = prev->depth == TBDK_DEPTH_16F || f32;  // the float pixel paths
    const int cn = prev->cn > 1 ? prev->cn : 1;
    if (cn != (next->cn > 1 ? next->cn : 1) || (cn > 1 && f16 && !f32)) return TBDK_EINVAL;
    const int pad_needed = p->win_w > p->win_h ? p->win_w + 2 : p->win_h + 2;
    int max_level = p->max_level;
    if (prev->nlevels - 1 < max_level) max_level = prev->nlevels - 1;
    if (next->nlevels - 1 < max_level) max_level = next->nlevels - 1;
    LkArgs a;
    std::memset(&a, 0, sizeof(a));
    for (int l = 0; l <= max_level; ++l) {
        const tbdk_level& I = prev->lv[l];
        const tbdk_level& J = next->lv[l];
        if (I.width != J.width || I.height != J.height) return TBDK_EINVAL;
        // a borrowed level 0 (the TBD loop's; pad 0) is read with reflect-101
        // coordinates at its edges by the several-points-per-wave kernel only
        const bool bI = l == 0 && (prev->flags & kPyrL0Borrowed) && I.pad == 0;
        const bool bJ = l == 0 && (next->flags & kPyrL0Borrowed) && J.pad == 0;
        if ((I.pad < pad_needed && !bI) || (J.pad < pad_needed && !bJ)) return TBDK_EINVAL;
        const tbdk_level& D = prev->dv[l];
        const int impl_eff = p->impl ? p->impl : ctx->opt_lk_impl;
        if ((bI || bJ) && (dense || cn > 1 || f16 || D.data || !lk_multi_supported(p->win_w, p->win_h) ||
                           (impl_eff != 0 && impl_eff != 3)))
            return TBDK_EINVAL;
        a.lv[l] = LkLevel{I.data, J.data, D.data, I.width, I.height, I.pitch, J.pitch, I.pad, J.pad, D.pitch, D.pad};
    }
    a.max_level = max_level;
    a.win_w = p->win_w;
    a.win_h = p->win_h;
    a.max_count = p->max_count < 0 ? 0 : (p->max_count > 100 ? 100 : p->max_count);
    double eps = p->epsilon < 0. ? 0. : (p->epsilon > 10. ? 10. : p->epsilon);
    a.eps2 = eps * eps;
    a.flags = p->flags;
    a.min_eig = p->min_eig_threshold;
    a.prev_pts = prev_pts;
    a.next_pts = next_pts;
    a.status = status;
    a.err = err;
    a.iters = iters;
    a.n = n;
    a.seg_counts = seg_counts;
    a.seg_list = seg_list;
    a.seg_stride = seg_stride > 0 ? seg_stride : 1;
    if ((seg_counts && seg_stride <= 0) || (seg_list && !seg_counts)) return TBDK_EINVAL;
    if (seg_list && seg_list_host && ctx->opt_lk_seg_inline) {  // the list into the kernel arguments
        const int nseg = (int)(((int64_t)n + a.seg_stride - 1) / a.seg_stride);
        bool fits = nseg <= kSegInline;
        for (int k = 0; fits && k < nseg; ++k) fits = (uint32_t)seg_list_host[k] <= 0xFFFFu;
        if (fits) {
            for (int k = 0; k < nseg; ++k) a.seg_inl[k] = (uint16_t)seg_list_host[k];
            a.seg_ninl = nseg;
            a.seg_list = nullptr;
        }
    }
    a.solo_min = ctx->opt_lk_solo;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    bool have_d = true;
    for (int l = 0; l <= max_level; ++l)
        if (!a.lv[l].D || a.lv[l].dpad < pad_needed) have_d = false;
    if (dense) {  // dense mode (klt_dense.hip): the planes instance of the several-points-per-wave kernel
        if (cn > 1 || f16 || p->impl != 0 || !have_d || !lk_multi_supported(p->win_w, p->win_h) || seg_counts)
            return TBDK_EINVAL;
        for (int l = 0; l <= max_level; ++l) {
            a.lv[l].C = dense->C[l];
            a.lv[l].cstride = dense->cstride[l];
            a.lv[l].cpitch = dense->cpitch[l];
        }
        a.dense_w = dense->w;
        a.flow = dense->flow;
        a.flow_pitch = dense->flow_pitch;
        a.dstatus = dense->status;
        a.dstatus_pitch = dense->status_pitch;
        int rec = timing_begin(ctx, "lk_dense", s);
        hipError_t e = launch_lk_multi_dense(a, s);
        timing_end(ctx, rec, s);
        return map_err(e);
    }
    // auto: several points per wave when the window has an instantiation, else the
    // one-point-per-wave strip kernel, else the generic LDS kernel (no derivative planes)
    if (p->impl < 0 || p->impl > 3) return TBDK_EINVAL;
    if (cn > 1 && f32) {  // multi-channel 16U / 32F frames: the fp32 cn kernel (klt_cn_f32.hip)
        if (p->impl != 0 || !have_d || lk_cn_f32_smem_bytes(p->win_w, p->win_h, cn) > 160 * 1024) return TBDK_EINVAL;
        a.cn = cn;
        int rec = timing_begin(ctx, "lk_sparse", s);
        hipError_t e = launch_lk_cn_f32(a, s);
        timing_end(ctx, rec, s);
        return map_err(e);
    }
    if (cn > 1) {  // multi-channel frames: one kernel (klt_cn.hip), on the derivative planes
        if (p->impl != 0 || !have_d || lk_cn_smem_bytes(p->win_w, p->win_h, cn) > 160 * 1024) return TBDK_EINVAL;
        a.cn = cn;
        int rec = timing_begin(ctx, "lk_sparse", s);
        hipError_t e = launch_lk_cn(a, s);
        timing_end(ctx, rec, s);
        return map_err(e);
    }
    if (f16) {  // the fp16 pixel path has one kernel (klt_f16.hip)
        if (p->impl != 0 || !have_d || !lk_f16_supported(p->win_w, p->win_h)) return TBDK_EINVAL;
        int rec = timing_begin(ctx, "lk_sparse", s);
        hipError_t e = launch_lk_f16(a, f32, s);
        timing_end(ctx, rec, s);
        return map_err(e);
    }
    const int impl = p->impl ? p->impl : ctx->opt_lk_impl;
    // the multi kernel derives the window's Scharr values itself when the
    // pyramid has no derivative planes, or when asked to (ctx option lk_scharr_fly)
    const bool fly = !have_d || ctx->opt_lk_scharr_fly;
    const bool multi = (impl == 0 || impl == 3) && lk_multi_supported(p->win_w, p->win_h);
    const bool strip = !multi && (impl == 0 || impl == 1) && have_d && lk_strip_supported(p->win_w, p->win_h);
    if ((p->impl == 1 && !strip) || (p->impl == 3 && !multi)) return TBDK_EINVAL;
    int rec = timing_begin(ctx, "lk_sparse", s);
    hipError_t e = multi ? launch_lk_multi(a, fly, s) : strip ? launch_lk_strip(a, s) : launch_lk_sparse(a, s);
    timing_end(ctx, rec, s);
    return map_err(e);
}

namespace tbdk {

int gftt_prepare(const tbdk_roi* rois, int nroi, int width, int height, const tbdk_gftt_params* p, GfttRoi* tab,
                 GfttPlan* plan)
{
    if (p->max_corners <= 0 || !(p->quality_level > 0) || p->min_distance < 0 || p->block_size < 1 ||
        p->block_size > 63 || (p->use_harris != 0 && p->use_harris != 1) || !std::isfinite(p->harris_k))
        return TBDK_EINVAL;
    if (gftt_generic(p) && nroi > 65535) return TBDK_EINVAL;  // the response launches' grid rows
    int64_t total = 0, ncblk = 0, words = 0;
    int max_area = 0;
    for (int i = 0; i < nroi; ++i) {
        const tbdk_roi& r = rois[i];
        if (r.x < 0 || r.y < 0 || r.width <= 0 || r.height <= 0 || r.x + r.width > width || r.y + r.height > height ||
            r.width > 65535 || r.height > 65535)
            return TBDK_EINVAL;
        tab[i] = GfttRoi{r.x, r.y, r.width, r.height, (int)total, (int)words, (int)ncblk};
        const int64_t strips = (r.width + kGfttStrip - 1) / kGfttStrip;
        total += (int64_t)gftt_epitch(r.width) * r.height;
        ncblk += strips;
        if (r.width >= 3 && r.height >= 3) words += strips * r.height;  // smaller ROIs have no interior
        max_area = std::max(max_area, r.width * r.height);
        plan->max_w = std::max(plan->max_w, r.width);
        plan->max_h = std::max(plan->max_h, r.height);
    }
    if (total > INT32_MAX || words > INT32_MAX) return TBDK_EINVAL;
    if (gftt_generic(p) && total > INT32_MAX / 3) return TBDK_EINVAL;
    plan->nroi = nroi;
    plan->total = total;
    plan->ncblk = (int)ncblk;
    plan->words = words;
    plan->max_area = max_area;
    return TBDK_OK;
}

static void gftt_resp_args(GfttRespArgs& ra, const GfttScratch& sc, const uint8_t* img, int pitch,
                           const GfttRoi* d_rois, int nroi, int block, int harris, double hk)
{
    ra.img = img;
    ra.pitch = pitch;
    ra.rois = d_rois;
    ra.nroi = nroi;
    ra.cov = static_cast<float*>(sc.resp);
    ra.rs = reinterpret_cast<double*>(static_cast<float*>(sc.resp) + 3 * (size_t)sc.cap_resp_px);
    ra.eig = static_cast<float*>(sc.planes);
    ra.blk_max = sc.blk;
    ra.lmax = static_cast<uint64_t*>(sc.cand);
    ra.block = block;
    ra.harris = harris;
    // cornerEigenValsVecs' scale for ksize 3 on 8-bit input (corner.cpp:248-255)
    const double scale = 1.0 / ((double)(1 << 2) * block * 255.0);
    ra.k = (float)(1.0 * scale);
    ra.k2 = (float)(2.0 * scale);
    ra.kf = (float)hk;
    ra.hk = hk;
}

void gftt_scratch_free(GfttScratch& sc)
{
    for (void** p : {&sc.rois, reinterpret_cast<void**>(&sc.blk), &sc.planes, &sc.cand, &sc.resp}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    sc.cap_rois = 0;
    sc.cap_px = 0;
    sc.cap_resp_px = 0;
}

int gftt_reserve_resp(GfttScratch& sc, int device, int64_t max_px)
{
    if (max_px <= sc.cap_resp_px) return TBDK_OK;
    DeviceGuard g(device);
    if (sc.resp) (void)hipFree(sc.resp);  // waits for the device: no launch still reads it
    sc.resp = nullptr;
    sc.cap_resp_px = 0;
    const hipError_t e = hipMalloc(&sc.resp, (sizeof(float) * 3 + sizeof(double) * 3) * (size_t)std::max<int64_t>(max_px, 1));
    if (e != hipSuccess) return map_err(e);
    sc.cap_resp_px = max_px;
    return TBDK_OK;
}

int gftt_reserve(GfttScratch& sc, int device, int max_rois, int64_t max_px)
{
    if (max_rois < 0 || max_px < 0) return TBDK_EINVAL;
    if (max_rois <= sc.cap_rois && max_px <= sc.cap_px) return TBDK_OK;
    DeviceGuard g(device);
    const int rois = std::max(max_rois, sc.cap_rois);
    const int64_t px = std::max(max_px, sc.cap_px);
    gftt_scratch_free(sc);  // hipFree waits for the device: no launch still reads it
    const int64_t ncb = gftt_max_cblocks(rois, px), nw = gftt_max_words(px);
    hipError_t e = hipMalloc(&sc.rois, sizeof(GfttRoi) * (size_t)std::max(rois, 1));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&sc.blk), sizeof(int) * (size_t)ncb);
    if (e == hipSuccess) e = hipMalloc(&sc.planes, sizeof(float) * (size_t)std::max<int64_t>(px, 1));
    if (e == hipSuccess) e = hipMalloc(&sc.cand, sizeof(uint64_t) * (size_t)nw);
    if (e != hipSuccess) {
        gftt_scratch_free(sc);
        return map_err(e);
    }
    sc.cap_rois = rois;
    sc.cap_px = px;
    return TBDK_OK;
}

int gftt_launch(tbdk_ctx* ctx, GfttScratch& sc, const uint8_t* img, int pitch, const GfttRoi* d_rois,
                const GfttPlan& plan, const tbdk_gftt_params* p, float* corners, int32_t* counts, hipStream_t s,
                hipEvent_t after_eig, int corner_stride, const GfttRoi* h_rois)
{
    if (corner_stride != 0 && corner_stride < p->max_corners) return TBDK_EINVAL;
    int rc = gftt_reserve(sc, ctx->device, plan.nroi, plan.total);
    if (rc != TBDK_OK) return rc;
    DeviceGuard g(ctx->device);
    int rec = timing_begin(ctx, "gftt", s);
    GfttArgs a;
    a.img = img;
    a.pitch = pitch;
    a.rois = d_rois;
    a.nroi = plan.nroi;
    a.ncblk = plan.ncblk;
    a.eig = static_cast<float*>(sc.planes);
    a.blk_max = sc.blk;
    a.lmax = static_cast<uint64_t*>(sc.cand);
    a.max_corners = p->max_corners;
    a.quality = p->quality_level;
    a.min_distance = p->min_distance;
    a.corners = reinterpret_cast<float2*>(corners);
    a.corner_stride = corner_stride ? corner_stride : p->max_corners;
    a.counts = counts;
    a.eig_redo = ctx->opt_gftt_eig_redo;
    a.compact = ctx->opt_gftt_compact && p->quality_level <= 1.0 && !gftt_generic(p) ? 1 : 0;
    a.ninl = 0;
    if (h_rois && ctx->opt_gftt_inline && plan.nroi <= kGfttInline) {  // the table into the kernel arguments
        bool fits = true;
        for (int r = 0; fits && r < plan.nroi; ++r) {
            const GfttRoi& R = h_rois[r];
            fits = R.x >= 0 && R.y >= 0 && R.w >= 0 && R.h >= 0 && R.x <= 0xFFFF && R.y <= 0xFFFF && R.w <= 0xFFFF &&
                   R.h <= 0xFFFF;
            if (fits)
                a.inl[r] = GfttRoiC{(uint16_t)R.x, (uint16_t)R.y, (uint16_t)R.w, (uint16_t)R.h, R.off, R.moff, R.cblk};
        }
        if (fits) a.ninl = plan.nroi;
    }
    gftt_plan(a, plan.max_area);
    hipError_t e;
    if (!gftt_generic(p)) {
        e = launch_gftt(a, s, after_eig);
    } else {
        rc = gftt_reserve_resp(sc, ctx->device, plan.total);
        if (rc != TBDK_OK) return rc;
        GfttRespArgs ra;
        gftt_resp_args(ra, sc, img, pitch, d_rois, plan.nroi, p->block_size, p->use_harris, p->harris_k);
        e = launch_gftt_resp(ra, plan.ncblk, plan.max_w, plan.max_h, plan.max_area, s);
        if (e == hipSuccess && after_eig) e = hipEventRecord(after_eig, s);
        if (e == hipSuccess) e = launch_gftt_select(a, s);
    }
    timing_end(ctx, rec, s);
    return map_err(e);
}

}  // namespace tbdk

extern "C" {

int tbdk_gftt_reserve(tbdk_ctx* ctx, int max_rois, int64_t max_total_pixels)
{
    if (!ctx || max_rois < 0 || max_total_pixels < 0) return TBDK_EINVAL;
    return gftt_reserve(ctx->gftt, ctx->device, max_rois, max_total_pixels);
}

int tbdk_gftt_rois(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, const tbdk_roi* rois,
                   int nroi, const tbdk_gftt_params* p, float* corners, int32_t* counts, void* stream)
{
    if (!ctx || !p || nroi < 0) return TBDK_EINVAL;
    if (nroi == 0) return TBDK_OK;
    if (!img || !rois || !corners || !counts || width <= 0 || height <= 0 || pitch < width) return TBDK_EINVAL;
    GfttPlan plan;
    std::vector<GfttRoi> tab((size_t)nroi);
    int rc = gftt_prepare(rois, nroi, width, height, p, tab.data(), &plan);
    if (rc != TBDK_OK) return rc;
    rc = tbdk_gftt_reserve(ctx, nroi, plan.total);
    if (rc != TBDK_OK) return rc;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // pageable source: the copy is staged and complete when the call returns
    hipError_t e = hipMemcpyAsync(ctx->gftt.rois, tab.data(), sizeof(GfttRoi) * (size_t)nroi, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return map_err(e);
    return gftt_launch(ctx, ctx->gftt, img, pitch, static_cast<const GfttRoi*>(ctx->gftt.rois), plan, p, corners,
                       counts, s, nullptr, 0, tab.data());
}

int tbdk_corner_min_eig_val(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, float* dst,
                            int dst_pitch, void* stream)
{
    if (!ctx || !img || !dst || width <= 0 || height <= 0 || pitch < width || dst_pitch < width * 4 ||
        dst_pitch % 4 != 0)
        return TBDK_EINVAL;
    tbdk_roi roi{0, 0, width, height};
    tbdk_gftt_params p{1, 0.01, 0.0, 3};
    GfttPlan plan;
    GfttRoi tab;
    int rc = gftt_prepare(&roi, 1, width, height, &p, &tab, &plan);
    if (rc != TBDK_OK) return rc;
    rc = tbdk_gftt_reserve(ctx, 1, plan.total);
    if (rc != TBDK_OK) return rc;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipMemcpyAsync(ctx->gftt.rois, &tab, sizeof(GfttRoi), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return map_err(e);
    int rec = timing_begin(ctx, "corner_min_eig", s);
    GfttArgs a{};
    a.img = img;
    a.pitch = pitch;
    a.rois = static_cast<const GfttRoi*>(ctx->gftt.rois);
    a.nroi = 1;
    a.ncblk = plan.ncblk;
    a.eig = static_cast<float*>(ctx->gftt.planes);
    a.blk_max = ctx->gftt.blk;
    a.lmax = static_cast<uint64_t*>(ctx->gftt.cand);
    a.eig_redo = ctx->opt_gftt_eig_redo;
    e = launch_gftt_eig(a, s);
    timing_end(ctx, rec, s);
    if (e == hipSuccess)
        e = hipMemcpy2DAsync(dst, (size_t)dst_pitch, ctx->gftt.planes, (size_t)gftt_epitch(width) * 4, (size_t)width * 4, height,
                             hipMemcpyDeviceToDevice, s);
    return map_err(e);
}

int tbdk_corner_response(tbdk_ctx* ctx, const uint8_t* img, int width, int height, int pitch, float* dst,
                         int dst_pitch, int block_size, int harris, double harris_k, void* stream)
{
    if (!ctx || !img || !dst || width <= 0 || height <= 0 || pitch < width || dst_pitch < width * 4 ||
        dst_pitch % 4 != 0 || block_size < 1 || block_size > 63 || !std::isfinite(harris_k))
        return TBDK_EINVAL;
    if (block_size == 3 && !harris)
        return tbdk_corner_min_eig_val(ctx, img, width, height, pitch, dst, dst_pitch, stream);
    tbdk_roi roi{0, 0, width, height};
    tbdk_gftt_params p{1, 0.01, 0.0, block_size, harris ? 1 : 0, harris_k};
    GfttPlan plan;
    GfttRoi tab;
    int rc = gftt_prepare(&roi, 1, width, height, &p, &tab, &plan);
    if (rc != TBDK_OK) return rc;
    rc = tbdk_gftt_reserve(ctx, 1, plan.total);
    if (rc == TBDK_OK) rc = gftt_reserve_resp(ctx->gftt, ctx->device, plan.total);
    if (rc != TBDK_OK) return rc;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipMemcpyAsync(ctx->gftt.rois, &tab, sizeof(GfttRoi), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return map_err(e);
    int rec = timing_begin(ctx, "corner_response", s);
    GfttRespArgs ra;
    gftt_resp_args(ra, ctx->gftt, img, pitch, static_cast<const GfttRoi*>(ctx->gftt.rois), 1, block_size,
                   harris ? 1 : 0, harris_k);
    e = launch_gftt_resp(ra, plan.ncblk, plan.max_w, plan.max_h, plan.max_area, s);
    timing_end(ctx, rec, s);
    if (e == hipSuccess)
        e = hipMemcpy2DAsync(dst, (size_t)dst_pitch, ctx->gftt.planes, (size_t)gftt_epitch(width) * 4, (size_t)width * 4, height,
                             hipMemcpyDeviceToDevice, s);
    return map_err(e);
}

int tbdk_box_propagate(tbdk_ctx* ctx, const float* prev_pts, const float* next_pts, const uint8_t* status,
                       const int32_t* offsets, const tbdk_roi* boxes, int nboxes, int min_points,
                       tbdk_box_fit* out, void* stream)
{
    if (!ctx || nboxes < 0) return TBDK_EINVAL;
    if (nboxes == 0) return TBDK_OK;
    if (!prev_pts || !next_pts || !offsets || !boxes || !out || min_points < 0) return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rec = timing_begin(ctx, "box_propagate", s);
    hipError_t e = launch_box_propagate(prev_pts, next_pts, status, offsets, boxes, nboxes, min_points, out, s);
    timing_end(ctx, rec, s);
    return map_err(e);
}

int tbdk_warp_affine_u8(tbdk_ctx* ctx, const uint8_t* src, int src_width, int src_height, int src_pitch,
                        uint8_t* dst, int dst_width, int dst_height, int dst_pitch, const double* M,
                        int flags, int border, int border_value, void* stream)
{
    if (!ctx || !src || !dst || !M) return TBDK_EINVAL;
    if (src_width <= 0 || src_height <= 0 || dst_width <= 0 || dst_height <= 0 || src_pitch < src_width ||
        dst_pitch < dst_width || src_width > 32767 || src_height > 32767)  // reference: SHRT_MAX maps
        return TBDK_EINVAL;
    int inter = flags & 7;
    if (inter == TBDK_INTER_AREA) inter = TBDK_INTER_LINEAR;
    if ((inter != TBDK_INTER_NEAREST && inter != TBDK_INTER_LINEAR && inter != TBDK_INTER_CUBIC) ||
        (flags & ~(7 | TBDK_WARP_INVERSE_MAP)))
        return TBDK_EINVAL;
    if (border < TBDK_BORDER_CONSTANT || border > TBDK_BORDER_TRANSPARENT) return TBDK_EINVAL;
    // dst == src: the reference clones src (imgwarp.cpp:2595-2596); here aliasing is an error
    const uint8_t* s0 = src;
    const uint8_t* s1 = src + (size_t)(src_height - 1) * src_pitch + src_width;
    const uint8_t* d0 = dst;
    const uint8_t* d1 = dst + (size_t)(dst_height - 1) * dst_pitch + dst_width;
    if (d0 < s1 && s0 < d1) return TBDK_EINVAL;
    double minv[6];
    if (flags & TBDK_WARP_INVERSE_MAP) {
        for (int i = 0; i < 6; ++i) minv[i] = M[i];
    } else {
        invert_affine(M, minv);
    }
    const int cval = border_value < 0 ? 0 : (border_value > 255 ? 255 : border_value);  // saturate_cast<uchar>
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rec = timing_begin(ctx, "warp_affine", s);
    hipError_t e = launch_warp_affine(src, src_width, src_height, src_pitch, dst, dst_width, dst_height, dst_pitch,
                                      minv, inter, border, cval, s);
    timing_end(ctx, rec, s);
    return map_err(e);
}

int tbdk_hbm_copy(tbdk_ctx* ctx, void* dst, const void* src, int64_t bytes, void* stream)
{
    if (!ctx || !dst || !src || bytes < 0 || (bytes & 15) != 0 ||
        ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) != 0)
        return TBDK_EINVAL;
    const char *d = static_cast<const char*>(dst), *sp = static_cast<const char*>(src);
    if (d < sp + bytes && sp < d + bytes && bytes > 0) return TBDK_EINVAL;  // overlapping
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rec = timing_begin(ctx, "hbm_copy", s);
    hipError_t e = launch_hbm_copy(src, dst, (size_t)bytes / 16, s);
    timing_end(ctx, rec, s);
    return map_err(e);
}

int tbdk_synth_render(tbdk_ctx* ctx, uint32_t seed, int width, int height, int nobj, int t0, int nframes,
                      uint8_t* out, int pitch, int32_t* gt_boxes, void* stream)
{
    if (!ctx || !out || width <= 0 || height <= 0 || nobj < 0 || nobj > SYN_MAX_OBJECTS || nframes <= 0 ||
        pitch < width)
        return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nob = nobj > 0 ? nobj : 1;
    syn_object* objs = static_cast<syn_object*>(std::malloc(sizeof(syn_object) * nob));
    syn_pose* poses = static_cast<syn_pose*>(std::malloc(sizeof(syn_pose) * (size_t)nob * nframes));
    if (!objs || !poses) {
        std::free(objs);
        std::free(poses);
        return TBDK_ENOMEM;
    }
    syn_make_objects(seed, width, height, nobj, objs);
    for (int f = 0; f < nframes; ++f)
        for (int o = 0; o < nobj; ++o) {
            syn_pose* p = &poses[(size_t)f * nobj + o];
            syn_pose_at(&objs[o], width, height, t0 + f, p);
            if (gt_boxes) {
                int32_t* gb = gt_boxes + ((size_t)f * nobj + o) * 5;
                gb[0] = syn_gt_box(p, width, height, gb + 1);
                if (!gb[0]) gb[1] = gb[2] = gb[3] = gb[4] = 0;
            }
        }
    void* dposes = nullptr;
    hipError_t e = hipMalloc(&dposes, sizeof(syn_pose) * (size_t)nob * nframes);
    if (e == hipSuccess)
        e = hipMemcpyAsync(dposes, poses, sizeof(syn_pose) * (size_t)nob * nframes, hipMemcpyHostToDevice, s);
    uint32_t bgseed = syn_hash(seed ^ 0xB6A5EEDU);
    if (e == hipSuccess) e = launch_synth(dposes, nobj, bgseed, width, height, nframes, out, pitch, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (dposes) (void)hipFree(dposes);
    std::free(objs);
    std::free(poses);
    return map_err(e);
}

}  // extern "C"
