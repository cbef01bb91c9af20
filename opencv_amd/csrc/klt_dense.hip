// klt_dense.hip — dense pyramidal Lucas-Kanade: cv::cuda::DensePyrLKOpticalFlow
// (cudaoptflow/include/opencv2/cudaoptflow.hpp:182-208, impl
// cudaoptflow/src/pyrlk.cpp:238-299, 352-391) as the CPU cv::calcOpticalFlowPyrLK
// (video/src/lkpyramid.cpp:1207-1377) evaluated at every pixel of the frame:
// the same LK kernels as tbdk_lk_sparse over the full pixel grid, then the
// flow u = nextPt.x - x, v = nextPt.y - y written as CV_32FC2.
//
// The CUDA module's dense kernel has no CPU counterpart (float pyrDown
// pyramids, texture bilinear, no minEig gate, its own stop rule); this entry
// point keeps the CPU semantics of the sparse path so that both LK forms of
// the library agree point for point.
//
// Dense-specific setup (ctx option lk_dense_case, default on): at level L the
// pixel (x, y) sits at (x / 2^L, y / 2^L), so its window is interpolated with
// one of 4^L sub-pixel phases ((x mod 2^L, y mod 2^L) / 2^L) at integer origin
// (x >> L, y >> L) - half.  The interpolated I x32, Ix and Iy of every level
// position are computed once per phase into "case images" (dense_case_kernel,
// 4^L images of the level's size: as many elements per level as the frame has
// pixels), and the PyrLK kernel reads each window from them
// (lk_multi_kernel's DENSE mode) instead of interpolating (win + 1)^2 pyramid
// and derivative-plane values per point and level: the window loads of
// neighbouring pixels are the same case-image rows, shifted by one column
// (cudaoptflow's denseKernel shares them in a block tile; here the bilinear
// work itself is shared).  Same integers as the per-point setup, so the flow
// and status are unchanged.
#include <cstring>

#include "lk_device.hpp"

namespace tbdk {

namespace {

// the pixel grid (x, y) of a w x h frame, one float2 per pixel
__global__ __launch_bounds__(256) void dense_grid_kernel(float2* pts, int w, int h)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x < w) pts[(size_t)y * w + x] = make_float2((float)x, (float)y);
}

// case image `c` of a level: element (y, x), y in [-B, h + B), x in [-B, w + B),
// at C + c * cstride + y * cpitch + x: (I x32 | Ix << 16, Iy) interpolated at
// (x + cx / 2^L, y + cy / 2^L), (cx, cy) = (c mod 2^L, c >> L), as the PyrLK
// setup interpolates a window element (lkpyramid.cpp:227-234, 268-303: weights
// cvRound(w * 2^14), I with CV_DESCALE by W_BITS1 - 5, the derivatives by
// W_BITS1; pair_step in klt_lk_multi.hip) from the padded level (reflect-101
// frame) and its derivative plane (zero frame)
struct DenseCaseArgs {
    const uint8_t* I;  // level, padded origin
    const uint8_t* D;  // derivative plane (Ix, Iy int16), padded origin
    int ipitch, ipad, dpitch, dpad, w, h, B, level;
    uint2* C;
    int cpitch;
    int64_t cstride;
};

__global__ __launch_bounds__(256) void dense_case_kernel(DenseCaseArgs a)
{
    using namespace lkdev;
    const int c = blockIdx.z;
    const int xx = (int)(blockIdx.x * 256 + threadIdx.x) - a.B, yy = (int)blockIdx.y - a.B;
    if (xx >= a.w + a.B) return;
    const int msk = (1 << a.level) - 1;
    const float sc = (float)(1. / (1 << a.level));
    uint32_t w0, w1;  // (iw00, iw01), (iw10, iw11)
    bilinear_weights((float)(c & msk) * sc, (float)(c >> a.level) * sc, w0, w1);
    const uint8_t* ip = a.I + (ptrdiff_t)(yy + a.ipad) * a.ipitch + xx + a.ipad;
    const uint32_t i0 = (uint32_t)ip[0] | ((uint32_t)ip[1] << 16);
    const uint32_t i1 = (uint32_t)ip[a.ipitch] | ((uint32_t)ip[a.ipitch + 1] << 16);
    const uint32_t* dp =
        reinterpret_cast<const uint32_t*>(a.D + (ptrdiff_t)(yy + a.dpad) * a.dpitch + 4 * (ptrdiff_t)(xx + a.dpad));
    const uint32_t* dq = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(dp) + a.dpitch);
    const uint32_t d00 = dp[0], d01 = dp[1], d10 = dq[0], d11 = dq[1];
    const uint32_t dx0 = __builtin_amdgcn_perm(d01, d00, 0x05040100u), dx1 = __builtin_amdgcn_perm(d11, d10, 0x05040100u);
    const uint32_t dy0 = __builtin_amdgcn_perm(d01, d00, 0x07060302u), dy1 = __builtin_amdgcn_perm(d11, d10, 0x07060302u);
    const int iv = sdot2(i0, w0, sdot2(i1, w1, 1 << (W_BITS1 - 5 - 1))) >> (W_BITS1 - 5);
    const int xv = sdot2(dx0, w0, sdot2(dx1, w1, 1 << (W_BITS1 - 1))) >> W_BITS1;
    const int yv = sdot2(dy0, w0, sdot2(dy1, w1, 1 << (W_BITS1 - 1))) >> W_BITS1;
    a.C[(int64_t)c * a.cstride + (int64_t)yy * a.cpitch + xx] =
        make_uint2(((uint32_t)iv & 0xFFFFu) | ((uint32_t)xv << 16), (uint32_t)yv & 0xFFFFu);
}

// flow = next - grid; status copied into a pitched plane when asked for
__global__ __launch_bounds__(256) void dense_flow_kernel(const float2* next, const uint8_t* st, int w, int h,
                                                         float* flow, int flow_pitch, uint8_t* status,
                                                         int status_pitch)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= w) return;
    const size_t i = (size_t)y * w + x;
    const float2 p = next[i];
    *reinterpret_cast<float2*>(reinterpret_cast<uint8_t*>(flow) + (size_t)y * flow_pitch + 8 * (size_t)x) =
        make_float2(p.x - (float)x, p.y - (float)y);
    if (status) status[(size_t)y * status_pitch + x] = st[i];
}

}  // namespace

}  // namespace tbdk

using namespace tbdk;

extern "C" {

int tbdk_lk_dense(tbdk_ctx* ctx, const tbdk_pyr* prev, const tbdk_pyr* next, float* flow, int flow_pitch,
                  uint8_t* status, int status_pitch, const tbdk_lk_params* p, void* stream)
{
    if (!ctx || !prev || !next || !flow || !p || prev->nlevels <= 0) return TBDK_EINVAL;
    if (prev->cn > 1 || next->cn > 1) return TBDK_EINVAL;  // the dense path takes one-channel pyramids
    // CV_Assert(winSize_[0] > 2 && winSize_[1] > 2) of PyrLKOpticalFlowBase::dense (pyrlk.cpp:243)
    if (p->win_w <= 2 || p->win_h <= 2) return TBDK_EINVAL;
    // the reference's dense() never reads the incoming flow, so useInitialFlow has
    // no effect there (pyrlk.cpp:238-299): drop the flag rather than reject it
    tbdk_lk_params prm = *p;
    prm.flags &= ~TBDK_OPTFLOW_USE_INITIAL_FLOW;
    const int w = prev->lv[0].width, h = prev->lv[0].height;
    if (next->nlevels <= 0 || next->lv[0].width != w || next->lv[0].height != h) return TBDK_EINVAL;
    if (flow_pitch < 8 * w || flow_pitch % 8 != 0 || (status && status_pitch < w)) return TBDK_EINVAL;
    const int64_t n = (int64_t)w * h;
    if (n > INT32_MAX) return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the case-image path: one-channel 8-bit pyramids with derivative planes and
    // a square window the several-points-per-wave kernel instantiates
    int max_level = prm.max_level;
    if (prev->nlevels - 1 < max_level) max_level = prev->nlevels - 1;
    if (next->nlevels - 1 < max_level) max_level = next->nlevels - 1;
    bool use_case = ctx->opt_lk_dense_case && prm.impl == 0 && prev->depth == TBDK_DEPTH_8U &&
                    next->depth == TBDK_DEPTH_8U && lk_multi_supported(prm.win_w, prm.win_h) && max_level >= 0 &&
                    max_level < 6;
    for (int l = 0; use_case && l <= max_level; ++l)
        if (!prev->dv[l].data || prev->dv[l].pad < prm.win_w + 2 || prev->lv[l].pad < prm.win_w + 2) use_case = false;
    if (use_case) {
        const int B = prm.win_w / 2;  // a window reaches half a window past its point
        LkDense d;
        std::memset(&d, 0, sizeof(d));
        size_t total = 0;
        int64_t off[TBDK_MAX_LEVELS];
        for (int l = 0; l <= max_level; ++l) {
            const tbdk_level& L = prev->lv[l];
            d.cpitch[l] = L.width + 2 * B;
            d.cstride[l] = (int64_t)d.cpitch[l] * (L.height + 2 * B);
            off[l] = (int64_t)total;
            total += (size_t)d.cstride[l] << (2 * l);
        }
        const size_t bytes = total * sizeof(uint2) + 256;
        if (bytes > ctx->dcase_cap) {
            if (ctx->dcase_buf) (void)hipFree(ctx->dcase_buf);
            ctx->dcase_buf = nullptr;
            ctx->dcase_cap = 0;
            if (hipMalloc(&ctx->dcase_buf, bytes) != hipSuccess) return TBDK_ENOMEM;
            ctx->dcase_cap = bytes;
        }
        uint2* base = static_cast<uint2*>(ctx->dcase_buf);
        for (int l = 0; l <= max_level; ++l) {
            const tbdk_level& L = prev->lv[l];
            const tbdk_level& D = prev->dv[l];
            DenseCaseArgs ca;
            ca.I = L.data;
            ca.D = D.data;
            ca.ipitch = L.pitch;
            ca.ipad = L.pad;
            ca.dpitch = D.pitch;
            ca.dpad = D.pad;
            ca.w = L.width;
            ca.h = L.height;
            ca.B = B;
            ca.level = l;
            ca.C = base + off[l] + (int64_t)B * d.cpitch[l] + B;  // element (0, 0) of case 0
            ca.cpitch = d.cpitch[l];
            ca.cstride = d.cstride[l];
            d.C[l] = ca.C;
            const dim3 cg((d.cpitch[l] + 255) / 256, L.height + 2 * B, 1u << (2 * l));
            hipLaunchKernelGGL(dense_case_kernel, cg, dim3(256), 0, s, ca);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return map_status(e);
        }
        d.w = w;
        d.flow = flow;
        d.flow_pitch = flow_pitch;
        d.status = status;
        d.status_pitch = status_pitch;
        return lk_internal(ctx, prev, next, nullptr, nullptr, nullptr, nullptr, nullptr, (int)n, &prm, nullptr, 0,
                           stream, nullptr, &d);
    }
    // scratch: grid points, next points (float2 each) and status per pixel
    if (n > ctx->dense_cap) {
        if (ctx->dense_buf) (void)hipFree(ctx->dense_buf);
        ctx->dense_buf = nullptr;
        ctx->dense_cap = 0;
        if (hipMalloc(&ctx->dense_buf, (size_t)n * 17 + 256) != hipSuccess) return TBDK_ENOMEM;
        ctx->dense_cap = n;
    }
    float2* pts = static_cast<float2*>(ctx->dense_buf);
    float2* nxt = pts + n;
    uint8_t* st = reinterpret_cast<uint8_t*>(nxt + n);
    const dim3 grid((w + 255) / 256, h);
    hipLaunchKernelGGL(dense_grid_kernel, grid, dim3(256), 0, s, pts, w, h);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return map_status(e);
    const int rc = lk_internal(ctx, prev, next, reinterpret_cast<const float*>(pts), reinterpret_cast<float*>(nxt),
                               st, nullptr, nullptr, (int)n, &prm, nullptr, 0, stream);
    if (rc != TBDK_OK) return rc;
    hipLaunchKernelGGL(dense_flow_kernel, grid, dim3(256), 0, s, nxt, st, w, h, flow, flow_pitch, status,
                       status_pitch);
    return map_status(hipGetLastError());
}

}  // extern "C"
